"""Worker of tests/test_gpu_workloads.py::test_sharded_solve_on_hip_matches_unsharded (not a test module).

Launched by torch.distributed.run with GYM_DIST_BACKEND=gloo (several ranks sharing one GPU: RCCL refuses two
ranks on one device).  Each rank solves its contiguous shard through distributed.solve_sharded on the HIP
solver and writes its lanes' results to <out>.rank<r>.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, total, max_iters, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    import torch
    from gymnast_optimalcontrol_amd import distributed as gd
    rank, local_rank, world = gd.init_process_group()
    torch.cuda.set_device(gd.local_device_index(local_rank))
    from bench import load_refs
    x_ref, u_ref = load_refs()
    x0 = sharded_x0(total, seed)
    lo, hi, res = gd.solve_sharded(x0, x_ref, u_ref, max_iters, keep_stats=True, tol=1e-4, gamma_0=0.1)
    import torch.distributed as dist
    g = gd.gather_sharded({"cost": res.cost, "n_iter": res.n_iter, "status": res.status}, total)
    np.savez(f"{out}.gathered.rank{rank}.npz", **{k: v.cpu().numpy() for k, v in g.items()})
    np.savez(f"{out}.rank{rank}.npz", lo=lo, hi=hi, x=res.x.cpu().numpy(), u=res.u.cpu().numpy(),
             K=res.K.cpu().numpy(), sigma=res.sigma.cpu().numpy(), cost=res.cost.cpu().numpy(),
             n_iter=res.n_iter.cpu().numpy(), status=res.status.cpu().numpy(),
             n_rollouts=res.n_rollouts.cpu().numpy(), stats=np.asarray(res.stats_log),
             schedule=np.array(res.schedule))
    # per-lane references (B_total, N, 4) / (B_total, T, 2): solve_sharded cuts them to the rank's shard
    xr3 = np.broadcast_to(x_ref, (total,) + x_ref.shape).copy()
    ur3 = np.broadcast_to(u_ref, (total,) + u_ref.shape).copy()
    ur3[1::3, :, 1] *= 0.8                       # every third lane follows another reference
    lo3, hi3, r3 = gd.solve_sharded(x0, xr3, ur3, 40, tol=1e-4, gamma_0=0.1)
    np.savez(f"{out}.perlane.rank{rank}.npz", lo=lo3, hi=hi3, x=r3.x.cpu().numpy(), cost=r3.cost.cpu().numpy(),
             n_iter=r3.n_iter.cpu().numpy())
    if total > 1000:   # hard lanes with lane compaction forced at every sync (rank-local) and the tail (global)
        xh = hard_x0(2000, 3)
        _, _, gh = gd.solve_sharded(xh, x_ref, u_ref, 200, gather=True, tol=1e-4, gamma_0=0.1, compact="force",
                                    tail_lanes=60, hist_len=200)
        np.savez(f"{out}.hard.rank{rank}.npz", **{k: v.cpu().numpy() for k, v in gh.items()})
    dist.barrier()
    dist.destroy_process_group()


def hard_x0(total: int, seed: int) -> np.ndarray:
    """SURVEY 8(d)'s stress distribution (theta0 ~ U(+-1.5), some initial velocities) with a NaN lane."""
    rng = np.random.default_rng(seed)
    x0 = np.zeros((total, 4))
    x0[:, :2] = rng.uniform(-1.5, 1.5, (total, 2))
    x0[::9, 2:] = rng.uniform(-2.0, 2.0, (len(x0[::9]), 2))
    x0[7] = np.nan
    return x0


def sharded_x0(total: int, seed: int) -> np.ndarray:
    """Headline-distribution lanes with every 37th lane a wide start (backtracking / LS failure)."""
    rng = np.random.default_rng(seed)
    x0 = np.zeros((total, 4))
    x0[:, :2] = rng.uniform(-0.5, 0.5, (total, 2))
    wide = np.arange(5, total, 37)
    x0[wide, :2] = rng.uniform(-1.5, 1.5, (wide.size, 2))
    x0[0] = 0.0
    return x0


if __name__ == "__main__":
    main()
