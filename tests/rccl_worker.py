"""Worker of tests/test_gpu_workloads.py::test_rccl_collectives_on_one_gpu (not a test module).

Runs in its own process: a 1-rank torch.distributed group on the RCCL backend ("nccl") with ``device_id``, and
drives distributed.solve_sharded(..., gather=True, force_collectives=True) through the device-tensor branches of
make_reduce_stats (SUM all-reduce of the statistics), gather_sharded (all-gather of every result field),
max_over_ranks and sum_over_ranks -- the branches the driver's 8-GPU run takes (RCCL refuses two ranks on one
device, so one rank is how a one-GPU box executes them).  Every collective call is recorded (tensor device,
dtype, the stream it was enqueued from).  The sharded results must be bit for bit the plain solve's.  Writes a
JSON summary to argv[1] and exits non-zero on any mismatch."""
import json
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    out, total, max_iters = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(_free_port()))
    os.environ.pop("GYM_DIST_BACKEND", None)
    import torch
    import torch.distributed as dist
    from gymnast_optimalcontrol_amd import distributed as gd
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from bench import load_refs
    from sharded_worker import sharded_x0

    calls = []

    def recording(name, fn):
        def wrapped(t, *a, **kw):
            first = t[0] if isinstance(t, (list, tuple)) else t
            src = a[0] if name == "all_gather" else t
            calls.append({"op": name, "device": str(src.device), "dtype": str(src.dtype),
                          "stream": torch.cuda.current_stream().cuda_stream, "out_device": str(first.device)})
            return fn(t, *a, **kw)
        return wrapped

    dist.all_reduce = recording("all_reduce", dist.all_reduce)
    dist.all_gather = recording("all_gather", dist.all_gather)

    rank, local_rank, world = gd.init_process_group(backend="nccl", force=True)
    assert dist.is_initialized() and dist.get_backend() == "nccl" and dist.get_world_size() == 1, dist.get_backend()
    torch.cuda.set_device(gd.local_device_index(local_rank))
    x_ref, u_ref = load_refs()
    x0 = sharded_x0(total, 7)           # seed 7: backtracking lanes at 301 lanes (test_sharded_solve_on_hip...)
    eng = AcrobotEngine()
    summary = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "schedules": {}}
    kw = dict(tol=1e-4, gamma_0=0.1)
    for sched, skw in (("persistent", {}), ("pipelined", {"pipeline": True}), ("serial", {"pipeline": False})):
        n0 = len(calls)
        lo, hi, g = gd.solve_sharded(x0, x_ref, u_ref, max_iters, engine=eng, gather=True, force_collectives=True,
                                     **kw, **skw)
        assert (lo, hi) == (0, total)
        mine = calls[n0:]
        ref = BatchedNewtonSolver(eng, x_ref, u_ref, total, **kw, **skw).solve(x0, max_iters)
        assert ref.schedule == sched, (ref.schedule, sched)
        for f in gd.GATHER_FIELDS:
            a, b = g[f].cpu().numpy(), getattr(ref, f).cpu().numpy()
            assert a.shape == b.shape and np.array_equal(a, b, equal_nan=True), f"{sched}: field {f} differs"
        ar = [c for c in mine if c["op"] == "all_reduce"]
        ag = [c for c in mine if c["op"] == "all_gather"]
        assert ar and all(c["device"].startswith("cuda") and c["dtype"] == "torch.float64" for c in ar), ar[:2]
        assert all(c["stream"] == eng.stream for c in ar), "all-reduce not enqueued from the solver's stream"
        assert len(ag) == len(gd.GATHER_FIELDS) and all(c["device"].startswith("cuda") for c in ag), ag
        summary["schedules"][sched] = {"all_reduce_calls": len(ar), "all_gather_calls": len(ag),
                                       "lanes": total, "lane_iterations": int(ref.lane_iterations),
                                       "backtracked": int((ref.n_rollouts > ref.n_iter).sum().item())}
    n0 = len(calls)
    assert gd.max_over_ranks(3.25, force=True) == 3.25 and gd.sum_over_ranks(2.5, force=True) == 2.5
    assert [c["op"] for c in calls[n0:]] == ["all_reduce", "all_reduce"]
    assert all(c["device"].startswith("cuda") for c in calls[n0:])
    # per-lane references are cut to the shard (one rank: the whole batch), bit for bit the shared-reference solve
    xr3 = np.broadcast_to(x_ref, (total,) + x_ref.shape).copy()
    ur3 = np.broadcast_to(u_ref, (total,) + u_ref.shape).copy()
    _, _, g3 = gd.solve_sharded(x0, xr3, ur3, 40, engine=eng, gather=True, force_collectives=True, **kw)
    r3 = BatchedNewtonSolver(eng, x_ref, u_ref, total, **kw).solve(x0, 40)
    for f in ("x", "u", "cost", "n_iter"):
        assert np.array_equal(g3[f].cpu().numpy(), getattr(r3, f).cpu().numpy(), equal_nan=True), f
    summary["collective_calls"] = len(calls)
    dist.barrier()
    dist.destroy_process_group()
    with open(out, "w") as f:
        json.dump(summary, f)
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
