#!/usr/bin/env python3
"""Why the MPC pair rollout with double-buffered feedback rows changed bits (round 3, profiles/r03/near_path/).

Round 3 unrolled k_track_rollout_pair's step loop by two with two register sets of the per-step feedback rows (K,
x_ff, u_ff), so that no row is copied between steps; that build failed the pair-vs-single-lane bitwise test and was
reverted without a diagnosis.  This probe rebuilds the variant from the committed kernel (a patched copy of
tracking_kernels.hip in a scratch directory) and tells the two candidate causes apart:

  * FMA contraction: the feedback u = u_ff + K (x - x_ff) is compiled under the file's default -ffp-contract=fast,
    so the backend picks which product of ((k0 d0 + k1 d1) + k2 d2) + k3 d3 it fuses, per code context.  --isa
    prints the instruction sequence that forms each feedback component in the single-lane kernel, the committed
    pair kernel and the variant; a different fused operand order is a contraction difference.
  * a wrong-row read: the variant reading step t's row from the wrong register set (or the wrong row).  --run (GPU)
    compares every step of every lane with the single-lane kernel and reports the first differing (lane, step); a
    read of the wrong row shows as a difference from the first step whose row is mis-read, for every lane,
    whereas a contraction difference shows only for lanes and steps where the two roundings differ.
  Each is built twice: with the feedback inlined under the file's default contraction (as in round 3) and through
  track_feedback (`#pragma clang fp contract(on)`, the committed form), which fixes the fused product.

    python tools/mpc_rowbuf_probe.py --isa            # CPU: build the four libraries + print the feedback ISA
    python tools/mpc_rowbuf_probe.py --run            # GPU (libraries built beforehand): bitwise comparison
"""
import argparse
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "gymnast_optimalcontrol_amd", "csrc")
OUT = os.path.join(ROOT, "build_ab")

LOOP_COMMITTED = "    for (int t = 0; t < T; ++t) {\n        const double d0 = n0 - r[0]"

VARIANT_LOOP = r'''    double kB[8], rB[4], fB[2];
    // rows double-buffered: step t reads set A (t even) or B (t odd); the other set is loaded for step t + 1
    auto step = [&](const double* kk, const double* rr, const double* ff, double* kn, double* rn, double* fn, int t) {
        const double d0 = n0 - rr[0], d1 = n1 - rr[1], d2 = n2 - rr[2], d3 = n3 - rr[3];
        const double v0 = ff[0] + (((kk[0] * d0 + kk[1] * d1) + kk[2] * d2) + kk[3] * d3);
        const double v1 = ff[1] + (((kk[4] * d0 + kk[5] * d1) + kk[6] * d2) + kk[7] * d3);
        if (t + 1 < T) {
            const double* kq = K + 8 * (t + 1);
#pragma unroll
            for (int q = 0; q < 8; ++q) kn[q] = kq[q];
#pragma unroll
            for (int q = 0; q < 4; ++q) rn[q] = x_ff[4 * (t + 1) + q];
            fn[0] = u_ff[2 * (t + 1)]; fn[1] = u_ff[2 * (t + 1) + 1];
        }
        if (!odd) st_nt2(ul + t, v0, v1);
        gym::rk4_pair_fast(dm, odd, n0, n1, n2, n3, v1, pk);
        if (odd) st_nt2(xl + 2 * (t + 1), n2, n3);
        else st_nt2(xl + 2 * (t + 1), n0, n1);
    };
    for (int t = 0; t < T; t += 2) {
        step(k, r, f, kB, rB, fB, t);
        if (t + 1 >= T) break;
        step(kB, rB, fB, k, r, f, t + 1);
    }
}
'''

INLINE_FAST = """        double v0, v1;
        track_feedback(k, f, d0, d1, d2, d3, v0, v1);"""
INLINE_FAST_BODY = """        const double v0 = f[0] + (((k[0] * d0 + k[1] * d1) + k[2] * d2) + k[3] * d3);
        const double v1 = f[1] + (((k[4] * d0 + k[5] * d1) + k[6] * d2) + k[7] * d3);"""


def patched_source(variant: bool, fast: bool) -> str:
    """The committed tracking_kernels.hip (feedback through track_feedback, contract(on)); ``fast``: the feedback
    inlined under the file's default -ffp-contract=fast, as before the fix; ``variant``: the pair rollout's loop
    unrolled by two with double-buffered rows (round 3's reverted build)."""
    s = open(os.path.join(CSRC, "tracking_kernels.hip")).read()
    if fast:
        assert s.count(INLINE_FAST) == 2
        s = s.replace(INLINE_FAST, INLINE_FAST_BODY)
    if variant:
        i = s.index("__global__ __launch_bounds__(64) void k_track_rollout_pair(")
        j = s.index(LOOP_COMMITTED, i)
        end = s.index("\n}\n", j) + 3
        loop = VARIANT_LOOP
        if not fast:
            loop = re.sub(r"const double v0 = ff\[0\].*?\n\s*const double v1 = ff\[1\][^\n]*\n",
                          "double v0, v1;\n        track_feedback(kk, ff, d0, d1, d2, d3, v0, v1);\n", loop,
                          flags=re.S)
        s = s[:j] + loop + s[end:]
    return s


def build(name: str, variant: bool, fast: bool) -> str:
    from gymnast_optimalcontrol_amd import _build
    tmp = tempfile.mkdtemp(prefix="gym_probe_")
    for f in os.listdir(CSRC):
        shutil.copy(os.path.join(CSRC, f), tmp)
    open(os.path.join(tmp, "tracking_kernels.hip"), "w").write(patched_source(variant, fast))
    os.makedirs(OUT, exist_ok=True)
    out = os.path.join(OUT, name)
    cmd = [_build.hipcc(), f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           f"-DGYM_BUILD_ID=\"{_build.source_hash()}\"", "-I", _build.INCLUDE, "-I", tmp,
           os.path.join(tmp, "acrobot_kernels.hip"), os.path.join(tmp, "tracking_kernels.hip"), "-o", out]
    subprocess.run(cmd, check=True)
    shutil.rmtree(tmp)
    return out


def feedback_isa(lib: str) -> dict:
    """Per rollout kernel, the instructions that form u = u_ff + K (x - x_ff) after each group of the four
    subtractions d = x - x_ff: which product of k0 d0 + k1 d1 is the separate v_mul (the other is fused)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from isa_diff import code_objects, kernels
    with tempfile.TemporaryDirectory() as tmp:
        ks = kernels(code_objects(lib, tmp))
    out = {}
    for name, ins in ks.items():
        if "k_track_rollout" not in name:
            continue
        idx = [i for i, x in enumerate(ins) if re.match(r"v_add_f64 v\[\d+:\d+\], v\[\d+:\d+\], -[sv]\[", x)]
        groups = []
        for i in idx:
            if groups and i - groups[-1][-1] <= 6:
                groups[-1].append(i)
            else:
                groups.append([i])
        segs = []
        for g in groups:
            if len(g) == 4:
                segs.append([x for x in ins[g[0]:g[-1] + 12] if re.match(r"v_(add|mul|fma|fmac)_f64", x)])
        out["pair" if "pair" in name else "single"] = segs
    return out


def run(libs):
    import numpy as np
    import torch
    os.environ["GYM_ALLOW_FOREIGN_BUILD"] = "1"
    from gymnast_optimalcontrol_amd import _lib, trajectory_tracking as tt
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    trk = np.load(os.path.join(ROOT, "tests", "golden", "tracking.npz"))
    base = tt._eng()
    B = 101
    rng = np.random.default_rng(11)
    x0 = trk["x_opt"][0] + rng.uniform(-0.1, 0.1, (B, 4))
    x0[3, 2:] = [45.0, -60.0]
    x0[7, 0] = np.nan
    x0[9, :2] = [3.0e3, -2.0e3]
    K0, _ = tt.mpc_gains(trk["x_opt"], trk["u_opt"], 50)
    for lib in libs:
        eng = AcrobotEngine(lib_path=lib)
        xp, up = eng.track_rollout(x0, trk["x_opt"], trk["u_opt"], K0)
        xs, us = eng.track_rollout(x0, trk["x_opt"], trk["u_opt"], K0, single=True)
        xp, xs = xp.cpu().numpy(), xs.cpu().numpy()
        up, us = up.cpu().numpy(), us.cpu().numpy()
        same_x = (xp == xs) | (np.isnan(xp) & np.isnan(xs))
        same_u = (up == us) | (np.isnan(up) & np.isnan(us))
        bad_u = np.argwhere(~same_u.all(2))
        bad_x = np.argwhere(~same_x.all(2))
        msg = f"{os.path.basename(lib)}: pair == single bitwise: {bool(same_x.all() and same_u.all())}"
        if len(bad_u) or len(bad_x):
            lanes = sorted(set(bad_u[:, 0].tolist()) | set(bad_x[:, 0].tolist()))
            first = {}
            for l in lanes:
                su = bad_u[bad_u[:, 0] == l][:, 1]
                sx = bad_x[bad_x[:, 0] == l][:, 1]
                first[l] = (int(su.min()) if len(su) else None, int(sx.min()) if len(sx) else None)
            l0 = min(first, key=lambda l: min(v for v in first[l] if v is not None))
            t0 = first[l0][0] if first[l0][0] is not None else first[l0][1] - 1
            msg += (f"; {len(lanes)} of {B} lanes differ; first (u step, x knot) per lane (10 shown): "
                    f"{dict(list(first.items())[:10])}; lane {l0} step {t0}: u pair {up[l0, t0].tolist()} "
                    f"single {us[l0, t0].tolist()} (ulps {np.abs(up[l0, t0].view(np.int64) - us[l0, t0].view(np.int64)).tolist()})")
        print(msg, flush=True)
    # cfg 5's rollout (8,192 lanes, the MPC gains) per library, alternating, event-timed on the engine's stream
    B5 = 8192
    g = np.load(os.path.join(ROOT, "tests", "golden", "task2_reference_output.npz"))
    x5 = g["x"][0] + np.random.default_rng(0).uniform(-0.1, 0.1, (B5, 4))
    K5, _ = tt.mpc_gains(g["x"], g["u"], 50)
    engs = {lib: AcrobotEngine(lib_path=lib) for lib in libs}
    xd, xr5, ur5 = base.t(x5), base.t(g["x"]), base.t(g["u"])
    times = {lib: [] for lib in libs}
    for rep in range(6):
        for lib, eng in engs.items():
            eng.track_rollout(xd, xr5, ur5, K5)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                eng.track_rollout(xd, xr5, ur5, K5)
            e1.record()
            torch.cuda.synchronize()
            times[lib].append(e0.elapsed_time(e1) / 5)
    for lib, ts in times.items():
        print(f"{os.path.basename(lib)}: cfg 5 rollout {min(ts):.4f}-{max(ts):.4f} ms (6 x 5 runs, alternating)",
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--isa", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--build-only", action="store_true")
    a = ap.parse_args()
    # (library, unrolled double-buffered variant?, feedback under -ffp-contract=fast?)
    names = [("rowbuf_committed_fast.so", False, True), ("rowbuf_variant_fast.so", True, True),
             ("rowbuf_committed_on.so", False, False), ("rowbuf_variant_on.so", True, False)]
    libs = [os.path.join(OUT, n) for n, _, _ in names]
    if a.isa or a.build_only:
        libs = [build(n, v, f) for n, v, f in names]
    if a.isa:
        for lib in libs:
            print(os.path.basename(lib))
            for k, segs in feedback_isa(lib).items():
                for n, seg in enumerate(segs):
                    print(f"  k_track_rollout {k}, feedback block {n}:")
                    for x in seg:
                        print("     ", x)
    if a.run:
        run(libs)


if __name__ == "__main__":
    main()
