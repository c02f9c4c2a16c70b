"""Fixture: the C oracle's outcome for every lane of bench.py's headline workload (test infrastructure only).

BASELINE cfg 3 exactly as `bench.py` builds it: 262,144 lanes, x0 = [th1, th2, 0, 0] with th ~ U(+-0.5) from
default_rng(0) (bench.make_x0), lane 0 = 0, task-2 reference and settings (trajectory_generation.py:298-398 with
tol 1e-4, beta 0.7, c 0.5, gamma_0 0.1, <= 20 Armijo trials, max_iters 5000).  Per lane: n_iter, status, n_rollouts,
final cost and the Armijo tie record (make_stress_oracle.solve_all).  bench.make_x0 draws the lanes in order, so these
are also the first 262,144 lanes of BASELINE cfg 4's 1,048,576-lane batch.  tests/test_gpu_parity.py
(test_full_size_properties) and tests/test_gpu_workloads.py (test_cfg4_global_batch_on_one_gpu) assert every lane
against it.  About 25 minutes on 8 host cores.

Usage:  python tests/golden/make_headline_oracle.py [--chunk 4096]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_stress_oracle import solve_all     # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--out", default=os.path.join(HERE, "headline_oracle.npz"))
    a = ap.parse_args()
    solve_all(0.5, a.out, a.chunk)


if __name__ == "__main__":
    main()
