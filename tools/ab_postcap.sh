#!/bin/bash
# A/B: grid caps of the post-trial kernels (sigma / candidates / retry launch every phase, mostly early exits).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_bench.py --batch 262144 --rounds 3 build_ab/base.so:pipe build_ab/cap256.so:pipe build_ab/cap64.so:pipe > gpurun_out/ab_postcap_262144.log 2>&1 || exit $?
tail -4 gpurun_out/ab_postcap_262144.log
timeout -k 10 300 python -u tools/ab_bench.py --batch 262144 --rounds 1 --spread 1.5 --max-iters 600 build_ab/base.so:pipe build_ab/cap256.so:pipe build_ab/cap64.so:pipe > gpurun_out/ab_postcap_stress.log 2>&1 || exit $?
tail -4 gpurun_out/ab_postcap_stress.log
