#!/bin/bash
# A/B: the Riccati step without the terms tau1-zero mode zeroes (sigma0, its dJ / max|sigma| terms, r0); GPU suite first.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/u0zstep_tests.log 2>&1 || { tail -30 gpurun_out/u0zstep_tests.log; exit 1; }
tail -2 gpurun_out/u0zstep_tests.log
timeout -k 10 300 python -u tools/ab_bench.py --batch 4096 --rounds 3 build_ab/base.so build_ab/u0zstep.so > gpurun_out/ab_u0zstep_4096.log 2>&1 || exit $?
tail -6 gpurun_out/ab_u0zstep_4096.log
timeout -k 10 400 python -u tools/ab_bench.py --batch 262144 --rounds 3 build_ab/base.so build_ab/u0zstep.so > gpurun_out/ab_u0zstep_262144.log 2>&1 || exit $?
tail -6 gpurun_out/ab_u0zstep_262144.log
