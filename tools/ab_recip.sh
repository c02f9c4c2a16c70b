#!/bin/bash
# A/B: 1/G11 of the Riccati step by rcp + two Newton steps instead of the IEEE division sequence; GPU suite first.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/recip_tests.log 2>&1 || { tail -40 gpurun_out/recip_tests.log; exit 1; }
tail -2 gpurun_out/recip_tests.log
timeout -k 10 400 python -u tools/ab_bench.py --batch 262144 --rounds 3 build_ab/u0zcost.so:pipe build_ab/recip.so:pipe > gpurun_out/ab_recip_pipe_262144.log 2>&1 || exit $?
tail -3 gpurun_out/ab_recip_pipe_262144.log
timeout -k 10 300 python -u tools/ab_bench.py --batch 4096 --rounds 3 build_ab/u0zcost.so:run build_ab/recip.so:run > gpurun_out/ab_recip_run_4096.log 2>&1 || exit $?
tail -3 gpurun_out/ab_recip_run_4096.log
