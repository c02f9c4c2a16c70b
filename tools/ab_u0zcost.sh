#!/bin/bash
# A/B: the trial's tau1-zero cost / control terms dropped at compile time; GPU suite first.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/u0zcost_tests.log 2>&1 || { tail -30 gpurun_out/u0zcost_tests.log; exit 1; }
tail -2 gpurun_out/u0zcost_tests.log
timeout -k 10 400 python -u tools/ab_bench.py --batch 262144 --rounds 3 build_ab/u0zstep.so:pipe build_ab/u0zcost.so:pipe > gpurun_out/ab_u0zcost_pipe_262144.log 2>&1 || exit $?
tail -3 gpurun_out/ab_u0zcost_pipe_262144.log
timeout -k 10 300 python -u tools/ab_bench.py --batch 4096 --rounds 3 build_ab/u0zstep.so:serial build_ab/u0zcost.so:serial > gpurun_out/ab_u0zcost_serial_4096.log 2>&1 || exit $?
tail -3 gpurun_out/ab_u0zcost_serial_4096.log
