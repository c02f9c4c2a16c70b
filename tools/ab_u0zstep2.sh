#!/bin/bash
# A/B of the tau1-zero Riccati step on the default schedules: persistent at 4,096 lanes, pipelined at 262,144.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_bench.py --batch 4096 --rounds 3 build_ab/base.so:run build_ab/u0zstep.so:run > gpurun_out/ab_u0zstep_run_4096.log 2>&1 || exit $?
tail -3 gpurun_out/ab_u0zstep_run_4096.log
timeout -k 10 400 python -u tools/ab_bench.py --batch 262144 --rounds 3 build_ab/base.so:pipe build_ab/u0zstep.so:pipe > gpurun_out/ab_u0zstep_pipe_262144.log 2>&1 || exit $?
tail -3 gpurun_out/ab_u0zstep_pipe_262144.log
