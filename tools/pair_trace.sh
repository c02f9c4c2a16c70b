#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
for v in run2_trace; do echo "variant $v"; timeout -k 10 100 python tools/run2_trace.py build_ab/$v.so --batch 4096 --iters 40 || exit 1; done
timeout -k 10 300 python -u tools/ab_bench.py --batch 4096 --rounds 3 build_ab/pair.so:run build_ab/pairv3.so:run > gpurun_out/ab_pairv3_run_4096.log 2>&1 || exit $?
tail -2 gpurun_out/ab_pairv3_run_4096.log
