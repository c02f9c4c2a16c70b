#!/bin/bash
# two-wavefront Riccati update in k_nt_run2: bitwise checks against the previous build, parity tests, A/B, trace
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
echo "== refactor only (serial schedule) vs previous build"; timeout -k 10 200 python tools/compare_libs.py build_ab/pairv3.so build_ab/nosplit.so --batch 8192 --iters 30 || exit $?
echo "== split vs previous build (persistent)"; timeout -k 10 200 python tools/compare_libs.py build_ab/pairv3.so build_ab/split.so --batch 4096 --iters 30 --schedule persistent || exit $?
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --tb=short --timeout 150 --timeout-method thread -k "persistent_schedule_matches_serial and 25" > gpurun_out/split_first.log 2>&1 || { echo "first failed rc=$?"; tail -30 gpurun_out/split_first.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -v -p no:cacheprovider --tb=short --timeout 200 --timeout-method thread -k "persistent or cfg2 or capture or sharded" > gpurun_out/split_tests.log 2>&1; rc=$?; tail -3 gpurun_out/split_tests.log; [ $rc -le 1 ] || exit $rc
echo "variant split_trace"; timeout -k 10 100 python tools/run2_trace.py build_ab/split_trace.so --batch 4096 --iters 40 || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --batch 4096 --rounds 3 build_ab/pairv3.so:run build_ab/split.so:run > gpurun_out/ab_split_4096.log 2>&1 || exit $?
tail -2 gpurun_out/ab_split_4096.log
timeout -k 10 300 python -u tools/ab_bench.py --batch 16384 --rounds 2 build_ab/pairv3.so:run build_ab/split.so:run > gpurun_out/ab_split_16384.log 2>&1 || exit $?
tail -2 gpurun_out/ab_split_16384.log
