#!/bin/bash
# persistent-schedule parity tests with the lane-pair trial, then same-process A/B against GYM_RUN2_PAIR=0
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --tb=short --timeout 150 --timeout-method thread -k "persistent_schedule_matches_serial and 25" > gpurun_out/pair_first.log 2>&1 || { echo "first failed rc=$?"; tail -30 gpurun_out/pair_first.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -v -p no:cacheprovider --tb=short --timeout 200 --timeout-method thread -k "persistent or cfg2 or capture" > gpurun_out/pair_tests.log 2>&1; rc=$?; tail -5 gpurun_out/pair_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_bench.py --batch 4096 --rounds 3 build_ab/base.so build_ab/pair.so > gpurun_out/ab_pair_4096.log 2>&1 || exit $?
tail -2 gpurun_out/ab_pair_4096.log
timeout -k 10 300 python -u tools/ab_bench.py --batch 16384 --rounds 2 build_ab/base.so build_ab/pair.so > gpurun_out/ab_pair_16384.log 2>&1 || exit $?
tail -2 gpurun_out/ab_pair_16384.log
timeout -k 10 200 python bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" > gpurun_out/pair_cfg2.log 2>&1 || exit $?
tail -1 gpurun_out/pair_cfg2.log | cut -c1-200
