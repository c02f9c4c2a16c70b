#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -v -p no:cacheprovider --tb=short --timeout 200 --timeout-method thread -k "straggler or pipelined_schedule_matches or persistent_schedule_matches_serial or cfg2 or sharded" > gpurun_out/tail_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/tail_tests.log | head -30; tail -2 gpurun_out/tail_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload stress --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_stress2.log 2>&1; rc=$?; tail -1 gpurun_out/bench_stress2.log | cut -c1-2500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --extra-legs "" > gpurun_out/bench_cfg3_tail.log 2>&1; rc=$?; tail -1 gpurun_out/bench_cfg3_tail.log | cut -c1-600; exit $rc
