cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --tb=short --timeout 150 --timeout-method thread -k "persistent_schedule_matches_serial and 25" > gpurun_out/r2_first.log 2>&1 || { echo "first failed rc=$?"; tail -30 gpurun_out/r2_first.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -v -p no:cacheprovider --tb=short --timeout 200 --timeout-method thread -k "persistent or cfg2 or capture" > gpurun_out/r2_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r2_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --batch 4096 --steps 3 --warmup 1 --no-cpu --extra-legs "" > gpurun_out/r2_c2_on.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --batch 4096 --steps 3 --warmup 1 --no-cpu --extra-legs "" --split-waves off > gpurun_out/r2_c2_off.log 2>&1 || exit $?
for f in r2_c2_on r2_c2_off; do grep '^{' gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
