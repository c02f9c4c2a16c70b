#!/bin/bash
# Round-5 GPU session: named steps, each under its own time limit, chained so that the first failure (a test
# failure, a fault, an abort, a time limit) ends the script.  Output under gpurun_out/r05/<name>.log.
#   tools/r05_session.sh tests smoke bench trace3 fetch write ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r05/${R05_TAG:-final}
mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a $OUT/steps.log
  tail -4 "$OUT/$name.log" | cut -c1-400
  return $rc
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
for s in "$@"; do
  case $s in
    tests_tail) step pytest_tail 600 $PYT tests/test_gpu_tail.py -m gpu || exit $? ;;
    tests_bench) step pytest_bench 600 $PYT tests/test_gpu_workloads.py -m gpu -k "bench_spawns or cfg2" || exit $? ;;
    tests_stress) step pytest_stress 600 $PYT tests/test_gpu_stress.py -m gpu || exit $? ;;
    tests_cand) step pytest_cand 600 $PYT tests/test_gpu_tail.py -m gpu -k "candidate_scratch" || exit $? ;;
    tests) step pytest_gpu 1100 $PYT tests -m gpu || exit $? ;;
    smoke) step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) step bench 600 python -u bench.py || exit $? ;;
    bench_cfg2) step bench_cfg2 300 python -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --no-box --extra-legs "" || exit $? ;;
    bench_stress) step bench_stress 300 python -u bench.py --workload stress --steps 2 --warmup 1 --no-cpu --no-box --extra-legs "" || exit $? ;;
    trace2) step trace_cfg2 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg2 -o run --output-format csv -- python3 -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --no-box --extra-legs "" || exit $? ;;
    trace3) step trace_cfg3 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg3 -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-box --extra-legs "" || exit $? ;;
    tracest) step trace_stress 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_stress -o run --output-format csv -- python3 -u bench.py --workload stress --steps 2 --warmup 1 --no-cpu --no-box --extra-legs "" || exit $? ;;
    tracem) step trace_mpc 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_mpc -o run --output-format csv -- python3 -u bench.py --workload mpc --steps 20 --warmup 3 || exit $? ;;
    fetch) step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_fetch -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-box --no-timing --max-iters 20 --extra-legs "" || exit $? ;;
    valu) step pmc_valu 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_nt_" -d $OUT/pmc_valu -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-box --no-timing --max-iters 20 --extra-legs "" || exit $? ;;
    write) step pmc_write 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_write -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-box --no-timing --max-iters 20 --extra-legs "" || exit $? ;;
    run2trace) step run2_trace 200 python -u tools/run2_trace.py build_ab/run2_trace.so || exit $? ;;
    legs) step leg_order 400 python -u tools/leg_order.py --order cfg3:5:20,general:1:2,cfg3:1:3 --out $OUT/leg_order.jsonl || exit $? ;;
    settle) step settle 500 python -u tools/stress_settle_dump.py --out $OUT/settle.npz || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
