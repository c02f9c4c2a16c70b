#!/bin/bash
# Round-4 GPU session: named steps, each under its own time limit, chained so that the first failure (a test
# failure, a fault, an abort, a time limit) ends the script.  Output under gpurun_out/r04/<name>.log.
#   tools/r04_session.sh probe stress tests_carry bench ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04
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
    probe) step mpc_rowbuf 150 python -u tools/mpc_rowbuf_probe.py --run || exit $? ;;
    stress) step stress_parity 400 python -u tools/stress_parity.py full hard --out $OUT/stress || exit $? ;;
    tests_carry) step pytest_carry 600 $PYT tests/test_gpu_parity.py -m gpu -k "carry or persistent_schedule or short_and_ragged" || exit $? ;;
    tests_tail) step pytest_tail 600 $PYT tests/test_gpu_tail.py -m gpu || exit $? ;;
    tests_bench) step pytest_bench 600 $PYT tests/test_gpu_workloads.py -m gpu -k "bench_spawns or cfg2" || exit $? ;;
    tests_stress) step pytest_stress 600 $PYT tests/test_gpu_stress.py -m gpu || exit $? ;;
    tests_cand) step pytest_cand 600 $PYT tests/test_gpu_tail.py -m gpu -k "candidate_scratch" || exit $? ;;
    cand_ab) step cand_ab 400 python -u tools/cand_ab.py --rounds 3 || exit $? ;;
    tail_ab) step tail_ab 500 env GYM_ALLOW_FOREIGN_BUILD=1 python -u tools/ab_bench.py --spread 1.5 --rounds 3 build_ab/tail_base.so build_ab/tail_new.so || exit $? ;;
    sw_ab) step sw_ab 500 env GYM_ALLOW_FOREIGN_BUILD=1 python -u tools/ab_bench.py --spread 1.5 --rounds 3 build_ab/sw_base.so build_ab/sw_new.so || exit $? ;;
    r2_ab) step r2_ab_cfg2 300 env GYM_ALLOW_FOREIGN_BUILD=1 python -u tools/ab_bench.py --batch 4096 --rounds 5 build_ab/r2_base.so:run build_ab/r2_new.so:run &&
           step r2_ab_stress 500 env GYM_ALLOW_FOREIGN_BUILD=1 python -u tools/ab_bench.py --spread 1.5 --rounds 3 build_ab/r2_base.so build_ab/r2_new.so || exit $? ;;
    r2_ab_run) step r2_ab_cfg2 300 env GYM_ALLOW_FOREIGN_BUILD=1 python -u tools/ab_bench.py --batch 4096 --rounds 5 build_ab/r2_base.so:run build_ab/r2_new.so:run || exit $? ;;
    th_ab) step th_ab 500 env GYM_ALLOW_FOREIGN_BUILD=1 python -u tools/ab_bench.py --spread 1.5 --rounds 3 build_ab/th_base.so build_ab/th_new.so || exit $? ;;
    tests) step pytest_gpu 1100 $PYT tests -m gpu || exit $? ;;
    smoke) step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) step bench 600 python -u bench.py || exit $? ;;
    bench_cfg2) step bench_cfg2 300 python -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" || exit $? ;;
    bench_stress) step bench_stress 300 python -u bench.py --workload stress --steps 2 --warmup 1 --no-cpu --extra-legs "" || exit $? ;;
    trace2) step trace_cfg2 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg2 -o run --output-format csv -- python3 -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" || exit $? ;;
    trace3) step trace_cfg3 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg3 -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --extra-legs "" || exit $? ;;
    tracest) step trace_stress 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_stress -o run --output-format csv -- python3 -u bench.py --workload stress --steps 2 --warmup 1 --no-cpu --extra-legs "" || exit $? ;;
    tracem) step trace_mpc 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_mpc -o run --output-format csv -- python3 -u bench.py --workload mpc --steps 20 --warmup 3 || exit $? ;;
    fetch) step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_fetch -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" || exit $? ;;
    write) step pmc_write 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_write -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" || exit $? ;;
    run2trace) step run2_trace 200 python -u tools/run2_trace.py build_ab/run2_trace.so || exit $? ;;
    general) bash tools/r04_general_profile.sh || exit $? ;;
    tailtrace) step tail_trace_base 200 python -u tools/tail_trace.py build_ab/tail_trace_base.so &&
               step tail_trace_new 200 python -u tools/tail_trace.py build_ab/tail_trace_new.so || exit $? ;;
    stress_ab) step stress_ab 600 env GYM_ALLOW_FOREIGN_BUILD=1 BENCH_ARGS="--workload stress --steps 2 --warmup 1 --no-cpu --extra-legs ''" \
               bash tools/ab_alt_bench.sh r04/stress_ab 2 262144 build_ab/tail_base.so build_ab/tail_new.so || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
