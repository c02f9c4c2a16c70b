#!/bin/bash
# One GPU session (round 3 on): the named steps in order, each under its own time limit.  pytest steps may end
# with status 1 (test failures: read the log, go on); any other non-zero status -- and any status from a bench,
# smoke or profiler step -- ends the script, as does a GPU fault string in a log.  No retries.
#   tools/gpu_session.sh <out-subdir> <step>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${1:?out subdir}; shift
mkdir -p "$OUT"
fault() { grep -q -i -E "illegal memory access|memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" "$1"; }
run() {  # run <tests|fatal> <name> <seconds> <cmd...>
  local kind=$1 name=$2 secs=$3; shift 3
  echo "[$(date +%T)] start $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.log" | cut -c1-400
  if fault "$OUT/$name.log"; then echo "GPU fault in $name: stopping"; exit 3; fi
  if [ $rc -ne 0 ]; then
    if [ "$kind" = tests ] && [ $rc -eq 1 ]; then return 0; fi
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
}
PYT="python -u -m pytest -p no:cacheprovider --tb=short --timeout 300 --timeout-method thread"
for s in "$@"; do
  case $s in
    smoke)   run fatal smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests)   run tests pytest_gpu 1100 $PYT tests -m gpu -v ;;
    t:*)     run tests "pytest_${s#t:}" 600 $PYT tests -m gpu -v -k "${s#t:}" ;;
    cfg3)    run fatal bench_cfg3 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --extra-legs "" ;;
    cfg2)    run fatal bench_cfg2 300 python -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" ;;
    stress)  run fatal bench_stress 400 python -u bench.py --workload stress --steps 2 --warmup 1 --no-cpu --extra-legs "" ;;
    mpc)     run fatal bench_mpc 300 python -u bench.py --workload mpc --steps 20 --warmup 3 ;;
    two)     run fatal bench_2rank 400 env GYM_DIST_BACKEND=gloo python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --extra-legs cfg4 ;;
    full)    run fatal bench_full 900 python -u bench.py ;;
    trace3)  run fatal trace_cfg3 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_cfg3" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --extra-legs "" ;;
    trace2)  run fatal trace_cfg2 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_cfg2" -o run --output-format csv -- python3 bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" ;;
    fetch)   run fatal pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_" -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" ;;
    write)   run fatal pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_" -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
