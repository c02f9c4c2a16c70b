#!/bin/bash
# Round-2 evidence run (one GPU box): kernel traces of the processes that print the bench lines, PMC passes of the
# dominant kernel, the GPU test suite and a default bench run.  Every GPU step has its own time limit; a fault /
# abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r02
mkdir -p $OUT
fault() { grep -q -i -E "illegal memory access|memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" "$1"; }
run() {  # run <name> <seconds> <cmd...>   (status 1 is tolerated for the pytest step only)
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log" | cut -c1-300
  if fault "$OUT/$name.log"; then echo "GPU fault in $name: stopping"; exit 3; fi
  if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [ "$name" = pytest_gpu ]; }; then echo "stopping after $name"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    trace3) run trace_cfg3 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --extra-legs "" ;;
    trace2) run trace_cfg2 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg2 -o run --output-format csv -- python3 bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" ;;
    tracem) run trace_mpc 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_mpc -o run --output-format csv -- python3 bench.py --workload mpc --steps 20 --warmup 3 ;;
    fetch) run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" ;;
    write) run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" ;;
    valu)  run pmc_valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_nt_" -d $OUT/pmc_valu -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" ;;
    fetch2) run pmc_fetch_cfg2 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_run" -d $OUT/pmc_fetch_cfg2 -o run --output-format csv -- python3 bench.py --batch 4096 --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" ;;
    write2) run pmc_write_cfg2 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_run" -d $OUT/pmc_write_cfg2 -o run --output-format csv -- python3 bench.py --batch 4096 --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20 --extra-legs "" ;;
    fetchm) run pmc_fetch_mpc 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_track|k_mpc" -d $OUT/pmc_fetch_mpc -o run --output-format csv -- python3 bench.py --workload mpc --steps 2 --warmup 1 ;;
    writem) run pmc_write_mpc 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_track|k_mpc" -d $OUT/pmc_write_mpc -o run --output-format csv -- python3 bench.py --workload mpc --steps 2 --warmup 1 ;;
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --tb=short --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench_default 900 python -u bench.py ;;
    *) echo "unknown $s" ;;
  esac
done
