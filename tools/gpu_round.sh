#!/bin/bash
# One GPU session for a round's checks: GPU tests, then the cfg 2 / cfg 3 bench lines.  Every GPU step has its
# own time limit; a fault / abort / timeout ends the script (no retries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -q -i -E "illegal memory access|memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" "gpurun_out/$name.log"; then
    echo "GPU fault in $name: stopping"; exit 3
  fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step pytest_gpu 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --tb=short --timeout 300 --timeout-method thread ;;
    cfg2)  step bench_cfg2 300 python -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" ;;
    cfg2s) step bench_cfg2_single 300 python -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" --split-waves off ;;
    cfg3)  step bench_cfg3 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --extra-legs "" ;;
    mpc)   step bench_mpc 300 python -u bench.py --workload mpc --steps 20 --warmup 3 ;;
    full)  step bench_full 900 python -u bench.py ;;
    *) echo "unknown step $s" ;;
  esac
done
