#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box through gpurun).
#   kernel trace + stats over a full bench step; then separate PMC passes (never combined with
#   runtime / sys traces) on a short 20-iteration solve, restricted to the solver kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
fault() { grep -q -i -E "illegal memory access|memory access fault|hipErrorIllegalAddress" "$1"; }
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  if [ $rc -ge 124 ] || fault "$OUT/$name.log"; then echo "stopping after $name"; exit $rc; fi
}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
BENCH="bench.py --steps 1 --warmup 1 --no-cpu"
SHORT="bench.py --steps 1 --warmup 0 --no-cpu --no-timing --max-iters 20"
SCHED="--schedule ${SCHEDULE:-auto}"
for s in "$@"; do
  case $s in
    trace) run trace 900 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH ;;
    fetch) run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_fetch -o run --output-format csv -- python3 $SHORT ;;
    write) run pmc_write 900 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_write -o run --output-format csv -- python3 $SHORT ;;
    valu)  run pmc_valu 900 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_nt_" -d $OUT/pmc_valu -o run --output-format csv -- python3 $SHORT ;;
    stall) run pmc_stall 900 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "k_nt_" -d $OUT/pmc_stall -o run --output-format csv -- python3 $SHORT $SCHED ;;
    *) echo "unknown $s" ;;
  esac
done
