#!/bin/bash
# Round 4: the general (tau1-streaming) phase kernel beside the specialised one, same process (tools/phase_pair.py):
# kernel trace, FETCH_SIZE, WRITE_SIZE and an SQ instruction / cycle pass, each in its own rocprofv3 run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r04_general
mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-300
  return $rc
}
step plain 120 python3 -u tools/phase_pair.py &&
step trace 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 -u tools/phase_pair.py &&
step fetch 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_phase" -d $OUT/fetch -o run --output-format csv -- python3 -u tools/phase_pair.py --rounds 1 --iters 8 &&
step write 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_phase" -d $OUT/write -o run --output-format csv -- python3 -u tools/phase_pair.py --rounds 1 --iters 8 &&
step sq 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex "k_nt_phase" -d $OUT/sq -o run --output-format csv -- python3 -u tools/phase_pair.py --rounds 1 --iters 8
