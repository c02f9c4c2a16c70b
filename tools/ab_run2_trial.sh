#!/bin/bash
# A/B of the pair-trial load-wait variants of k_nt_run2 (build_ab/v*.so, v*_tr.so; tools/ab_run2_trial.py builds them)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-ab_run2_trial}; mkdir -p "$OUT"; shift
for v in "$@"; do
  timeout -k 10 120 python -u tools/run2_trace.py build_ab/${v}_tr.so --batch 4096 --iters 40 > "$OUT/trace_$v.log" 2>&1 || { echo "trace $v rc=$?"; tail -5 "$OUT/trace_$v.log"; exit 1; }
  grep "per stage" "$OUT/trace_$v.log" | sed "s/^/$v /"
done
args=""; for v in "$@"; do args="$args build_ab/$v.so:run"; done
timeout -k 10 400 python -u tools/ab_bench.py --batch 4096 --rounds 5 $args > "$OUT/ab.log" 2>&1 || { echo "ab rc=$?"; tail -5 "$OUT/ab.log"; exit 1; }
tail -8 "$OUT/ab.log"
