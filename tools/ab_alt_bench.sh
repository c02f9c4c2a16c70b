#!/bin/bash
# bench.py in alternating processes, one library variant per process (GYM_LIB_PATH):
#   tools/ab_alt_bench.sh <out-subdir> <rounds> <batch> build_ab/a.so build_ab/b.so ...
# BENCH_ARGS overrides the bench arguments after --batch (default: the cfg 2 line's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/$1; R=$2; B=$3; shift 3; mkdir -p "$OUT"
ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu --extra-legs ""}
for r in $(seq 1 "$R"); do
  for lib in "$@"; do
    v=$(basename "$lib" .so)
    eval "GYM_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --batch $B $ARGS" > "$OUT/${v}_$r.log" 2>&1 || { echo "$v rc=$?"; tail -5 "$OUT/${v}_$r.log"; exit 1; }
    grep '^{' "$OUT/${v}_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $r, round(d['value']/1e6,4), round(d['ms_per_step'],3), (d.get('roofline') or {}).get('frac'))"
  done
done
