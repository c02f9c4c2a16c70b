#!/bin/bash
# bench.py's cfg 2 line in alternating processes, one library variant per process (GYM_LIB_PATH):
#   tools/ab_alt_bench.sh <out-subdir> <rounds> <batch> build_ab/a.so build_ab/b.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/$1; R=$2; B=$3; shift 3; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for lib in "$@"; do
    v=$(basename "$lib" .so)
    GYM_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --batch "$B" --steps 5 --warmup 1 --no-cpu --extra-legs "" > "$OUT/${v}_$r.log" 2>&1 || { echo "$v rc=$?"; tail -5 "$OUT/${v}_$r.log"; exit 1; }
    grep '^{' "$OUT/${v}_$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $r, round(d['value']/1e6,4), round(d['ms_per_step'],3))"
  done
done
