#!/bin/bash
# Straggler-tail threshold sweep on the stress workload (and the headline at the default), one GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${1:-tail_sweep}; shift
mkdir -p "$OUT"
for tl in "$@"; do
  echo "[$(date +%T)] stress tail_lanes=$tl" | tee -a "$OUT/steps.log"
  timeout -k 10 300 python -u bench.py --workload stress --steps 1 --warmup 1 --no-cpu --extra-legs "" \
      --tail-lanes "$tl" > "$OUT/stress_$tl.log" 2>&1 || { echo "rc=$? at $tl"; exit 1; }
  python - "$OUT/stress_$tl.log" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"  {d['value']/1e6:.2f} M it/s  {d['ms_per_step']:.0f} ms/solve  tail {d['straggler_tail']}")
PY
done
