#!/bin/bash
# Throughput vs lanes per GPU (occupancy sweep) -- measurement tool.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for b in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --batch $b > gpurun_out/sweep_$b.log 2>&1
  rc=$?
  python3 - "$b" <<'PY'
import json, re, sys
b = sys.argv[1]
s = open(f"gpurun_out/sweep_{b}.log").read()
m = re.search(r'(\{"metric.*\})', s)
if m:
    d = json.loads(m.group(1))
    k = d.get("kernels", {})
    print(f"batch {b}: value {d['value']/1e6:.2f} M it/s  bwd {k.get('backward',{}).get('avg_ms',0):.3f} ms  trial {k.get('trial',{}).get('avg_ms',0):.3f} ms  iters {d['parity']['outer_iterations']}")
else:
    print(f"batch {b}: no result"); print(s[-2000:])
PY
  if [ $rc -ne 0 ]; then exit $rc; fi
done
