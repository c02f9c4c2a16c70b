#!/bin/bash
# Throughput of the solver schedules at the given batch sizes (measurement tool); SCHEDS selects them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for b in "$@"; do
  for s in ${SCHEDS:-serial pipelined persistent}; do
    timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --extra-legs '' --batch $b --schedule $s > gpurun_out/sched_${b}_$s.log 2>&1
    rc=$?
    python3 - "$b" "$s" <<'PY'
import json, re, sys
b, s = sys.argv[1], sys.argv[2]
t = open(f"gpurun_out/sched_{b}_{s}.log").read()
m = re.search(r'(\{"metric.*\})', t)
if m:
    d = json.loads(m.group(1))
    print(f"batch {b:>7} {s:>9}: {d['value']/1e6:7.2f} M it/s  {d['ms_per_step']:8.1f} ms/solve  iters {d['parity']['outer_iterations']}")
else:
    print(f"batch {b} {s}: no result"); print(t[-1500:])
PY
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
