#!/bin/bash
# Host-side sanitizer run of the C oracle (oracle/acrobot_oracle.c): an ASan + UBSan build, loaded into a Python
# process with the sanitizer runtimes preloaded, solving short, ragged and full horizons with a NaN lane.
# CPU only (this container); the GPU box runs no sanitizers.
set -euo pipefail
cd "$(dirname "$0")/.."
out=${TMPDIR:-/tmp}/gym_asan
mkdir -p "$out"
gcc -O1 -g -fPIC -fopenmp -std=c11 -Wall -Wextra -fsanitize=address,undefined -fno-omit-frame-pointer \
    -fno-sanitize-recover=undefined -shared -o "$out/libacrobot_oracle.so" oracle/acrobot_oracle.c -lm
cat > "$out/run.py" <<PY
import sys
import numpy as np
sys.path.insert(0, "$PWD")
import oracle.c_oracle as co
co._SO = "$out/libacrobot_oracle.so"
from bench import load_refs
xr, ur = load_refs()
for N in (2, 3, 37, 501):
    x0 = np.zeros((9, 4)); x0[1:, :2] = np.random.default_rng(N).uniform(-1.5, 1.5, (8, 2)); x0[4] = np.nan
    o = co.newton_solve(x0, xr[:N], ur[:N - 1], max_iters=60, tol=1e-4, gamma_0=0.1)
    print("N", N, "iterations", o["n_iter"].tolist(), "status", o["status"].tolist())
x = np.random.default_rng(0).normal(size=(64, 4)); u = np.random.default_rng(1).normal(size=(64, 2))
co.rk4(x, u); co.jacobians(x, u)
print("sanitized oracle run: no reports")
PY
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 OMP_NUM_THREADS=4 \
    LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" python "$out/run.py"
