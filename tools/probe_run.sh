#!/bin/bash
# Microbenchmarks on the GPU box: fp64 issue/latency probe, then FETCH_SIZE / WRITE_SIZE calibration passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/probe
mkdir -p $OUT
timeout -k 10 60 tools/fp64_probe > $OUT/fp64_probe.log 2>&1 || exit $?
timeout -k 10 60 tools/fetch_calib > $OUT/fetch_calib_plain.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cal -d $OUT/fetch -o run --output-format csv -- tools/fetch_calib > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cal -d $OUT/write -o run --output-format csv -- tools/fetch_calib > $OUT/write.log 2>&1 || exit $?
echo done
