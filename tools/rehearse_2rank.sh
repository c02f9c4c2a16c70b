#!/bin/bash
# 2-rank rehearsal of the default bench on ONE GPU (gloo: RCCL refuses two ranks on one device)
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
GYM_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --extra-steps 1 \
  > gpurun_out/rehearse_2rank.log 2>&1
rc=$?; tail -3 gpurun_out/rehearse_2rank.log | cut -c1-1500; exit $rc
