#!/bin/bash
# A/B: three-address Horner steps (GYM_HORNER_VOP3) in the solver kernels; tracking tests + MPC bench first.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
bash tools/mpc_check.sh || exit $?
timeout -k 10 300 python -u tools/ab_bench.py --batch 4096 --rounds 3 build_ab/base.so build_ab/vop3.so > gpurun_out/ab_vop3_4096.log 2>&1 || exit $?
tail -6 gpurun_out/ab_vop3_4096.log
timeout -k 10 300 python -u tools/ab_bench.py --batch 262144 --rounds 2 build_ab/base.so build_ab/vop3.so > gpurun_out/ab_vop3_262144.log 2>&1 || exit $?
tail -6 gpurun_out/ab_vop3_262144.log
