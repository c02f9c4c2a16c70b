#!/bin/bash
# Round-6 GPU session: named steps, each under its own time limit, chained so that the first failure (a test
# failure, a fault, an abort, a time limit) ends the script.  Output under gpurun_out/r06/<tag>/<name>.log.
#   R06_TAG=place tools/r06_session.sh avail place p_utcl p_lat p_tccstall p_tcc
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r06/${R06_TAG:-run}
mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] end $name rc=$rc" | tee -a $OUT/steps.log
  tail -4 "$OUT/$name.log" | cut -c1-400
  return $rc
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
PP="python3 -u tools/placement_pmc.py --sets ${PSETS:-6}"
LIB=gymnast_optimalcontrol_amd/libgymnast_acrobot.so
pmc() {  # pmc <name> <format> <counters...>: one rocprofv3 pass over tools/placement_pmc.py, then its summary
  local name=$1 fmt=$2; shift 2
  step $name 300 rocprofv3 --pmc "$@" --kernel-include-regex k_nt_phase -d $OUT/$name -o run --output-format $fmt \
    -- $PP --out $OUT/$name/run.json || return $?
  step ${name}_parse 120 python3 -u tools/placement_pmc_parse.py $OUT/$name $OUT/$name/run.json $OUT/$name/summary.json \
    || return $?
  rm -f $OUT/$name/*/*.db $OUT/$name/*.db 2>/dev/null
  return 0
}
for s in "$@"; do
  case $s in
    avail) step list_avail 120 rocprofv3 --list-avail || exit $? ;;
    place) step place 300 $PP --out $OUT/place.json || exit $? ;;
    place2) step place2 300 $PP --out $OUT/place2.json || exit $? ;;
    scan) step scan 400 python3 -u tools/placement_scan.py --out $OUT/scan.json || exit $? ;;
    p_utcl) pmc p_utcl csv TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum \
              TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE || exit $? ;;
    p_lat) pmc p_lat csv TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum \
              TCP_TCR_TCP_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum || exit $? ;;
    p_tccstall) pmc p_tccstall csv TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum \
              TCC_BUSY_sum || exit $? ;;
    p_tcc) pmc p_tcc "csv rocpd" TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ_LEVEL || exit $? ;;
    timeline) step stress_timeline 300 python3 -u tools/stress_timeline.py || exit $? ;;
    tracest) step trace_stress 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_stress -o run --output-format csv -- python3 -u bench.py --workload stress --steps 2 --warmup 1 --no-cpu --no-box --extra-legs "" || exit $? ;;
    gaps) step trace_gaps 120 python3 -u tools/trace_gaps.py $OUT/trace_cfg3 || exit $? ;;
    fetch) step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_fetch -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-box --no-timing --max-iters 20 --extra-legs "" || exit $? ;;
    write) step pmc_write 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_" -d $OUT/pmc_write -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-box --no-timing --max-iters 20 --extra-legs "" || exit $? ;;
    valu) step pmc_valu 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_nt_" -d $OUT/pmc_valu -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-box --no-timing --max-iters 20 --extra-legs "" || exit $? ;;
    wltest) step pytest_workloads 600 $PYT tests/test_gpu_workloads.py -m gpu -k "rank_share" || exit $? ;;
    l6) step layout6 300 python3 -u tools/layout6_probe.py --out $OUT/l6.json || exit $? ;;
    l6b) step layout6b 300 python3 -u tools/layout6_probe.py --sep-sets 6 --rec-sets 6 --seconds 0.6 --out $OUT/l6b.json || exit $? ;;
    l6c) step layout6c 300 python3 -u tools/layout6_probe.py --sep-sets 6 --rec-sets 6 --seconds 0.6 --out $OUT/l6c.json || exit $? ;;
    lsearch) step layout_search 400 python3 -u tools/layout_search.py --out $OUT/search.json || exit $? ;;
    pvk) step probe_vs_kernel 300 python3 -u tools/probe_vs_kernel.py --out $OUT/pvk.json || exit $? ;;
    pvk2) step probe_vs_kernel2 300 python3 -u tools/probe_vs_kernel.py --out $OUT/pvk2.json || exit $? ;;
    greedy) step greedy 300 python3 -u tools/greedy_streams.py --out $OUT/g.json || exit $? ;;
    greedy2) step greedy2 300 python3 -u tools/greedy_streams.py --out $OUT/g2.json || exit $? ;;
    cfg2ab) step cfg2_4waves 300 python3 -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" && step cfg2_1wave 300 python3 -u bench.py --batch 4096 --steps 5 --warmup 1 --no-cpu --extra-legs "" --split-waves off || exit $? ;;
    first) step first_solve 300 python3 -u tools/first_solve.py --out $OUT/first.json || exit $? ;;
    tietest) step pytest_ties 300 $PYT tests/test_gpu_stress.py -m gpu -k tie_lanes -s || exit $? ;;
    ttest) step pytest_tracking 300 $PYT tests/test_tracking.py -m gpu || exit $? ;;
    ptest) step pytest_place 300 $PYT tests/test_gpu_parity.py -m gpu -k placement || exit $? ;;
    benchmain) step benchmain 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --extra-legs "" || exit $? ;;
    tests) step pytest_gpu 1100 $PYT tests -m gpu || exit $? ;;
    smoke) step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) step bench 600 python -u bench.py || exit $? ;;
    bench20) step bench20 600 python -u bench.py --steps 20 --warmup 2 --extra-legs "" || exit $? ;;
    main20a) step main20a 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --extra-legs "" || exit $? ;;
    main20b) step main20b 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --extra-legs "" || exit $? ;;
    driver) step bench_driver 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $? ;;
    trace3) step trace_cfg3 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_cfg3 -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-box --extra-legs "" || exit $? ;;
    two) GYM_DIST_BACKEND=gloo step bench_2rank 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
           --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 || exit $? ;;
    four) GYM_DIST_BACKEND=gloo step bench_4rank 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
           --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1 || exit $? ;;
    pd2cmp) GYM_ALLOW_FOREIGN_BUILD=1 step pd2_compare 300 python3 -u tools/compare_libs.py $LIB build_ab/libpd2.so --batch 131072 --iters 6 \
              --schedule pipelined || exit $? ;;
    pd2ab) for b in ${PD2_BATCHES:-131072 98304 196608 262144}; do
             GYM_ALLOW_FOREIGN_BUILD=1 step pd2_ab_$b 400 python3 -u tools/ab_bench.py --batch $b --rounds 3 $LIB:pipe build_ab/libpd2.so:pipe \
               || exit $?; done ;;
    spread) for b in ${SP_BATCHES:-114688 131072 163840 196608 262144}; do
             GYM_ALLOW_FOREIGN_BUILD=1 step spread_ab_$b 400 python3 -u tools/ab_bench.py --batch $b --rounds 3 \
               build_ab/libA.so:pipe build_ab/libB.so:pipe build_ab/libC.so:pipe build_ab/libD.so:pipe || exit $?; done ;;
    lotest) step pytest_lo 600 $PYT tests/test_gpu_workloads.py -m gpu -k "two_wavefront or rank_share" || exit $? ;;
    sharebench) step bench_share 600 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --extra-legs cfg4share,cfg4 \
                  || exit $? ;;
    w3ab) for b in ${W3_BATCHES:-147456 163840 180224 196608}; do
             GYM_ALLOW_FOREIGN_BUILD=1 step w3_ab_$b 400 python3 -u tools/ab_bench.py --batch $b --rounds 3 $LIB:pipe \
               build_ab/libw3.so:pipe || exit $?; done ;;
    pmc131) 
            step pmc131_fetch 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_nt_phase" -d $OUT/pmc131_fetch -o run --output-format csv -- python3 -u bench.py --batch 131072 --steps 1 --warmup 0 --no-cpu --no-box --no-timing --max-iters 20 --extra-legs "" && \
            step pmc131_write 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_nt_phase" -d $OUT/pmc131_write -o run --output-format csv -- python3 -u bench.py --batch 131072 --steps 1 --warmup 0 --no-cpu --no-box --no-timing --max-iters 20 --extra-legs "" && \
            step trace131 300 rocprofv3 --kernel-trace --stats -d $OUT/trace131 -o run --output-format csv -- python3 -u bench.py --batch 131072 --steps 3 --warmup 1 --no-cpu --no-box --extra-legs "" || exit $? ;;
    curve) for b in ${CURVE_BATCHES:-16384 32768 65536 98304 131072 196608 262144 393216 524288 1048576}; do
             step curve_$b 300 python3 -u bench.py --batch $b --steps 2 --warmup 1 --no-cpu --no-box --extra-legs "" \
               || exit $?; done ;;
    sched) for b in ${SCHED_BATCHES:-16384 24576 32768 40960 49152}; do for sc in serial pipelined persistent; do
             step sched_${b}_$sc 300 python3 -u bench.py --batch $b --steps 3 --warmup 1 --no-cpu --no-box --extra-legs "" \
               --schedule $sc || exit $?; done; done ;;
    small) for b in 16384 24576 32768; do
             step small_$b 300 python3 -u bench.py --batch $b --steps 3 --warmup 1 --no-cpu --no-box --extra-legs "" \
               || exit $?; done ;;
    mid) for b in ${MID_BATCHES:-98304 114688 118784 122880 126976}; do for sc in serial pipelined; do
             step mid_${b}_$sc 300 python3 -u bench.py --batch $b --steps 3 --warmup 1 --no-cpu --no-box --extra-legs "" \
               --schedule $sc || exit $?; done; done ;;
    cfg1prof) step cfg1_cprofile 300 python3 -u tools/cfg1_profile.py --cprofile $OUT/cfg1_cprofile.txt && \
              step cfg1_trace 300 rocprofv3 --kernel-trace --stats -d $OUT/cfg1_trace -o run --output-format csv -- \
                python3 -u tools/cfg1_profile.py || exit $? ;;
    sigtest) step pytest_sig 600 $PYT tests/test_gpu_parity.py tests/test_armijo_sweep.py tests/test_report.py \
               -m gpu -k "streamed_sigma or task2 or task1 or batched_lanes or armijo or reference_history or report" \
               && step pytest_sig2 600 $PYT tests/test_gpu_workloads.py -m gpu -k "capture_lanes" || exit $? ;;
    cfg1) step cfg1_time 300 python3 -u tools/cfg1_profile.py || exit $? ;;
    tailsw) for tl in ${TAIL_SET:-1024 2048 512}; do
             step tail_$tl 300 python3 -u bench.py --workload stress --steps 2 --warmup 1 --no-cpu --no-box --extra-legs "" \
               --tail-lanes $tl || exit $?; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
