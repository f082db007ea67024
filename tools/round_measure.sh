#!/bin/bash
# Every GPU measurement of a round, as modes of one script (run from the repo
# root through gpurun; outputs under gpurun_out/, copied to profiles/ by the
# builder, indexed in profiles/INDEX.md):
#
#   tests <pytest args>      the -m gpu suite or a subset       -> tests.log
#   bench <name> <args>      one bench.py line                  -> bench_<name>.json
#   quick                    the driver's C2 line, C2 / 8192 with the
#                            selection pipeline, C5 in LN_SBPLX mode
#   benches                  every workload's bench line
#   profiles                 rocprofv3 kernel stats + HBM PMC passes (profile.sh),
#                            SQ instruction-mix passes (pmc_sq.sh), batch sweep
#   ablation [bench args]    every libmtg_hip_<v>.so variant (build_variant.sh)
#                            against the product library, alternating 3 times;
#                            default the C2 line at K = 200   -> ablation.txt
#   tube                     the tube parity tests, the config-3 line and the
#                            400-seed status agreement with the oracle
#   ab <ENV> <args>          A/B of an environment switch of the library
#                            (e.g. MTG_WAVE2, MTG_STD_RUNTIME_S) on one bench
#                            line, alternating 3 times         -> ab_<ENV>.txt
#   envs                     HIP runtime switches (kernel arguments, graph
#                            packets) on the C2 line at K = 20  -> envs.txt
#   events                   bench.py --events device vs system (timing-event
#                            release scope) on C2 at K = 20 / 200 and B = 8192,
#                            alternating 3 times                -> events.txt
#   stamps                   s_memtime phase stamps of the C2 kernel and the
#                            tube IPM (make STAMPS=1 build first)
#   ubench                   tools/ubench microbenchmarks (built in-tree)
#
# Helpers: tools/profile.sh, tools/pmc_sq.sh, tools/pmc_lds.sh,
# tools/build_variant.sh; summaries: tools/pmc_summary.py,
# tools/sq_summary.py, tools/sq_executed.py, tools/stamps_std.py.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B() { timeout -k 10 300 python bench.py "$@"; }
kline() {  # <json> <tag>: kernel_ms and ms_per_step of a bench line
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us  step', round(d['ms_per_step']*1e3,3), 'us')" "$1" "$2"
}
mode=${1:-benches}
shift || true
case "$mode" in
  tests)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/tests.log 2>&1
    ;;
  bench)
    name=$1; shift
    B "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err
    ;;
  quick)
    B --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_c2_driver.json 2> gpurun_out/bench_c2_driver.err
    B --steps 20 --warmup 5 --select --no-cpu-baseline > gpurun_out/bench_c2_select.json 2> gpurun_out/bench_c2_select.err
    B --steps 20 --warmup 5 --batch 8192 --select --no-cpu-baseline > gpurun_out/bench_8192_select.json 2> gpurun_out/bench_8192_select.err
    B --workload time --steps 5 --warmup 2 --optimizer sbplx > gpurun_out/bench_time_sbplx.json 2> gpurun_out/bench_time_sbplx.err
    ;;
  benches)
    B > gpurun_out/bench_linear.json 2> gpurun_out/bench_linear.err
    B --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_c2_driver.json 2> gpurun_out/bench_c2_driver.err
    B --batch 8192 --no-cpu-baseline > gpurun_out/bench_linear_8192.json 2> gpurun_out/bench_linear_8192.err
    B --batch 8192 --select --no-cpu-baseline > gpurun_out/bench_8192_select.json 2> gpurun_out/bench_8192_select.err
    B --batch 65536 --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/bench_linear_65536.json 2> gpurun_out/bench_linear_65536.err
    B --workload tube --steps 20 --warmup 3 > gpurun_out/bench_tube.json 2> gpurun_out/bench_tube.err
    B --workload time --steps 20 --warmup 3 > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
    B --workload time --optimizer sbplx --steps 20 --warmup 3 > gpurun_out/bench_time_sbplx.json 2> gpurun_out/bench_time_sbplx.err
    B --workload time --soft --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_time_soft.json 2> gpurun_out/bench_time_soft.err
    B --workload time-qcqp --steps 5 --warmup 1 > gpurun_out/bench_time_qcqp.json 2> gpurun_out/bench_time_qcqp.err
    B --workload time-qcqp --optimizer sbplx --steps 3 --warmup 1 > gpurun_out/bench_time_qcqp_sbplx.json 2> gpurun_out/bench_time_qcqp_sbplx.err
    B --workload time --optimizer sbplx --soft --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_time_sbplx_soft.json 2> gpurun_out/bench_time_sbplx_soft.err
    B --workload extrema > gpurun_out/bench_extrema.json 2> gpurun_out/bench_extrema.err
    B --workload sample > gpurun_out/bench_sample.json 2> gpurun_out/bench_sample.err
    B --workload collision --steps 5 --warmup 1 > gpurun_out/bench_collision.json 2> gpurun_out/bench_collision.err
    ;;
  profiles)
    bash tools/profile.sh linear
    bash tools/profile.sh linear_8192 --batch 8192 --steps 20 --warmup 2
    bash tools/profile.sh linear_65536 --batch 65536 --steps 20 --warmup 2
    bash tools/profile.sh tube --workload tube --steps 5 --warmup 1
    bash tools/profile.sh time --workload time --steps 5 --warmup 1
    bash tools/profile.sh time_sbplx --workload time --optimizer sbplx --steps 5 --warmup 1
    bash tools/profile.sh time_qcqp_sbplx --workload time-qcqp --optimizer sbplx --steps 2 --warmup 1
    bash tools/pmc_sq.sh linear
    bash tools/pmc_sq.sh linear_8192 --batch 8192 --steps 20 --warmup 2
    bash tools/pmc_sq.sh linear_65536 --batch 65536 --steps 20 --warmup 2
    bash tools/pmc_sq.sh tube --workload tube --steps 5 --warmup 1
    bash tools/pmc_sq.sh time --workload time --steps 5 --warmup 1
    timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep_linear.jsonl 2>&1
    ;;
  ablation)  # [bench args]: default the C2 line at K = 200
    mkdir -p gpurun_out/abl
    P=mav_tube_trajectory_generation_amd
    args=("$@"); [ ${#args[@]} -eq 0 ] && args=(--steps 200 --warmup 20)
    for rep in 1 2 3; do
      for lib in $P/libmtg_hip.so $P/libmtg_hip_*.so; do
        v=$(basename $lib .so); v=${v#libmtg_hip}; v=${v#_}; v=${v:-base}
        MTG_LIB_PATH=$lib B --no-cpu-baseline "${args[@]}" \
          > gpurun_out/abl/${v}_$rep.json 2> gpurun_out/abl/${v}_$rep.err
        kline gpurun_out/abl/${v}_$rep.json ${v}_$rep
      done
    done | tee gpurun_out/ablation.txt
    ;;
  tube)
    mkdir -p gpurun_out/tube
    timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
      tests/test_tube_gpu.py tests/test_tube_time_gpu.py tests/test_configs_gpu.py -k "tube or config3" \
      > gpurun_out/tube/tests.log 2>&1
    B --workload tube --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/tube/bench.json 2> gpurun_out/tube/bench.err
    kline gpurun_out/tube/bench.json tube
    timeout -k 10 300 python tools/tube_status_agreement.py r06 > gpurun_out/tube/agreement.txt 2>&1
    ;;
  ab)
    env=$1; shift
    mkdir -p gpurun_out/ab
    for rep in 1 2 3; do
      for v in 0 1; do
        env $env=$v timeout -k 10 300 python bench.py --no-cpu-baseline "$@" \
          > gpurun_out/ab/${env}_${v}_$rep.json 2> gpurun_out/ab/${env}_${v}_$rep.err
        kline gpurun_out/ab/${env}_${v}_$rep.json ${env}=${v}_$rep
      done
    done | tee -a gpurun_out/ab_$env.txt
    ;;
  events)
    mkdir -p gpurun_out/ev
    for rep in 1 2 3; do
      for ev in system device; do
        for cfg in "k20:--steps 20 --warmup 5" "k200:--steps 200 --warmup 20" "b8192:--batch 8192 --steps 20 --warmup 5"; do
          tag=${cfg%%:*}; a=${cfg#*:}
          B --no-cpu-baseline --events $ev $a > gpurun_out/ev/${tag}_${ev}_$rep.json 2> gpurun_out/ev/${tag}_${ev}_$rep.err
          kline gpurun_out/ev/${tag}_${ev}_$rep.json ${tag}_${ev}_$rep
        done
      done
    done | tee gpurun_out/events.txt
    ;;
  envs)  # HIP runtime switches on the C2 line at K = 20 (one run each, twice)
    mkdir -p gpurun_out/envs
    for rep in 1 2; do
      for e in ${MTG_ENVS:-NONE=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 \
               HIP_FORCE_DEV_KERNARG=0 HIP_FORCE_DEV_KERNARG=1 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 \
               DEBUG_HIP_KERNARG_COPY_OPT=0 DEBUG_HIP_KERNARG_COPY_OPT=1 ROC_USE_FGS_KERNARG=0}; do
        env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 \
          > gpurun_out/envs/${e}_$rep.json 2> gpurun_out/envs/${e}_$rep.err || { echo "$e failed"; exit 1; }
        kline gpurun_out/envs/${e}_$rep.json ${e}_$rep
      done
    done | tee gpurun_out/envs.txt
    ;;
  stamps)
    STAMPS_SYM=wave MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so \
      timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_c2.txt 2>&1
    MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so \
      timeout -k 10 120 python tools/tube_stamps.py 4096 > gpurun_out/stamps_tube.txt 2>&1
    ;;
  ubench)
    for u in launch_floor fp64_latency store_tail graph_fixed last_arriver fetch_calib; do
      [ -x tools/ubench/$u ] && timeout -k 10 120 tools/ubench/$u > gpurun_out/ubench_$u.txt 2>&1
    done
    ;;
  *)
    echo "unknown mode $mode" >&2
    exit 2
    ;;
esac
echo ALLDONE
