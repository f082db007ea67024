#!/bin/bash
# Whole measurement pass of a round, in two gpurun calls from the repo root:
#   bash tools/round_measure.sh benches    -- every bench line
#   bash tools/round_measure.sh profiles   -- rocprofv3 kernel stats, HBM PMC
#                                             passes, SQ counters, batch sweep
# Then, in the container: tools/pmc_summary.py / tools/sq_summary.py per tag
#  and copy the bench lines to profiles/<round>_bench_*.json.
set -e -o pipefail
mkdir -p gpurun_out
B() { timeout -k 10 300 python bench.py "$@"; }
case "${1:-benches}" in
  tests)  # bash tools/round_measure.sh tests <test files / pytest args>
    shift
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/tests.log 2>&1
    ;;
  bench)  # bash tools/round_measure.sh bench <name> <bench args>
    name=$2; shift 2
    B "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err
    ;;
  quick)  # the verdict's C2 / selection / SBPLX lines
    B --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_c2_driver.json 2> gpurun_out/bench_c2_driver.err
    B --steps 20 --warmup 5 --select --no-cpu-baseline > gpurun_out/bench_c2_select.json 2> gpurun_out/bench_c2_select.err
    B --steps 20 --warmup 5 --batch 8192 --select --no-cpu-baseline > gpurun_out/bench_8192_select.json 2> gpurun_out/bench_8192_select.err
    B --workload time --steps 5 --warmup 2 --optimizer sbplx > gpurun_out/bench_time_sbplx.json 2> gpurun_out/bench_time_sbplx.err
    ;;
  benches)
    B > gpurun_out/bench_linear.json 2> gpurun_out/bench_linear.err
    B --batch 8192 --no-cpu-baseline > gpurun_out/bench_linear_8192.json 2> gpurun_out/bench_linear_8192.err
    B --batch 65536 --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/bench_linear_65536.json 2> gpurun_out/bench_linear_65536.err
    B --workload tube --steps 20 --warmup 3 > gpurun_out/bench_tube.json 2> gpurun_out/bench_tube.err
    B --workload time --steps 20 --warmup 3 > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
    B --workload time --soft --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_time_soft.json 2> gpurun_out/bench_time_soft.err
    B --workload time-qcqp --steps 5 --warmup 1 > gpurun_out/bench_time_qcqp.json 2> gpurun_out/bench_time_qcqp.err
    B --workload extrema > gpurun_out/bench_extrema.json 2> gpurun_out/bench_extrema.err
    B --workload sample > gpurun_out/bench_sample.json 2> gpurun_out/bench_sample.err
    B --workload collision --steps 5 --warmup 1 > gpurun_out/bench_collision.json 2> gpurun_out/bench_collision.err
    B --batch 8192 --kernel lane --no-cpu-baseline > gpurun_out/bench_linear_8192_lane.json 2> gpurun_out/bench_linear_8192_lane.err
    ;;
  profiles)
    bash tools/profile.sh linear
    bash tools/profile.sh linear_65536 --batch 65536 --steps 20 --warmup 2
    bash tools/profile.sh tube --workload tube --steps 5 --warmup 1
    bash tools/profile.sh time --workload time --steps 5 --warmup 1
    bash tools/pmc_sq.sh tube --workload tube --steps 5 --warmup 1
    bash tools/pmc_sq.sh linear_65536 --batch 65536 --steps 20 --warmup 2
    bash tools/pmc_sq.sh linear
    timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep_linear.jsonl 2>&1
    ;;
esac
echo ALLDONE
