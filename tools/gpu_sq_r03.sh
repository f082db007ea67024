#!/bin/bash
# Round-3 counter refresh on the final build: SQ counters and kernel stats
# for C2, C5 and C5 + soft.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_sq.sh linear --steps 200 --warmup 20 > gpurun_out/sq_linear.log 2>&1
bash tools/pmc_sq.sh time --workload time --steps 3 --warmup 1 > gpurun_out/sq_time.log 2>&1
bash tools/pmc_sq.sh time_soft --workload time --soft --steps 3 --warmup 1 > gpurun_out/sq_time_soft.log 2>&1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print('C2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
find gpurun_out/sq_linear gpurun_out/sq_time gpurun_out/sq_time_soft -name "*kernel_stats.csv"
