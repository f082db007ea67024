#!/bin/bash
# Bench lines for every workload (run via gpurun from the repo root).
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_linear.json 2> gpurun_out/bench_linear.err
timeout -k 10 300 python bench.py --batch 8192 --no-cpu-baseline > gpurun_out/bench_linear_8192.json 2> gpurun_out/bench_linear_8192.err
timeout -k 10 300 python bench.py --batch 65536 --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/bench_linear_65536.json 2> gpurun_out/bench_linear_65536.err
timeout -k 10 300 python bench.py --workload tube --steps 10 --warmup 2 > gpurun_out/bench_tube.json 2> gpurun_out/bench_tube.err
timeout -k 10 300 python bench.py --workload time --steps 20 --warmup 3 > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
timeout -k 10 300 python bench.py --workload time-qcqp --steps 5 --warmup 1 > gpurun_out/bench_time_qcqp.json 2> gpurun_out/bench_time_qcqp.err
echo ALLDONE
