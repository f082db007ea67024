#!/bin/bash
# Kernarg-preload build: every -m gpu test, smoke, the default bench and the
# other workloads' bench lines (no CPU baselines).
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh
tail -1 gpurun_out/pytest_gpu.log
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('C2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/pl_$tag.json 2> gpurun_out/pl_$tag.err; python3 -c "import json; d=json.load(open('gpurun_out/pl_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
run l8192 --batch 8192
run l65536 --batch 65536 --steps 50 --warmup 5
run sel8192 --batch 8192 --select
run tube --workload tube --steps 10 --warmup 2
run time --workload time --steps 5 --warmup 1
run soft --workload time --soft --steps 3 --warmup 1
run extrema --workload extrema
run sample --workload sample
run coll --workload collision --steps 5 --warmup 1
