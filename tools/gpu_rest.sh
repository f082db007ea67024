#!/bin/bash
# Bench lines of the workloads not in gpu_preload.sh: the QCQP time objective
# and the lane kernel forced at one C4 shard.
set -e -o pipefail
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/pl_$tag.json 2> gpurun_out/pl_$tag.err; python3 -c "import json; d=json.load(open('gpurun_out/pl_$tag.json')); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], (r.get('hbm') or {}).get('frac'))"; }
run timeqcqp --workload time-qcqp --steps 5 --warmup 1
run lane8192 --batch 8192 --kernel lane
