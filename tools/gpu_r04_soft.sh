#!/bin/bash
# Round-4 soft search (two coefficient arrays live, no MachineLICM in the
# time TU): the time parity tests, then C5 and C5 + soft on the
# compile-time-S kernels and the runtime-S ones (MTG_STD_RUNTIME_S=1).
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_time_gpu.py tests/test_extrema_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_soft.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_soft.log; exit 1; }
tail -1 gpurun_out/pytest_soft.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,4), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3), 'kernel', d['roofline'].get('kernel'))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/sf_$tag.json 2> gpurun_out/sf_$tag.err; line gpurun_out/sf_$tag.json $tag; }
run c5 --workload time --steps 5 --warmup 1
run c5soft --workload time --soft --steps 3 --warmup 1
MTG_STD_RUNTIME_S=1 run c5soft_rt --workload time --soft --steps 3 --warmup 1
run c2 --steps 200 --warmup 20
