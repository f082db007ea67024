#!/bin/bash
# Lane-pair staging from 4096 trajectories only: parity tests and times.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_linear_lane_gpu.py tests/test_linear_gpu.py tests/test_select_gpu.py tests/test_configs_gpu.py tests/test_time_gpu.py > gpurun_out/l2s2_tests.log 2>&1 || { tail -30 gpurun_out/l2s2_tests.log; exit 1; }
tail -2 gpurun_out/l2s2_tests.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us', d['roofline'].get('kernel'), 'value', round(d['value']/1e6,1))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/l2s2_$tag.json 2> gpurun_out/l2s2_$tag.err; line gpurun_out/l2s2_$tag.json $tag; }
for b in 2048 2560 3072 4096 8192 65536; do
  run pair_$b --batch $b --kernel lane_pair --steps 100 --warmup 10
done
run std_2560 --batch 2560 --kernel standard --steps 100 --warmup 10
run std_3072 --batch 3072 --kernel standard --steps 100 --warmup 10
