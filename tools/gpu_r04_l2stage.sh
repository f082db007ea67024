#!/bin/bash
# Lane-pair kernel with the coefficients staged in LDS and copied out
# coalesced (and the wave kernel likewise): parity tests, then the kernel
# time at 2048 .. 65536 and at C2.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_linear_lane_gpu.py tests/test_linear_gpu.py tests/test_select_gpu.py tests/test_configs_gpu.py > gpurun_out/l2s_tests.log 2>&1 || { tail -30 gpurun_out/l2s_tests.log; exit 1; }
tail -2 gpurun_out/l2s_tests.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us', d['roofline'].get('kernel'), 'value', round(d['value']/1e6,1))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/l2s_$tag.json 2> gpurun_out/l2s_$tag.err; line gpurun_out/l2s_$tag.json $tag; }
for b in 2048 2560 4096 8192 65536; do
  run pair_$b --batch $b --kernel lane_pair --steps 100 --warmup 10
done
run std_2048 --batch 2048 --kernel standard --steps 100 --warmup 10
run auto_8192 --batch 8192 --steps 20 --warmup 5
for rep in 1 2; do
  run c2_k200_$rep --steps 200 --warmup 20
  run c2_k20_$rep --steps 20 --warmup 5
done
