#!/bin/bash
# Lane-pair kernel with LDS-staged inputs: lane tests, then B = 8192 and
# 65536 against libmtg_hip_base.so, alternating.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_linear_lane_gpu.py tests/test_linear_gpu.py tests/test_select_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_l2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_l2.log; exit 1; }
tail -1 gpurun_out/pytest_l2.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us', d['roofline']['kernel'])" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/l2_$tag.json 2> gpurun_out/l2_$tag.err; line gpurun_out/l2_$tag.json $tag; }
for i in 1 2 3; do
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base8k_$i --batch 8192 --steps 200 --warmup 20
  run new8k_$i --batch 8192 --steps 200 --warmup 20
done
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base64k --batch 65536 --steps 50 --warmup 5
run new64k --batch 65536 --steps 50 --warmup 5
run new4k --batch 4096 --steps 200 --warmup 20
