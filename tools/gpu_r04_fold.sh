#!/bin/bash
# End-vertex terms folded into the wave solver's assembly: linear, time and
# config tests, then C2 A/B against libmtg_hip_base.so and C5.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_linear_gpu.py tests/test_linear_lane_gpu.py tests/test_time_gpu.py tests/test_configs_gpu.py tests/test_select_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_fold.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_fold.log; exit 1; }
tail -1 gpurun_out/pytest_fold.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us')" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/fd_$tag.json 2> gpurun_out/fd_$tag.err; line gpurun_out/fd_$tag.json $tag; }
for i in 1 2 3 4; do
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base200_$i --steps 200 --warmup 20
  run new200_$i --steps 200 --warmup 20
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base20_$i --steps 20 --warmup 5
  run new20_$i --steps 20 --warmup 5
done
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run c5base --workload time --steps 5 --warmup 1
run c5new --workload time --steps 5 --warmup 1
