#!/bin/bash
# A/B of the current build against libmtg_hip_base.so (alternating, K = 200
# and the driver's K = 20), after the linear and selection tests; then the
# HBM PMC passes of the current C2 kernel.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_linear_gpu.py tests/test_select_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab3.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_ab3.log; exit 1; }
tail -1 gpurun_out/pytest_ab3.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us  step', round(d['ms_per_step']*1e3,3), ' sel', round(d['config'].get('selection_overhead_ms',0)*1e3,3))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err; line gpurun_out/ab_$tag.json $tag; }
for i in 1 2 3 4; do
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base200_$i --steps 200 --warmup 20
  run new200_$i --steps 200 --warmup 20
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base20_$i --steps 20 --warmup 5
  run new20_$i --steps 20 --warmup 5
done

