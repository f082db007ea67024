#!/bin/bash
# Runtime-S standard kernel with staged coefficient outputs: parity tests and
# its C2 time (MTG_STD_RUNTIME_S=1 forces it where the wave kernel exists).
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_linear_gpu.py tests/test_linear_lane_gpu.py tests/test_free_gpu.py tests/test_configs_gpu.py > gpurun_out/stds_tests.log 2>&1 || { tail -30 gpurun_out/stds_tests.log; exit 1; }
tail -2 gpurun_out/stds_tests.log
MTG_STD_RUNTIME_S=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_linear_gpu.py > gpurun_out/stds_tests_rt.log 2>&1 || { tail -30 gpurun_out/stds_tests_rt.log; exit 1; }
tail -2 gpurun_out/stds_tests_rt.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us', d['roofline'].get('kernel'))" "$1" "$2"; }
for rep in 1 2; do
  MTG_STD_RUNTIME_S=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/stds_rt_$rep.json 2> gpurun_out/stds_rt_$rep.err
  line gpurun_out/stds_rt_$rep.json rt_$rep
done
# A/B: the same with the previous mtg_linear_std.o (per-lane stores), linked
# into libmtg_hip_stdold.so in the container (not committed).
if [ -f mav_tube_trajectory_generation_amd/libmtg_hip_stdold.so ]; then
  for rep in 1 2; do
    MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stdold.so MTG_STD_RUNTIME_S=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/stds_old_$rep.json 2> gpurun_out/stds_old_$rep.err
    line gpurun_out/stds_old_$rep.json old_$rep
  done
fi
