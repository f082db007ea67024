#!/bin/bash
# Round-4 compile-time-S wave kernel: its parity tests first, then the C2
# bench (K = 200 and the driver's K = 20, with and without device kernel
# arguments), then stamps.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_linear_gpu.py tests/test_linear_lane_gpu.py tests/test_select_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_wave.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_wave.log; exit 1; }
tail -2 gpurun_out/pytest_wave.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us  sel', round(d['config'].get('selection_overhead_ms',0)*1e3,3))" "$1" "$2"; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/w_new_$i.json 2> gpurun_out/w_new_$i.err; line gpurun_out/w_new_$i.json new200
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/w_new20_$i.json 2> gpurun_out/w_new20_$i.err; line gpurun_out/w_new20_$i.json new20
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/w_dk20_$i.json 2> gpurun_out/w_dk20_$i.err; line gpurun_out/w_dk20_$i.json devkarg20
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/w_dk200_$i.json 2> gpurun_out/w_dk200_$i.err; line gpurun_out/w_dk200_$i.json devkarg200
done
STAMPS_SYM=wave MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_wave.txt 2>&1
cat gpurun_out/stamps_wave.txt
