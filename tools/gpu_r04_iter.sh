#!/bin/bash
# Round-4 C2 iteration: wave-kernel parity tests, batch sweep, K = 20 line,
# stamps.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_linear_gpu.py tests/test_linear_lane_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3))" "$1" "$2"; }
for B in 256 512 1024 2048; do
  timeout -k 10 300 python bench.py --batch $B --kernel standard --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/it_$B.json 2> gpurun_out/it_$B.err; line gpurun_out/it_$B.json B$B
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/it_k20.json 2> gpurun_out/it_k20.err; line gpurun_out/it_k20.json K20
timeout -k 10 300 python bench.py --batch 8192 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/it_8192.json 2> gpurun_out/it_8192.err; line gpurun_out/it_8192.json lane2_B8192
timeout -k 10 300 python bench.py --batch 65536 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/it_65536.json 2> gpurun_out/it_65536.err; line gpurun_out/it_65536.json lane2_B65536
STAMPS_SYM=wave MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_wave.txt 2>&1
cat gpurun_out/stamps_wave.txt
