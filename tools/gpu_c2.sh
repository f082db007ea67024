#!/bin/bash
# C2 iteration pass: standard-kernel and time-kernel parity tests, the default
# bench line and the phase stamps of the standard-pattern linear kernel.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_linear_gpu.py tests/test_configs_gpu.py tests/test_time_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_c2.log; exit 1; }
tail -1 gpurun_out/pytest_c2.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'])"
[ -f mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so ] && MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_std.txt 2>&1 && cat gpurun_out/stamps_std.txt || true
timeout -k 10 60 ./tools/ubench/launch_floor > gpurun_out/launch_floor.txt 2>&1 && cat gpurun_out/launch_floor.txt || true
