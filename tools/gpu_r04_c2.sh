#!/bin/bash
# C2 iteration: linear parity tests, the driver's command and K = 200, and
# the wave kernel's phase stamps (diagnostic build).
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_linear_gpu.py tests/test_linear_lane_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_c2.log; exit 1; }
tail -1 gpurun_out/pytest_c2.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], round(d['value']/1e6,3), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us', d['roofline'].get('kernel'))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/c2_$tag.json 2> gpurun_out/c2_$tag.err; line gpurun_out/c2_$tag.json $tag; }
run k200 --steps 200 --warmup 20
run k20a --steps 20 --warmup 5
run k20b --steps 20 --warmup 5
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so STAMPS_SYM=mtg_debug_stamps_wave timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_wave.txt 2>&1
cat gpurun_out/stamps_wave.txt
