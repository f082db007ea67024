#!/bin/bash
# Round-3 pass: phase stamps of the standard linear kernel, C5 / C5 + soft
# bench lines and the rocprofv3 kernel stats of the C5 + soft launch.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_std.txt 2>&1
cat gpurun_out/stamps_std.txt
timeout -k 10 300 python bench.py --workload time --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
timeout -k 10 300 python bench.py --workload time --soft --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_time_soft.json 2> gpurun_out/bench_time_soft.err
python3 -c "
import json
for f in ['gpurun_out/bench_time.json','gpurun_out/bench_time_soft.json']:
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_soft -o run -- python3 bench.py --workload time --soft --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_soft.log 2>&1
find gpurun_out/prof_soft -name "*stats*"
