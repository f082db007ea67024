#!/bin/bash
# Round-3 pass: standard/time parity tests, C2 bench line, C5 and C5 + soft
# bench lines, rocprofv3 kernel stats of C2 and of the C5 + soft launch.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_linear_gpu.py tests/test_configs_gpu.py tests/test_time_gpu.py tests/test_linear_lane_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_c2.log; exit 1; }
tail -1 gpurun_out/pytest_c2.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print('C2 value', d['value'], 'ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'])"
timeout -k 10 300 python bench.py --workload time --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
timeout -k 10 300 python bench.py --workload time --soft --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_time_soft.json 2> gpurun_out/bench_time_soft.err
python3 -c "
import json
for f in ['gpurun_out/bench_time.json','gpurun_out/bench_time_soft.json']:
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_soft -o run -- python3 bench.py --workload time --soft --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_soft.log 2>&1
find gpurun_out/prof_c2 gpurun_out/prof_soft -name "*stats*"
