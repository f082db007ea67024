#!/bin/bash
# C5 / C5 + soft bench lines and the time-kernel parity tests.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload time --soft --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_time_soft.json 2> gpurun_out/bench_time_soft.err
timeout -k 10 300 python bench.py --workload time --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
python3 -c "
import json
for f in ['gpurun_out/bench_time.json','gpurun_out/bench_time_soft.json']:
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'])"
timeout -k 10 600 python -u -m pytest tests/test_time_gpu.py tests/test_linear_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_soft.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_soft.log; exit 1; }
tail -1 gpurun_out/pytest_soft.log
