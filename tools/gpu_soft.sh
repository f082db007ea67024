#!/bin/bash
# GPU pass for the soft-constraint time objective: tests and the C5 + soft
# bench line with its kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_time_gpu.py tests/test_extrema_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_soft.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_soft.log; exit 1; }
tail -2 gpurun_out/pytest_soft.log
timeout -k 10 300 python bench.py --workload time --soft --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_time_soft.json 2> gpurun_out/bench_time_soft.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_time_soft.json')); print(d['value'], d['ms_per_step'])"
