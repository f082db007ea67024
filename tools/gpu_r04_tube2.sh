#!/bin/bash
# Tube kernel (compile-time S, XCD-aware problem index): tube tests, C3 bench
# line, kernel stats + HBM PMC passes, SQ counters.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tube_gpu.py tests/test_tube_time_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_tube2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_tube2.log; exit 1; }
tail -1 gpurun_out/pytest_tube2.log
timeout -k 10 300 python bench.py --workload tube --steps 20 --warmup 3 > gpurun_out/bench_tube.json 2> gpurun_out/bench_tube.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_tube.json')); print('tube', d['value'], d['roofline']['kernel_ms'])"
bash tools/profile.sh tube --workload tube --steps 5 --warmup 1
bash tools/pmc_sq.sh tube --workload tube --steps 5 --warmup 1
