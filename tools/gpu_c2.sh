#!/bin/bash
# C2 iteration pass: standard-pattern and time parity tests, then the C2
# bench line twice (box-to-box noise is ~1 %).
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_linear_gpu.py tests/test_configs_gpu.py tests/test_time_gpu.py tests/test_cpp_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_c2.log; exit 1; }
tail -1 gpurun_out/pytest_c2.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_c2_$i.json 2> gpurun_out/bench_c2_$i.err
  python3 -c "import json; d=json.load(open('gpurun_out/bench_c2_$i.json')); print('C2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
