#!/bin/bash
# GPU pass for the tube QCQP: tests, the 400-problem status agreement with
# the oracle, the config-3 bench line and its kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tube_gpu.py tests/test_tube_time_gpu.py tests/test_configs_gpu.py -k "tube or config3" -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/pytest_tube.log 2>&1 || { echo "pytest failed"; tail -5 gpurun_out/pytest_tube.log; exit 1; }
tail -3 gpurun_out/pytest_tube.log
timeout -k 10 300 python tools/tube_status_agreement.py r03 > gpurun_out/tube_agreement.txt 2>&1 || exit 1
cat gpurun_out/tube_agreement.txt | tail -2
timeout -k 10 300 python bench.py --workload tube --steps 10 --warmup 2 > gpurun_out/bench_tube.json 2> gpurun_out/bench_tube.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tube -o run -- python3 bench.py --workload tube --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_tube.log 2>&1 || exit 1
echo ok
