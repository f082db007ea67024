#!/bin/bash
# Round-3 SQ instruction-mix passes for the bench workloads (executed FP64
# work per trajectory, profiles/sq_executed.json) + the linear golden tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_linear_gpu.py -k golden -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_golden.log 2>&1 || { echo "golden failed"; tail -5 gpurun_out/pytest_golden.log; exit 1; }
tail -1 gpurun_out/pytest_golden.log
bash tools/pmc_sq.sh r03_linear --steps 20 --warmup 3 || exit 1
bash tools/pmc_sq.sh r03_lane2_8192 --batch 8192 --steps 20 --warmup 3 || exit 1
bash tools/pmc_sq.sh r03_lane2_65536 --batch 65536 --steps 10 --warmup 2 || exit 1
bash tools/pmc_sq.sh r03_time --workload time --steps 3 --warmup 1 || exit 1
bash tools/pmc_sq.sh r03_time_soft --workload time --soft --steps 2 --warmup 1 || exit 1
bash tools/pmc_sq.sh r03_tube --workload tube --steps 2 --warmup 1 || exit 1
echo ok
