#!/bin/bash
# GPU pass for the fused selection and the linear kernels, then bench lines
# per linear kernel at the config-2 (1024), config-4 shard (8192) and large
# (65536) batches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_select_gpu.py tests/test_linear_gpu.py tests/test_linear_lane_gpu.py tests/test_cpp_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_select.log 2>&1 || { echo "pytest failed"; exit 1; }
echo "pytest ok"
timeout -k 10 300 python bench.py > gpurun_out/bench_linear.json 2> gpurun_out/bench_linear.err || exit 1
for k in lane lane_pair; do
  timeout -k 10 200 python bench.py --batch 8192 --kernel $k --no-cpu-baseline > gpurun_out/bench_8192_$k.json 2> gpurun_out/bench_8192_$k.err || exit 1
  timeout -k 10 200 python bench.py --batch 65536 --kernel $k --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/bench_65536_$k.json 2> gpurun_out/bench_65536_$k.err || exit 1
done
timeout -k 10 200 python bench.py --batch 1024 --kernel lane_pair --no-cpu-baseline > gpurun_out/bench_1024_lane_pair.json 2> gpurun_out/bench_1024_lane_pair.err || exit 1
echo "bench ok"
