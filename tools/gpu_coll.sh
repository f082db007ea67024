#!/bin/bash
# Focused GPU pass for the collision objectives and the kernels they touch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_coll_gpu.py tests/test_collision_gpu.py tests/test_cpp_api.py tests/test_time_gpu.py tests/test_extrema_gpu.py tests/test_tube_time_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_coll.log 2>&1
echo "pytest rc=$?"
