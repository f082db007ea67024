#!/bin/bash
# GPU pass for the collision objectives (tests, C++ demo test) and the
# collision bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_coll_gpu.py tests/test_collision_gpu.py tests/test_cpp_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_coll.log 2>&1 || { echo "pytest failed"; tail -5 gpurun_out/pytest_coll.log; exit 1; }
tail -2 gpurun_out/pytest_coll.log
timeout -k 10 300 python bench.py --workload collision --steps 5 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_collision.json 2> gpurun_out/bench_collision.err || exit 1
echo ok
