#!/bin/bash
# GPU: the stale-J probe (tools/stale_j_probe.cpp), then the tube-time tests
# and the C++ API suite.  Run via gpurun from the repo root.
set -e -o pipefail
mkdir -p gpurun_out
tools/stale_j_probe.sh
timeout -k 10 240 tools/stale_j_probe 30 > gpurun_out/stale_j_probe.txt 2>&1 || echo "probe exit $?" >> gpurun_out/stale_j_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_tube_time_gpu.py tests/test_cpp_api.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_tube_time.txt 2>&1
echo ALLDONE
