#!/bin/bash
# GPU pass for the magnitude-extrema paths (candidate lists, maxima, the C++
# API's ExtremaOfMagnitude port).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_extrema_candidates_gpu.py tests/test_extrema_gpu.py tests/test_cpp_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_extrema.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_extrema.log
exit $rc
