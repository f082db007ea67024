set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cpp_api.py tests/test_tube_time_gpu.py -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_cpp.log 2>&1
