set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tube_time_gpu.py tests/test_tube_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_tube_time.log 2>&1
