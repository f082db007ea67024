set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_free_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_free.log 2>&1
echo ALLDONE
