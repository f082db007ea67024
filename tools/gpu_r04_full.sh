#!/bin/bash
# Full GPU suite + smoke + the driver's bench command on the current build.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_full.log; exit 1; }
tail -3 gpurun_out/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/full_bench.json 2> gpurun_out/full_bench.err
cat gpurun_out/full_bench.json
