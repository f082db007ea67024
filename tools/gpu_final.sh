#!/bin/bash
# End-of-round GPU pass: every -m gpu test, smoke, the default bench line,
# then the C2 kernel's rocprofv3 stats and SQ counters.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh
tail -1 gpurun_out/pytest_gpu.log
tail -1 gpurun_out/smoke.log
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('C2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
bash tools/pmc_sq.sh linear --steps 200 --warmup 20 > gpurun_out/sq_linear.log 2>&1
find gpurun_out/sq_linear -name "*.csv" | sort
