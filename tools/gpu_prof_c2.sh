#!/bin/bash
# rocprofv3 kernel stats of the default C2 bench command and its SQ counters.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_sq.sh linear --steps 200 --warmup 20 > gpurun_out/sq_linear.log 2>&1
sed -n 2p gpurun_out/sq_linear/trace/run_kernel_stats.csv | cut -c1-200
