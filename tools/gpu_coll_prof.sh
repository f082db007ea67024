#!/bin/bash
# Kernel statistics of the collision bench (rocprofv3 --kernel-trace --stats).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_coll -o run -- python3 bench.py --workload collision --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_coll.log 2>&1 || { tail -5 gpurun_out/prof_coll.log; exit 1; }
find gpurun_out/prof_coll -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/coll_kernel_stats.csv
head -8 gpurun_out/coll_kernel_stats.csv
