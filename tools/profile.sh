#!/bin/bash
# Run on the GPU box (via gpurun) from the repo root:
#   bash tools/profile.sh <tag> [bench args...]
# 1) rocprofv3 --kernel-trace --stats of bench.py
# 2) separate --pmc passes for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md
#    HBM section: FETCH_SIZE and WRITE_SIZE cannot share a pass)
# Outputs under gpurun_out/prof_<tag>/.
set -e -o pipefail
TAG=${1:-linear}; shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="$@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline $ARGS > "$OUT/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline $ARGS > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline $ARGS > "$OUT/bench_write.log" 2>&1
find "$OUT" -name "*.csv" | sort > "$OUT/files.txt"
echo done
