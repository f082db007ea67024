#!/bin/bash
# LDS / memory-pipe counters of one bench workload (run via gpurun from the
# repo root): bash tools/pmc_lds.sh <tag> [bench args...].  One --pmc pass
# per block group (SQ <= 8, TA <= 2, TCP <= 4 per pass).
set -e -o pipefail
TAG=${1:-linear}; shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/lds_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d "$OUT/p3" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/p3.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum --output-format csv -d "$OUT/p4" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/p4.log" 2>&1
echo done
