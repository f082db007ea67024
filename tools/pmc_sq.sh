#!/bin/bash
# SQ instruction-mix / lane-utilisation counters for one bench workload (run
# via gpurun from the repo root):  bash tools/pmc_sq.sh <tag> [bench args...]
# Two --pmc passes of <= 8 SQ counters each (MI355X_MICROARCH.md: SQ block
# has 8 slots per pass), plus the kernel-trace stats.
set -e -o pipefail
TAG=${1:-linear}; shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d "$OUT/p1" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/p1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM --output-format csv -d "$OUT/p2" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/p2.log" 2>&1
echo done
