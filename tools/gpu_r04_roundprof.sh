#!/bin/bash
# Round-4 profile pass (two gpurun calls from the repo root: `traffic`, `sq`): FETCH/WRITE calibration
# of the access widths, kernel stats + separate FETCH_SIZE / WRITE_SIZE
# passes per bench workload (tools/profile.sh), SQ counters per workload
# (tools/pmc_sq.sh).  Summaries: tools/pmc_summary.py, tools/sq_summary.py.
set -e -o pipefail
mkdir -p gpurun_out/calib
export TMPDIR=/tmp
ROOT=$(pwd)
if [ "${1:-traffic}" = traffic ]; then
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/calib/fetch -o run -- $ROOT/tools/ubench/fetch_calib > gpurun_out/calib/fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/gpurun_out/calib/write -o run -- $ROOT/tools/ubench/fetch_calib > gpurun_out/calib/write.log 2>&1
echo calib done
bash tools/profile.sh linear --steps 50 --warmup 5
bash tools/profile.sh linear_8192 --batch 8192 --steps 50 --warmup 5
bash tools/profile.sh linear_65536 --batch 65536 --steps 20 --warmup 2
bash tools/profile.sh tube --workload tube --steps 5 --warmup 1
bash tools/profile.sh time --workload time --steps 5 --warmup 1
bash tools/profile.sh time_soft --workload time --soft --steps 3 --warmup 1
echo traffic done
else
bash tools/pmc_sq.sh linear --steps 50 --warmup 5
bash tools/pmc_sq.sh linear_8192 --batch 8192 --steps 50 --warmup 5
bash tools/pmc_sq.sh tube --workload tube --steps 5 --warmup 1
bash tools/pmc_sq.sh time_soft --workload time --soft --steps 3 --warmup 1
fi
echo ALLDONE
