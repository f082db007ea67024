#!/bin/bash
# Round-4 selection step (DPP select_reduce_kernel): the selection tests, then
# C2 (K = 200 and the driver's K = 20) and B = 8192 with selection_overhead,
# and the kernel stats of a C2 run.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_select_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_select.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_select.log; exit 1; }
tail -1 gpurun_out/pytest_select.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], round(d['value']/1e6,3), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us  sel', round(c.get('selection_overhead_ms',0)*1e3,3), d['roofline'].get('kernel'))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/sl_$tag.json 2> gpurun_out/sl_$tag.err; line gpurun_out/sl_$tag.json $tag; }
run c2k200 --steps 200 --warmup 20
run c2k20 --steps 20 --warmup 5
run b8192 --batch 8192 --steps 200 --warmup 20
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_sel -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_sel.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/prof_sel -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $GRAFT_REPO_ROOT/gpurun_out/sel_kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/sel_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'])
"
