#!/bin/bash
# Round-4 C2 wave kernel: batch sweep (waves per CU), SQ and LDS counters.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3))" "$1" "$2"; }
for B in 128 256 512 768 1024 2048; do
  timeout -k 10 300 python bench.py --batch $B --kernel standard --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/sw_$B.json 2> gpurun_out/sw_$B.err; line gpurun_out/sw_$B.json B$B
done
bash tools/pmc_sq.sh wave --steps 50 --warmup 5 > gpurun_out/sq_wave.log 2>&1 || { echo "pmc_sq failed"; tail -5 gpurun_out/sq_wave.log; }
python3 tools/sq_summary.py wave linear_wave_kernel 1024 || true
bash tools/pmc_lds.sh wave --steps 50 --warmup 5 > gpurun_out/lds_wave.log 2>&1 || { echo "pmc_lds failed"; tail -5 gpurun_out/lds_wave.log; }
for p in p3 p4; do
  f=gpurun_out/lds_wave/$p/run_counter_collection.csv
  [ -f $f ] && python3 -c "
import csv,statistics,sys
per={}
for r in csv.DictReader(open('$f')):
    if 'linear_wave_kernel' not in r['Kernel_Name']: continue
    per.setdefault(r['Counter_Name'],{}).setdefault(r['Dispatch_Id'],0.0)
    per[r['Counter_Name']][r['Dispatch_Id']]+=float(r['Counter_Value'])
for k,d in per.items(): print('$p',k,statistics.median(d.values()))
" || echo "no $p csv"; tail -3 gpurun_out/lds_wave/$p.log || true
done
