#!/bin/bash
# Round-4 A/B of a kernel variant library against the default build at C2
# (K = 200 and K = 20), three alternations.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=${1:-mav_tube_trajectory_generation_amd/libmtg_hip_sc1.so}
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3))" "$1" "$2"; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ab_a_$i.json 2> gpurun_out/ab_a_$i.err; line gpurun_out/ab_a_$i.json base200
  MTG_LIB_PATH=$VAR timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ab_b_$i.json 2> gpurun_out/ab_b_$i.err; line gpurun_out/ab_b_$i.json var200
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_a20_$i.json 2> gpurun_out/ab_a20_$i.err; line gpurun_out/ab_a20_$i.json base20
  MTG_LIB_PATH=$VAR timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_b20_$i.json 2> gpurun_out/ab_b20_$i.err; line gpurun_out/ab_b20_$i.json var20
done
bash tools/pmc_sq.sh time --workload time --steps 3 --warmup 1 > gpurun_out/sq_time.log 2>&1 || { echo "pmc_sq time failed"; tail -5 gpurun_out/sq_time.log; }
python3 tools/sq_summary.py time time_optimize_std_kernel 4096 || true
bash tools/pmc_lds.sh time --workload time --steps 3 --warmup 1 > gpurun_out/lds_time.log 2>&1 || { echo "pmc_lds time failed"; }
for p in p3 p4; do
  f=gpurun_out/lds_time/$p/run_counter_collection.csv
  [ -f $f ] && python3 -c "
import csv,statistics
per={}
for r in csv.DictReader(open('$f')):
    if 'time_optimize_std_kernel' not in r['Kernel_Name']: continue
    per.setdefault(r['Counter_Name'],{}).setdefault(r['Dispatch_Id'],0.0)
    per[r['Counter_Name']][r['Dispatch_Id']]+=float(r['Counter_Value'])
for k,d in per.items(): print('$p',k,statistics.median(d.values()))
" || echo "no $p csv"
done
