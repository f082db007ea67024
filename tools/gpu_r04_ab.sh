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
