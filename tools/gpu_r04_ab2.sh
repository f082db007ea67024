#!/bin/bash
# A/B of the wave kernel against libmtg_hip_base.so (the previous build),
# alternating, K = 200 and the driver's K = 20; then the phase stamps.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us  step', round(d['ms_per_step']*1e3,3))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err; line gpurun_out/ab_$tag.json $tag; }
for i in 1 2 3; do
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base200_$i --steps 200 --warmup 20
  run new200_$i --steps 200 --warmup 20
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base20_$i --steps 20 --warmup 5
  run new20_$i --steps 20 --warmup 5
done
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so STAMPS_SYM=wave timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_wave.txt 2>&1
cat gpurun_out/stamps_wave.txt
