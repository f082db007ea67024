#!/bin/bash
# C5 + soft with the soft optimiser forced to three waves per SIMD
# (libmtg_hip_w3.so, amdgpu_waves_per_eu(3), 168 VGPRs + 320 B scratch)
# against the default build (250 VGPRs, two waves), alternating; then the
# C2 LDS counters.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms'],3), 'ms')" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/w3_$tag.json 2> gpurun_out/w3_$tag.err; line gpurun_out/w3_$tag.json $tag; }
for i in 1 2; do
  run base_$i --workload time --soft --steps 3 --warmup 1
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_w3.so run w3_$i --workload time --soft --steps 3 --warmup 1
done
bash tools/pmc_lds.sh c2 --steps 50 --warmup 5
