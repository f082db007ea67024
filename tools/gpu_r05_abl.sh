#!/bin/bash
# Round 5: where does the C2 kernel's time go?  Ablation variants of
# mtg_linear_wave.hip (tools/build_variant.sh; flags MTG_ABL_* in
# mtg_wave_device.h / mtg_linear_wave.hip: results are wrong, only the launch
# time is read), alternated with the product build, K = 200, kernel_ms.
set -e -o pipefail
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
P=mav_tube_trajectory_generation_amd
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us')" "$1" "$2"; }
run() { local tag=$1; local lib=$2; shift 2; MTG_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/abl/$tag.json 2> gpurun_out/abl/$tag.err; line gpurun_out/abl/$tag.json $tag; }
for rep in 1 2 3; do
  for v in base noend noc nob noasm nocoef; do
    lib=$P/libmtg_hip_$v.so; [ $v = base ] && lib=$P/libmtg_hip.so
    run ${v}_$rep $lib --steps 200 --warmup 20
  done
done
run sel8192 $P/libmtg_hip.so --batch 8192 --select --steps 20 --warmup 5
run plain8192 $P/libmtg_hip.so --batch 8192 --steps 20 --warmup 5
