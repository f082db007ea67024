#!/bin/bash
# Lane-pair kernel at B = 8192: where does the time go?  Variant libraries
# built with the lane-pair object compiled with -DMTG_EXP_SAME_LOAD (every
# lane loads trajectory 0's inputs: one cache line per load instruction) or
# -DMTG_EXP_NO_COEFF (no coefficient stores), against the product build.
# The two flags were a temporary patch of mtg_linear_lane2.hip at commit
# 1cdf1a5 (before the staged outputs): in Half::load, `b = 0; d = 0;` under
# MTG_EXP_SAME_LOAD; in lane2_half, `cb = nullptr;` under MTG_EXP_NO_COEFF.
# Libraries: the lane-pair object rebuilt with the flag, linked with the
# other objects of the product build into libmtg_hip_exp_<FLAG>.so.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=mav_tube_trajectory_generation_amd
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us', d['roofline'].get('kernel'))" "$1" "$2"; }
run() { local tag=$1; local lib=$2; shift 2; MTG_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/l2x_$tag.json 2> gpurun_out/l2x_$tag.err; line gpurun_out/l2x_$tag.json $tag; }
for rep in 1 2; do
  for b in 4096 8192; do
    run base_$b $P/libmtg_hip.so --batch $b --kernel lane_pair --steps 100 --warmup 10
    run same_$b $P/libmtg_hip_exp_SAME_LOAD.so --batch $b --kernel lane_pair --steps 100 --warmup 10
    run nocoef_$b $P/libmtg_hip_exp_NO_COEFF.so --batch $b --kernel lane_pair --steps 100 --warmup 10
  done
done
