#!/bin/bash
# Wave kernel against the lane-pair kernel between 2048 and 4096 (the AUTO
# crossover).
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us', d['roofline'].get('kernel'))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/cx2_$tag.json 2> gpurun_out/cx2_$tag.err; line gpurun_out/cx2_$tag.json $tag; }
for b in 2048 2560 3072 3584 4096; do
  run std_$b --batch $b --kernel standard --steps 100 --warmup 10
  run pair_$b --batch $b --kernel lane_pair --steps 100 --warmup 10
done
