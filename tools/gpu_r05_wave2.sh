#!/bin/bash
# Round 5: the two-wave C2 kernel (MTG_WAVE2=1) against the one-wave kernel:
# the linear parity tests under MTG_WAVE2=1, then alternating A/B bench
# lines (kernel_ms) at K = 200 and the driver's K = 20.
set -e -o pipefail
mkdir -p gpurun_out/w2
export TMPDIR=/tmp
MTG_WAVE2=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_linear_gpu.py tests/test_configs_gpu.py -k "linear or config2 or golden or exact or fixture or segment or orders or pattern" \
  > gpurun_out/w2/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/w2/tests.log; exit 1; }
tail -2 gpurun_out/w2/tests.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us  step', round(d['ms_per_step']*1e3,3), 'us')" "$1" "$2"; }
run() { local tag=$1; local w=$2; shift 2; MTG_WAVE2=$w timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/w2/$tag.json 2> gpurun_out/w2/$tag.err; line gpurun_out/w2/$tag.json $tag; }
for rep in 1 2 3; do
  run one200_$rep 0 --steps 200 --warmup 20
  run two200_$rep 1 --steps 200 --warmup 20
  run one20_$rep 0 --steps 20 --warmup 5
  run two20_$rep 1 --steps 20 --warmup 5
done
for b in 512 2048; do
  run one_b$b 0 --batch $b --kernel standard --steps 200 --warmup 20
  run two_b$b 1 --batch $b --kernel standard --steps 200 --warmup 20
done
