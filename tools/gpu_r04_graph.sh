#!/bin/bash
# Round-4: graph chunking of the timed region at the driver's K = 20 and the
# C2 phase stamps.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us  sel', round(d['config'].get('selection_overhead_ms',0)*1e3,3))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/g_$tag.json 2> gpurun_out/g_$tag.err; line gpurun_out/g_$tag.json $tag; }
for i in 1 2; do
  run base$i
  run spin$i --sync spin
  run h1_$i --sync spin --graph-head 1
  run c5_$i --sync spin --graph-chunk 5
  run c2_$i --sync spin --graph-chunk 2
  run c1_$i --sync spin --graph-chunk 1
  run h1c4_$i --sync spin --graph-head 1 --graph-chunk 4
  run h2c6_$i --sync spin --graph-head 2 --graph-chunk 6
done
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_c2.txt 2>&1
cat gpurun_out/stamps_c2.txt
timeout -k 10 900 python -u -m pytest tests/test_linear_lane_gpu.py tests/test_extrema_candidates_gpu.py tests/test_cpp_api.py tests/test_coll_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_r04a.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r04a.log; exit 1; }
tail -2 gpurun_out/pytest_r04a.log
