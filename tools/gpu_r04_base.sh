#!/bin/bash
# Round-4 baseline: the driver's C2 command (K = 20, W = 5) three times with
# the runtime's default host wait and three times with spin, K = 200 once,
# and the C2 phase stamps (diagnostic build, built beforehand in-tree).
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3), 'us  sel', round(d['config'].get('selection_overhead_ms',0)*1e3,3))" "$1" "$2"; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_auto_$i.json 2> gpurun_out/b_auto_$i.err
  line gpurun_out/b_auto_$i.json auto20
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sync spin > gpurun_out/b_spin_$i.json 2> gpurun_out/b_spin_$i.err
  line gpurun_out/b_spin_$i.json spin20
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/b_200.json 2> gpurun_out/b_200.err
line gpurun_out/b_200.json auto200
if [ -f mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so ]; then
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_c2.txt 2>&1
  cat gpurun_out/stamps_c2.txt
fi
timeout -k 10 900 python -u -m pytest tests/test_linear_lane_gpu.py tests/test_extrema_candidates_gpu.py tests/test_cpp_api.py tests/test_coll_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_r04a.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r04a.log; exit 1; }
tail -2 gpurun_out/pytest_r04a.log
