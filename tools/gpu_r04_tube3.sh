#!/bin/bash
# Tube reductions (DPP max/min, one barrier per block reduction): outputs
# bit-identical to the previous build, tube tests, C3 A/B.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/tube_bitcmp.py gpurun_out/tube_new.npz
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so timeout -k 10 200 python tools/tube_bitcmp.py gpurun_out/tube_base.npz
python3 -c "
import numpy as np
a=np.load('gpurun_out/tube_new.npz'); b=np.load('gpurun_out/tube_base.npz')
for k in a.files:
    same = np.array_equal(a[k], b[k], equal_nan=True) if a[k].dtype.kind == 'f' else np.array_equal(a[k], b[k])
    print(k, 'bit-identical' if same else 'DIFFERENT')
"
timeout -k 10 900 python -u -m pytest tests/test_tube_gpu.py tests/test_tube_time_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_tube3.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_tube3.log; exit 1; }
tail -1 gpurun_out/pytest_tube3.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel', round(d['roofline']['kernel_ms'],4), 'ms')" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/t3_$tag.json 2> gpurun_out/t3_$tag.err; line gpurun_out/t3_$tag.json $tag; }
for i in 1 2; do
  MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_base.so run base_$i --workload tube --steps 10 --warmup 2
  run new_$i --workload tube --steps 10 --warmup 2
done
