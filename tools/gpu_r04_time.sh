#!/bin/bash
# Round-4 compile-time-S solver in the time kernels: their parity tests, the
# linear tests, then C5 (and C5 + soft) against the runtime-S kernels
# (MTG_STD_RUNTIME_S=1), C2, and the sc1-store A/B if its library exists.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_time_gpu.py tests/test_linear_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_time.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_time.log; exit 1; }
tail -1 gpurun_out/pytest_time.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,4), 'M/s  step', round(d['ms_per_step']*1e3,3), 'us  kernel', round(d['roofline']['kernel_ms']*1e3,3), 'kernel', d['roofline'].get('kernel'))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/tm_$tag.json 2> gpurun_out/tm_$tag.err; line gpurun_out/tm_$tag.json $tag; }
run c5_new --workload time --steps 5 --warmup 1
MTG_STD_RUNTIME_S=1 run c5_old --workload time --steps 5 --warmup 1
run c5soft_new --workload time --soft --steps 3 --warmup 1
MTG_STD_RUNTIME_S=1 run c5soft_old --workload time --soft --steps 3 --warmup 1
run c2 --steps 200 --warmup 20
run c2k20 --gpus 1 --steps 20 --warmup 5
if [ -f mav_tube_trajectory_generation_amd/libmtg_hip_sc1.so ]; then
  for i in 1 2; do
    MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_sc1.so run c2sc1_$i --steps 200 --warmup 20
    run c2base_$i --steps 200 --warmup 20
  done
fi
