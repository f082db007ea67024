#!/bin/bash
# Compile-time-S tube kernel: the tube parity tests (incl. config 3 at size
# and the tube time objective), then C3 against the runtime-S kernel
# (MTG_TUBE_RUNTIME_S=1), alternating.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tube_gpu.py tests/test_tube_time_gpu.py tests/test_configs_gpu.py tests/test_cpp_api.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_tube.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_tube.log; exit 1; }
tail -1 gpurun_out/pytest_tube.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], round(d['value']/1e3,2), 'k/s  kernel', round(d['roofline']['kernel_ms'],4), 'ms', d['roofline'].get('kernel'), c.get('converged_per_step'))" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/tb_$tag.json 2> gpurun_out/tb_$tag.err; line gpurun_out/tb_$tag.json $tag; }
for i in 1 2; do
  run s_$i --workload tube --steps 10 --warmup 2
  MTG_TUBE_RUNTIME_S=1 run rt_$i --workload tube --steps 10 --warmup 2
done
run qcqp --workload time-qcqp --steps 5 --warmup 1
