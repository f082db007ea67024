# GPU check of an IPM change (tube): tube / tube-time / SBPLX-QCQP / config-3
# tests, the 400-seed status agreement, and the C3, time-qcqp (FD) and
# time-qcqp (LN_SBPLX) bench lines.  Outputs under gpurun_out/ipm/.
set -e -o pipefail
mkdir -p gpurun_out/ipm
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_tube_gpu.py tests/test_tube_time_gpu.py tests/test_tube_time_sbplx_gpu.py \
  tests/test_configs_gpu.py tests/test_cpp_api.py -k "tube or config3 or cpp" > gpurun_out/ipm/tests.log 2>&1
timeout -k 10 300 python tools/tube_status_agreement.py ipm > gpurun_out/ipm/agreement.txt 2>&1
timeout -k 10 300 python bench.py --workload tube --steps 20 --warmup 3 > gpurun_out/ipm/bench_tube.json 2> gpurun_out/ipm/bench_tube.err
timeout -k 10 300 python bench.py --workload time-qcqp --steps 5 --warmup 2 > gpurun_out/ipm/bench_time_qcqp.json 2> gpurun_out/ipm/bench_time_qcqp.err
timeout -k 10 600 python bench.py --workload time-qcqp --optimizer sbplx --steps 3 --warmup 1 > gpurun_out/ipm/bench_time_qcqp_sbplx.json 2> gpurun_out/ipm/bench_time_qcqp_sbplx.err
