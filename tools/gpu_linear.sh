set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_linear_gpu.py tests/test_time_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_linear.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_std.json 2> gpurun_out/bench_std.err
timeout -k 10 300 python bench.py --workload time --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_std.txt 2>&1
echo ALLDONE
