# Whole measurement pass of a round (run on the GPU box via gpurun from the
# repo root): default bench (with the CPU baseline), the other workloads,
# rocprofv3 kernel-trace + PMC passes per workload, the batch sweep.
# Then, in the container: tools/pmc_summary.py per tag.
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_linear.json 2> gpurun_out/bench_linear.err
timeout -k 10 300 python bench.py --workload time --steps 20 --warmup 3 > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
timeout -k 10 300 python bench.py --workload time --soft --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_time_soft.json 2> gpurun_out/bench_time_soft.err
timeout -k 10 300 python bench.py --workload tube --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_tube.json 2> gpurun_out/bench_tube.err
timeout -k 10 300 python bench.py --workload time-qcqp --steps 5 --warmup 1 > gpurun_out/bench_time_qcqp.json 2> gpurun_out/bench_time_qcqp.err
bash tools/profile.sh linear
bash tools/profile.sh time --workload time --steps 5 --warmup 1
bash tools/profile.sh tube --workload tube --steps 5 --warmup 1
timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep_linear.jsonl 2>&1
echo ALLDONE
