set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_linear.json 2> gpurun_out/bench_linear.err
timeout -k 10 300 python bench.py --workload time --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_time.json 2> gpurun_out/bench_time.err
timeout -k 10 300 python bench.py --workload tube --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_tube.json 2> gpurun_out/bench_tube.err
bash tools/profile.sh linear
bash tools/profile.sh time --workload time --steps 5 --warmup 1
bash tools/profile.sh tube --workload tube --steps 5 --warmup 1
timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep_linear.jsonl 2>&1
echo ALLDONE
