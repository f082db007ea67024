# Round-6 closing measurements of the kernels changed late in the round
# (C2 max-ILP object, tube IPM scaled start): bench lines with their CPU
# baselines, rocprofv3 kernel stats + HBM PMC passes, SQ passes.
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B() { timeout -k 10 300 python bench.py "$@"; }
B > gpurun_out/bench_linear.json 2> gpurun_out/bench_linear.err
B --workload tube --steps 20 --warmup 3 > gpurun_out/bench_tube.json 2> gpurun_out/bench_tube.err
B --workload time-qcqp --steps 5 --warmup 1 > gpurun_out/bench_time_qcqp.json 2> gpurun_out/bench_time_qcqp.err
B --workload time-qcqp --optimizer sbplx --steps 3 --warmup 1 > gpurun_out/bench_time_qcqp_sbplx.json 2> gpurun_out/bench_time_qcqp_sbplx.err
bash tools/profile.sh linear
bash tools/profile.sh tube --workload tube --steps 5 --warmup 1
bash tools/profile.sh time_qcqp_sbplx --workload time-qcqp --optimizer sbplx --steps 2 --warmup 1
bash tools/pmc_sq.sh linear
bash tools/pmc_sq.sh tube --workload tube --steps 5 --warmup 1
