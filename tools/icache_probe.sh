set -o pipefail
mkdir -p gpurun_out/icache
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/icache/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_INSTS_[A-Z_0-9]*" gpurun_out/icache/avail.txt | sort -u | tr '\n' ' '
echo
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES --output-format csv -d gpurun_out/icache/p1 -o run -- python3 bench.py --workload time --soft --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/icache/p1.log 2>&1
echo rc=$?
