#!/bin/bash
# Linear-kernel bench lines over batch sizes and kernels (no CPU baseline).
set -e -o pipefail
mkdir -p gpurun_out/lb
for K in ${KERNELS:-standard lane_dim lane}; do
for B in ${BATCHES:-1024 4096 8192 16384 65536 262144}; do
  timeout -k 10 120 python bench.py --kernel $K --batch $B --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/lb/${K}_$B.json 2> gpurun_out/lb/${K}_$B.err
  python -c "
import json
d = json.loads(open('gpurun_out/lb/${K}_$B.json').read().strip().splitlines()[-1])
print('$K', $B, '%.1f M traj/s' % (d['value'] / 1e6), 'kernel %.2f us' % (d['roofline']['kernel_ms'] * 1e3), 'fp64 frac %.3f' % d['roofline']['frac'])
"
done
done
