#!/bin/bash
# Latency of the drop-in single-trajectory call PolynomialOptimization<10>::
# solveLinear() (tests/cpp "latency" group), and a rocprofv3 HIP API trace of
# the same run (no hipMalloc / hipHostMalloc per call in steady state).
#   tools/single_latency.sh OUT_PREFIX        (on the GPU box, from the repo root)
set -euo pipefail
out=${1:-gpurun_out/single}
mkdir -p "$(dirname "$out")"
bin=/tmp/mtg_cpp_latency
g++ -std=c++17 -O2 -Wall -Wextra -Werror -D__HIP_PLATFORM_AMD__ -Iinclude -Ioracle \
  -I/opt/rocm/include tests/cpp/test_polynomial_optimization.cpp -o $bin \
  -Lmav_tube_trajectory_generation_amd -lmtg_hip -Loracle -loracle -L/opt/rocm/lib -lamdhip64 \
  -Wl,-rpath,$PWD/mav_tube_trajectory_generation_amd:$PWD/oracle:/opt/rocm/lib
timeout -k 10 120 $bin latency > "$out.txt" 2>&1
grep LATENCY "$out.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-trace --stats -d "$OLDPWD/$out.prof" -o run -- $bin latency \
  > "$OLDPWD/$out.prof.log" 2>&1
