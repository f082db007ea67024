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
cd "$OLDPWD"
python3 - "$out" <<'PY'
import glob, sqlite3, sys
out = sys.argv[1]
db = glob.glob(f"{out}.prof/**/*.db", recursive=True)[0]
rows = sqlite3.connect(db).execute(
    "select name, count(*), avg(end-start) from regions group by name order by count(*) desc")
with open(f"{out}_hip_api.txt", "w") as f:
    f.write("HIP API calls of the latency run under rocprofv3 --hip-trace: name, count, mean ns\n")
    for n, c, a in rows:
        f.write(f"{n:32s} {c:8d} {a:14.1f}\n")
print(open(f"{out}_hip_api.txt").read())
PY
