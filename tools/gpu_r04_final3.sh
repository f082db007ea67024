#!/bin/bash
# After tools/pmc_summary.py on gpu_r04_final2.sh's profiles: the B = 65536
# profile, then the linear bench lines again (their traffic entries are now
# from this build).
set -e -o pipefail
export TMPDIR=/tmp
bash tools/profile.sh linear_65536 --batch 65536 --steps 20 --warmup 2
B() { timeout -k 10 300 python bench.py "$@"; }
B --gpus 1 --steps 20 --warmup 5 > gpurun_out/f3_driver.json 2> gpurun_out/f3_driver.err
B > gpurun_out/f3_linear.json 2> gpurun_out/f3_linear.err
B --batch 8192 --no-cpu-baseline > gpurun_out/f3_linear_8192.json 2> gpurun_out/f3_linear_8192.err
B --batch 8192 --select --no-cpu-baseline > gpurun_out/f3_linear_8192_sel.json 2> gpurun_out/f3_linear_8192_sel.err
B --select --no-cpu-baseline > gpurun_out/f3_linear_sel.json 2> gpurun_out/f3_linear_sel.err
echo FINAL3DONE
