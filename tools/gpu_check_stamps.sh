#!/bin/bash
# gpu_check.sh plus the phase stamps of the standard-pattern linear kernel.
set -e -o pipefail
mkdir -p gpurun_out
bash tools/gpu_check.sh
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_std.txt 2>&1
echo STAMPSDONE
