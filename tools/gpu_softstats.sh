#!/bin/bash
# Per-lane search statistics of the soft time objective (diagnostic build).
set -e -o pipefail
mkdir -p gpurun_out
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 180 python tools/soft_search_stats.py 4 > gpurun_out/soft_stats.txt 2>&1
cat gpurun_out/soft_stats.txt
