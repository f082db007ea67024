#!/bin/bash
# Phase stamps of the standard linear kernel from the diagnostic build alone.
set -e -o pipefail
mkdir -p gpurun_out
MTG_LIB_PATH=mav_tube_trajectory_generation_amd/libmtg_hip_stamps.so timeout -k 10 120 python tools/stamps_std.py 1024 > gpurun_out/stamps_std.txt 2>&1
cat gpurun_out/stamps_std.txt
