#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/launch_floor > gpurun_out/launch_floor.txt 2>&1
cat gpurun_out/launch_floor.txt
