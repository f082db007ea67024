#!/bin/bash
# Final measurement pass on the staged-output build: GPU suite, smoke, the
# driver's bench command, every bench line, kernel stats + HBM PMC for C2 and
# B = 8192.
set -e -o pipefail
bash tools/gpu_r04_full.sh
bash tools/round_measure.sh benches
bash tools/profile.sh linear
bash tools/profile.sh linear_8192 --batch 8192
echo FINAL2DONE
