#!/bin/bash
# Builds tools/stale_j_probe (CPU container or GPU box) against the in-tree
# libmtg_hip.so.  Run: tools/stale_j_probe.sh build && tools/stale_j_probe [reps]
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
PKG="$REPO/mav_tube_trajectory_generation_amd"
g++ -std=c++17 -O2 -Wall -D__HIP_PLATFORM_AMD__ -I"$REPO/include" -I/opt/rocm/include \
  "$REPO/tools/stale_j_probe.cpp" -o "$REPO/tools/stale_j_probe" -L"$PKG" -lmtg_hip \
  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,"$PKG:/opt/rocm/lib"
