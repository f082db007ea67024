#!/bin/bash
# Diagnostic variant library: one object of the product build recompiled with
# extra flags and linked with the other product objects into
# mav_tube_trajectory_generation_amd/libmtg_hip_<tag>.so (load it with
# MTG_LIB_PATH=...).  Never shipped; the flags are ablations/experiments.
#   bash tools/build_variant.sh <tag> <source.hip> <flags...>
set -e -o pipefail
tag=$1; src=$2; shift 2
C=mav_tube_trajectory_generation_amd/csrc
obj=/tmp/variant_${tag}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$(pwd)/include \
  -munsafe-fp-atomics -mllvm -amdgpu-kernarg-preload-count=16 "$@" -c $C/$src -o $obj
objs=""
for o in $C/*.o; do [ "$(basename $o .o)" = "$(basename $src .hip)" ] || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o mav_tube_trajectory_generation_amd/libmtg_hip_${tag}.so $obj $objs
echo built libmtg_hip_${tag}.so
