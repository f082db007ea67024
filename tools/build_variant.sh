#!/bin/bash
# Diagnostic variant library: one object of the product build recompiled
# (from the in-tree source, or from a copy given by path, e.g. a previous
# round's source extracted with git show) with extra flags, linked with the
# other product objects into mav_tube_trajectory_generation_amd/
# libmtg_hip_<tag>.so (load it with MTG_LIB_PATH=...).  Never shipped.
#   bash tools/build_variant.sh <tag> <source.hip | /path/to/source.hip> <flags...>
set -e -o pipefail
tag=$1; src=$2; shift 2
C=mav_tube_trajectory_generation_amd/csrc
case "$src" in /*) path=$src ;; *) path=$C/$src ;; esac
base=$(basename $src .hip)
extra=""
[ "$base" = mtg_tube ] || [ "$base" = mtg_time_std ] && extra="-mllvm -disable-machine-licm"
obj=/tmp/variant_${tag}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I$(pwd)/$C -I$(pwd)/include \
  -munsafe-fp-atomics -mllvm -amdgpu-kernarg-preload-count=16 $extra "$@" -c $path -o $obj
objs=""
for o in $C/*.o; do [ "$(basename $o .o)" = "$base" ] || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o mav_tube_trajectory_generation_amd/libmtg_hip_${tag}.so $obj $objs
echo built libmtg_hip_${tag}.so
