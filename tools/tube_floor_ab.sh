set -e -o pipefail
P=mav_tube_trajectory_generation_amd
mkdir -p gpurun_out/floor
for lib in $P/libmtg_hip.so $P/libmtg_hip_fl*.so; do
  v=$(basename $lib .so)
  MTG_LIB_PATH=$lib timeout -k 10 300 python tools/tube_floor_ab.py $v >> gpurun_out/floor/hist.txt 2>&1
done
bash tools/round_measure.sh ablation --workload tube --steps 20 --warmup 3 > /dev/null
cp gpurun_out/ablation.txt gpurun_out/floor/ablation.txt
