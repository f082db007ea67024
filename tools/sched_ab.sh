# Scheduler-strategy A/B on the GPU box (profiles/r06_sched_ab.txt, parts 4-6):
# the time-kernel variants (libmtg_hip_time*.so from tools/build_variant.sh)
# on the C5 lines, then the product against stash/libmtg_hip_noilp.so (the
# wave kernel's object without -amdgpu-sched-strategy=max-ilp:
# build_variant.sh noilp mtg_linear_wave.hip, moved to stash/) over C2
# shapes, then the linear parity tests.
set -e -o pipefail
P=mav_tube_trajectory_generation_amd
bash tools/round_measure.sh ablation --workload time --steps 5 --warmup 2 > /dev/null
cp gpurun_out/ablation.txt gpurun_out/abl_sched_time.txt
bash tools/round_measure.sh ablation --workload time --soft --steps 3 --warmup 1 > /dev/null
cp gpurun_out/ablation.txt gpurun_out/abl_sched_time_soft.txt
rm $P/libmtg_hip_time*.so
cp stash/libmtg_hip_noilp.so $P/
i=0
for a in "--steps 200 --warmup 20" "--steps 20 --warmup 5" "--segments 3" "--segments 6" "--segments 16" "--batch 256" "--batch 2048"; do
  i=$((i+1))
  bash tools/round_measure.sh ablation $a > /dev/null
  (echo "## $a"; cat gpurun_out/ablation.txt) >> gpurun_out/abl_sched_c2.txt
done
timeout -k 10 600 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_gpu.py tests/test_select_gpu.py tests/test_graph_capture_gpu.py tests/test_configs_gpu.py -k "linear or select or capture or config2 or config1" > gpurun_out/ilp_tests.log 2>&1
