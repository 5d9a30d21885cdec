# round 5 evidence run: slow-sync timings (maps parse), the fused-decoder occupancy experiment, then the
# full bench line and the multi-rank rehearsals (tools/gpu_run.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out/r05c_slow_sync.txt; : > $O
for a in "7 ramp 1e-3" "7 sine 1e-5" "11 normal 1e-3" "5 ramp 1e-3" "7 u10 1e-3"; do
  set -- $a
  timeout -k 10 120 python3 -u tools/seg_time.py 24 $1 16 $3 $2 >> $O 2>&1 || { tail -20 $O; exit 1; }
done
cat $O
timeout -k 10 400 python3 -u tools/experiments/fusion_occupancy.py > gpurun_out/r05c_fusion_occupancy.txt 2>&1 || { tail -20 gpurun_out/r05c_fusion_occupancy.txt; exit 1; }
tail -15 gpurun_out/r05c_fusion_occupancy.txt
bash tools/gpu_run.sh r05c bench gloo2 gloo3
