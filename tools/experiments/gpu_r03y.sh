# r03y: rocprof kernel trace + FETCH/WRITE PMC of the final round-3 code
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03y.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
bash tools/profile.sh r03e --steps 20 --no-extra || exit $?
python3 tools/kstats.py gpurun_out/prof_r03e/run_kernel_stats.csv | head -8
