# r03t: decode3 store policy A/B (lib_b: plain stores) + rocprof kernel trace and HBM PMC of the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03t.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
bash tools/gpu_ab.sh data-compression_amd/lib_b/libdcamd.so || exit $?
bash tools/profile.sh r03c --steps 20 --no-extra || exit $?
python3 tools/kstats.py gpurun_out/prof_r03c/run_kernel_stats.csv | head -12
cat gpurun_out/r03c_pmc.json | head -30
