# r03p: debug the segment decoder's decline on u10 100003
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03p.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 120 python3 -u tools/dbg_o.py 2>&1 | tee gpurun_out/p_dbg.log
