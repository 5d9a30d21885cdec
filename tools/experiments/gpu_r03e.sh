# r03e: token walk latency hiding (waves per SIMD x chains per lane)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03e.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 240 python3 -u tools/walk_bench3.py > gpurun_out/walk_bench3b.txt 2>&1
