# r03c: token-walk variants (one atomic per wave)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03c.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 240 python3 -u tools/walk_bench.py > gpurun_out/walk_bench3.txt 2>&1
