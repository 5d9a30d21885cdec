# r03d: the token walk alone (layout x length)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03d.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 240 python3 -u tools/walk_bench2.py > gpurun_out/walk_bench2b.txt 2>&1
