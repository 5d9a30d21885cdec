set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_dbg3b.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
DC_DEC3_DEBUG=1 DC_DEBUG_ERR=1 timeout -k 10 100 python3 -u -m pytest tests/test_gpu_decode3.py -x -v -k golden --timeout 30 --timeout-method thread > gpurun_out/t_dec3b.log 2>&1
grep -E "PASS|FAIL|stuck|finished|declined|Timeout|ctr|job|rec0" gpurun_out/t_dec3b.log | head -60
