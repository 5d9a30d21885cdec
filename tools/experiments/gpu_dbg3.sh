set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_dbg3.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
DC_DEBUG_ERR=1 timeout -k 10 120 python3 -u tools/dbg_dec3.py 1e-6 u10_16k 7 > gpurun_out/dbg3.txt 2>&1
DC_DEBUG_ERR=1 timeout -k 10 120 python3 -u tools/dbg_dec3.py 1e-6 rand16k 7 >> gpurun_out/dbg3.txt 2>&1
DC_DEBUG_ERR=1 timeout -k 10 120 python3 -u tools/dbg_dec3.py 1e-3 u10_16k 7 >> gpurun_out/dbg3.txt 2>&1
cat gpurun_out/dbg3.txt
