# r03b: instruction-sequence costs + token-walk variants (staging fixed)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03b.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 240 python3 -u tools/isa_bench2.py > gpurun_out/isa_bench2.txt 2>&1 && \
timeout -k 10 240 python3 -u tools/walk_bench.py > gpurun_out/walk_bench2.txt 2>&1
rc=$?
tail -n 2 gpurun_out/isa_bench2.txt gpurun_out/walk_bench2.txt
exit $rc
