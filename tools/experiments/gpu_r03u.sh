# r03u: the sharded encode -> gather -> decode path with two gloo ranks on the one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03u.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_u.log 2>&1
rc=$?
tail -n 15 gpurun_out/t_u.log
exit $rc
