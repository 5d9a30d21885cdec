# r03f: segment decoder parity + quick bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03f.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
DC_DEBUG_ERR=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_decode3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dec3.log 2>&1
rc=$?
tail -n 30 gpurun_out/t_dec3.log
[ $rc -eq 0 ] || exit $rc
DC_DEBUG_ERR=1 timeout -k 10 300 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/bench_r03f.json 2> gpurun_out/bench_r03f.err
rc=$?
tail -n 3 gpurun_out/bench_r03f.err
exit $rc
