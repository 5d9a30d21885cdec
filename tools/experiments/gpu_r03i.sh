# r03i: codec parity (single-pass encoder) + segment decoder + quick bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03i.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_decode3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r03i.log 2>&1
rc=$?
tail -n 30 gpurun_out/t_r03i.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/bench_r03i.json 2> gpurun_out/bench_r03i.err
rc=$?
tail -n 3 gpurun_out/bench_r03i.err
python3 -c "import json;d=json.loads(open('gpurun_out/bench_r03i.json').readline());print(d['value'],d['kernels_ms'])"
exit $rc
