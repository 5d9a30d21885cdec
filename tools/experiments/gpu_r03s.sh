# r03s: zero-run fast path of the segment decoder: parity + config 3 in the bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03s.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode3.py tests/test_gpu_codec.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_s.log 2>&1
rc=$?
tail -n 3 gpurun_out/t_s.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_s.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u bench.py --no-cpu --no-pipelined --no-extra --ct 7 --input eq --log2n 28 --steps 8 > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err || { tail -20 gpurun_out/s_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/s_bench.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms'])"
