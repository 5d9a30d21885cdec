# r03w: 8-chunk segments for streams below 80 MB of capacity: parity + the size sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03w.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_decode3.py tests/test_gpu_codec.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_w.log 2>&1
rc=$?
tail -n 3 gpurun_out/t_w.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_w.log | head -20; exit $rc; }
timeout -k 10 400 python3 -u bench.py --no-cpu --no-pipelined --steps 20 > gpurun_out/w_bench.json 2> gpurun_out/w_bench.err || { tail -20 gpurun_out/w_bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/w_bench.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms'])
for k,v in d['sweep'].items(): print(k, v['value'], v['ms_per_step'], v['fast_path'], v['kernels_ms'])
"
