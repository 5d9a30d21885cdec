# r03o: count kernel group scans + pack offsets (no encode scan launch); parse3 waits for the link into
# its job and its last wave checks the rest, decode3 sums the parse totals (no scan3 launch)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03o.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode3.py tests/test_gpu_codec.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_o.log 2>&1
rc=$?
tail -n 15 gpurun_out/t_o.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/o_bench.json 2> gpurun_out/o_bench.err || { tail -20 gpurun_out/o_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/o_bench.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms'],d['phases_ms'])"
