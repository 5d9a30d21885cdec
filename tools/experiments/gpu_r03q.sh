# r03q: parity (segment decoder, codec, full size) + bench + decoder section profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03q.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode3.py tests/test_gpu_codec.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_q.log 2>&1
rc=$?
tail -n 3 gpurun_out/t_q.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { tail -20 gpurun_out/q_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/q_bench.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms'],d['phases_ms'])"
DCAMD_LIB=data-compression_amd/lib_p/libdcamd.so timeout -k 10 200 python3 -u tools/dec3_prof.py 7 26 1e-3 > gpurun_out/q_prof3.txt 2>&1 || exit $?
cat gpurun_out/q_prof3.txt
