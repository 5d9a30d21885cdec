set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode_runs.py tests/test_gpu_codec.py -m gpu -x -q -k "runs or halo" --timeout 120 --timeout-method thread > gpurun_out/rp_t.log 2>&1 || { tail -30 gpurun_out/rp_t.log; exit 1; }
tail -1 gpurun_out/rp_t.log
DCAMD_LIB=data-compression_amd/lib_rp/libdcamd.so timeout -k 10 120 python3 -u tools/runs_prof.py || exit 1
timeout -k 10 200 python3 -u bench.py --halo --steps 50 > gpurun_out/halo.json 2> gpurun_out/halo.err || { tail -20 gpurun_out/halo.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/halo.json').readline());print('halo',d['value'],d['ms_per_step'])"
