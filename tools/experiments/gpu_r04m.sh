# round-4: small-stream decoder (scan + values kernels): tests, --halo, 2^14/2^16; parse walk two steps per
# round (lib_w2) A/B; halo kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_decode_runs.py tests/test_gpu_codec.py tests/test_gpu_decode3.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m_t.log 2>&1 || { tail -40 gpurun_out/r04m_t.log; exit 1; }
tail -1 gpurun_out/r04m_t.log
timeout -k 10 200 python3 -u bench.py --halo --steps 50 > gpurun_out/halo.json 2> gpurun_out/halo.err || { tail -20 gpurun_out/halo.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/halo.json').readline());print('halo',d['value'],d['ms_per_step'],d['config']['stream_bytes'])"
run() {
  DCAMD_LIB=data-compression_amd/$1/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 $2 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(*sys.argv[1:],d['value'],d['ms_per_step'],d['kernels_ms'])" $1 "$2"
}
run lib "--log2n 12 --steps 50" && run lib "--log2n 14 --steps 50" || exit 1
for i in 1 2; do run lib && run lib_w2 && run lib_f7 || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_halo -o run -- python3 bench.py --halo --steps 20 > gpurun_out/prof_halo.log 2>&1 || { tail -20 gpurun_out/prof_halo.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof_halo/run_kernel_stats.csv | head -12
