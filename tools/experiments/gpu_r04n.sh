# round-4: parse exits published after the main walk (lib, 8/16-chunk segments) vs after in-job repairs (lib_xl)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode3.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_t.log 2>&1 || { tail -30 gpurun_out/r04n_t.log; exit 1; }
tail -1 gpurun_out/r04n_t.log
run() {
  DCAMD_LIB=data-compression_amd/$1/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 $2 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(*sys.argv[1:],d['value'],d['ms_per_step'],d['kernels_ms'])" $1 "$2"
}
for i in 1 2 3; do run lib && run lib_xl || exit 1; done
for i in 1 2; do run lib "--ct 6" && run lib_xl "--ct 6" || exit 1; done
