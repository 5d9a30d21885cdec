# round-4 experiment batch: default-library GPU tests; the 2-phase parse build (lib_2p) under the decoder
# tests; bench A/B of encoder variants and decoder builds (lib_ns: no output stores, diagnostic); stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="tests/test_gpu_codec.py tests/test_gpu_fullsize.py tests/test_gpu_decode3.py"
timeout -k 10 700 python3 -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_t.log 2>&1 || { tail -40 gpurun_out/r04_t.log; exit 1; }
tail -1 gpurun_out/r04_t.log
DCAMD_LIB=data-compression_amd/lib_2p/libdcamd.so timeout -k 10 700 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_decode3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_t2.log 2>&1 || { tail -40 gpurun_out/r04_t2.log; exit 1; }
tail -1 gpurun_out/r04_t2.log
run() {  # lib passes scan
  DC_ENC_PASSES=$2 DC_ENC_SCAN=$3 DCAMD_LIB=data-compression_amd/$1/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(*sys.argv[1:],d['value'],d['ms_per_step'],d['kernels_ms'])" $1 $2 $3
}
for i in 1 2; do
  run lib 2 1 && run lib 1 1 && run lib 1 0 && run lib_2p 1 1 && run lib_ns 1 1 || exit 1
done
DC_DEBUG_STAMPS=1 timeout -k 10 120 python3 -u tools/fused_stamps.py > gpurun_out/fs.txt 2>&1 || { tail -20 gpurun_out/fs.txt; exit 1; }
head -12 gpurun_out/fs.txt
