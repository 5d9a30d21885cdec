# round-4: codec + decode3 GPU tests, then bench A/B: two-pass encoder (DC_ENC_PASSES=2), single pass with the
# scanner block (default), single pass with the chained look-back (DC_ENC_SCAN=0), then single-pass stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || { timeout -k 10 700 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py tests/test_gpu_decode3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_t.log 2>&1 || { tail -40 gpurun_out/r04_t.log; exit 1; }; tail -1 gpurun_out/r04_t.log; }
for i in 1 2; do
for cfg in "2 1" "1 1" "1 0"; do
  set -- $cfg
  DC_ENC_PASSES=$1 DC_ENC_SCAN=$2 DCAMD_LIB=data-compression_amd/lib_k4/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print('passes',sys.argv[1],'scan',sys.argv[2],d['value'],d['ms_per_step'],d['kernels_ms'])" $1 $2
done
done
DCAMD_LIB=data-compression_amd/lib_k4/libdcamd.so DC_DEBUG_STAMPS=1 timeout -k 10 120 python3 -u tools/fused_stamps.py > gpurun_out/fs.txt 2>&1 || { tail -20 gpurun_out/fs.txt; exit 1; }
head -12 gpurun_out/fs.txt; sed -n 13,40p gpurun_out/fs.txt | awk 'NR%3==1'
for lib in lib_k4 lib_ns lib_2p; do
  DCAMD_LIB=data-compression_amd/$lib/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(sys.argv[1],d['value'],d['ms_per_step'],d['kernels_ms'])" $lib
done
