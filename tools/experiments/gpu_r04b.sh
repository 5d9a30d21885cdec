# round-4 diagnostics: encoder parity, single-pass stamps, look-back variants (lib_k2/k16/s10), decoder sections
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_t.log 2>&1 || { tail -40 gpurun_out/r04_t.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/r04_t.log
DC_DEBUG_STAMPS=1 timeout -k 10 120 python3 -u tools/fused_stamps.py > gpurun_out/fs.txt 2>&1 || { tail -20 gpurun_out/fs.txt; exit 1; }
cat gpurun_out/fs.txt
for lib in ${LIBS:-lib lib_k2 lib_k16}; do
  for v in ${VARIANTS:-1}; do
  DC_ENC_PASSES=$v DCAMD_LIB=data-compression_amd/$lib/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(sys.argv[1],sys.argv[2],d['value'],d['ms_per_step'],d['kernels_ms'])" $lib $v
  done
done
[ -n "$SKIP_PROF" ] || DCAMD_LIB=data-compression_amd/lib_p/libdcamd.so timeout -k 10 120 python3 -u tools/dec3_prof.py 7 26 > gpurun_out/prof.txt 2>&1 || { tail -20 gpurun_out/prof.txt; exit 1; }
[ -n "$SKIP_PROF" ] || cat gpurun_out/prof.txt
