# round-4: look-back window A/B (DC_LB_KS 1/2/4/8 x 64 states per round trip over the scanner's states);
# parse3 repairs stopping at the first chunk entry where every lane has met its path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py tests/test_gpu_decode3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_t.log 2>&1 || { tail -40 gpurun_out/r04_t.log; exit 1; }
tail -1 gpurun_out/r04_t.log
run() {
  DCAMD_LIB=data-compression_amd/$1/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(*sys.argv[1:],d['value'],d['ms_per_step'],d['kernels_ms'])" $1
}
for i in 1 2; do run lib && run lib_k1 && run lib_k2 && run lib_k8 || exit 1; done
DC_DEBUG_STAMPS=1 timeout -k 10 120 python3 -u tools/fused_stamps.py > gpurun_out/fs.txt 2>&1 || { tail -20 gpurun_out/fs.txt; exit 1; }
head -8 gpurun_out/fs.txt
DCAMD_LIB=data-compression_amd/lib_p/libdcamd.so timeout -k 10 150 python3 -u tools/dec3_prof.py > gpurun_out/p3.txt 2>&1 || { tail -20 gpurun_out/p3.txt; exit 1; }
cat gpurun_out/p3.txt
for lg in 18 14; do
DC_DEC3_MIN_BYTES=0 DCAMD_LIB=data-compression_amd/lib_p/libdcamd.so timeout -k 10 150 python3 -u tools/dec3_prof.py 7 $lg > gpurun_out/p3_$lg.txt 2>&1 || { tail -20 gpurun_out/p3_$lg.txt; exit 1; }
cat gpurun_out/p3_$lg.txt
done
