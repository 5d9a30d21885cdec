# A/B of two library builds on one box: tools/gpu_ab.sh LIB_B [tests]
# (tests: decode3 + codec parity of the default build first); bench (no extras) A B A B, kernel table of
# each, also appended to gpurun_out/ab_results.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_ab.sh $* $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
LB=$1
if [ "$2" = "tests" ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_decode3.py tests/test_gpu_codec.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
  tail -1 gpurun_out/ab_t.log
fi
for i in 1 2; do
  for lib in data-compression_amd/lib/libdcamd.so $LB; do
    DCAMD_LIB=$lib timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 $BENCH_ARGS > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(sys.argv[1].split('/')[1],d['value'],d['ms_per_step'],d['kernels_ms'])" $lib | tee -a gpurun_out/ab_results.txt
  done
done
