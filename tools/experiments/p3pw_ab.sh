# parse3's pre-walk for 4-chunk segments (small streams): parity of variant builds (codec + decode3 tests), then the
# sweep sizes' step per build.  tools/experiments/p3pw_ab.sh "LIBS..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ "${P3_TESTS:-1}" = "1" ]; then
for lib in $1; do
  DCAMD_LIB=$lib timeout -k 10 600 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_decode3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p3_t.log 2>&1 || { tail -30 gpurun_out/p3_t.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/p3_t.log)"
done
fi
for lg in 14 18 22; do
  for r in 1 2; do
    for lib in data-compression_amd/lib/libdcamd.so $1; do
      DCAMD_LIB=$lib timeout -k 10 120 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 50 --warmup 10 --log2n $lg > gpurun_out/sm.json 2> gpurun_out/sm.err || { tail -20 gpurun_out/sm.err; exit 1; }
      python3 -c "import json,sys;d=json.loads(open('gpurun_out/sm.json').readline());print(sys.argv[1],sys.argv[2].split('/')[1],d['ms_per_step'],d['self_check'],d.get('decoder_fast_path'),d['kernels_ms'])" $lg $lib | tee -a gpurun_out/p3pw_ab.txt
    done
  done
done
