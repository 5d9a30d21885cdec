# A/B/C of library builds on one box: tools/gpu_abc.sh LIB... ; decode3 parity of each variant, then the
# bench (no extras) over all builds twice; lines also appended to gpurun_out/ab_results.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_abc.sh $* $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
for lib in "$@"; do
  DCAMD_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decode3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abc_t.log 2>&1 || { tail -30 gpurun_out/abc_t.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/abc_t.log)"
done
for i in 1 2; do
  for lib in data-compression_amd/lib/libdcamd.so "$@"; do
    DCAMD_LIB=$lib timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(sys.argv[1].split('/')[1],d['value'],d['ms_per_step'],d['kernels_ms'])" $lib | tee -a gpurun_out/ab_results.txt
  done
done
