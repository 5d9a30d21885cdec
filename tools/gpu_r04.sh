# round-4 GPU check: tools/gpu_r04.sh [tests...] -- the listed GPU test files (default: codec + full size),
# then the bench A/B of encoder variants (DC_ENC_PASSES=1 single pass vs 2) and decoder settings, twice each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r04.sh $* $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
T="${TESTS:-tests/test_gpu_codec.py tests/test_gpu_fullsize.py}"
if [ "$T" != "none" ]; then
  timeout -k 10 900 python3 -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_t.log 2>&1 || { tail -40 gpurun_out/r04_t.log; exit 1; }
  tail -2 gpurun_out/r04_t.log
fi
for i in 1 2; do
  for v in ${VARIANTS:-1 2}; do
    DC_ENC_PASSES=$v timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 $BENCH_ARGS > gpurun_out/r04_b.json 2> gpurun_out/r04_b.err || { tail -20 gpurun_out/r04_b.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/r04_b.json').readline());print('enc',sys.argv[1],d['value'],d['ms_per_step'],d['kernels_ms'])" $v | tee -a gpurun_out/r04_results.txt
  done
done
