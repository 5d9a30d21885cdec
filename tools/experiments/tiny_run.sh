# the one-workgroup decoder: parity (tests/test_gpu_tiny.py) of the default build and of variant builds, then the
# 2^14 step of each build (and of the segment decoder, DC_TINY=0)
#   tools/experiments/tiny_run.sh "VARIANT_LIBS..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tiny.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tiny_t.log 2>&1 || { tail -40 gpurun_out/tiny_t.log; exit 1; }
tail -1 gpurun_out/tiny_t.log
for lib in $1; do
  DCAMD_LIB=$lib timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tiny.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tiny_t.log 2>&1 || { tail -40 gpurun_out/tiny_t.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/tiny_t.log)"
done
for r in 1 2; do
  for v in "DC_TINY=0" "DCAMD_LIB=data-compression_amd/lib/libdcamd.so" $(for l in $1; do echo DCAMD_LIB=$l; done); do
    env $v timeout -k 10 120 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 100 --warmup 10 --log2n 14 > gpurun_out/sm.json 2> gpurun_out/sm.err || { tail -20 gpurun_out/sm.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/sm.json').readline());print(sys.argv[1],d['ms_per_step'],d['self_check'],d['kernels_ms'])" "$v" | tee -a gpurun_out/small_ab.txt
  done
done
