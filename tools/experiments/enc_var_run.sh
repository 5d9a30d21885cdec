# one GPU call: exactness of variant encoder builds (full-size tests), then the encoder-only A/B and phase stamps
#   tools/experiments/enc_var_run.sh "LIB_FOR_TESTS..." "LIBS_FOR_AB..." "LIBS_FOR_STAMPS..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in $1; do
  DCAMD_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ct7_u10 or back_to_back or occupying" > gpurun_out/ev_t.log 2>&1 || { tail -30 gpurun_out/ev_t.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/ev_t.log)"
done
bash tools/experiments/enc_ab.sh $2 || exit 1
for lib in $3; do
  echo "== stamps $lib"
  DC_DEBUG_STAMPS=1 DCAMD_LIB=$lib timeout -k 10 120 python3 tools/fused_stamps.py 2>&1 | head -12 || exit 1
done
