# encoder-only A/B of library builds on one box: tools/experiments/enc_ab.sh LIB... (each: 20 launches of
# tools/experiments/enc_time.py, 2^26 CT7, alternating, two rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in "$@"; do
    DCAMD_LIB=$lib timeout -k 10 120 python3 tools/experiments/enc_time.py ${ENC_LG:-26} ${ENC_CT:-7} $lib 2>&1 | grep encode | tee -a gpurun_out/enc_ab.txt || exit 1
  done
done
