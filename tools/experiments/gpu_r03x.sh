# r03x: scan in the pack kernel (default build, poll sleep 8) vs the scan launch (lib_b): CT7 and CT6 2^26, CT7 EQ 2^28
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03x.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_decode3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/x_t.log 2>&1 || { tail -30 gpurun_out/x_t.log; exit 1; }
tail -1 gpurun_out/x_t.log
bash tools/gpu_ab.sh data-compression_amd/lib_b/libdcamd.so || exit $?
BENCH_ARGS="--ct 6" bash tools/gpu_ab.sh data-compression_amd/lib_b/libdcamd.so || exit $?
BENCH_ARGS="--input eq --log2n 28 --steps 8" bash tools/gpu_ab.sh data-compression_amd/lib_b/libdcamd.so || exit $?
