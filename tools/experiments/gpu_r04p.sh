# round-4: CRC-32 blocks staged through LDS with coalesced loads (lib) vs per-lane runs (lib_cs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_codec.py tests/test_gpu_f64.py tests/test_mpi_wrappers.py -m gpu -x -q -k "crc or config5 or ct9 or hamming or flip or bcast" --timeout 120 --timeout-method thread > gpurun_out/r04p_t.log 2>&1 || { tail -30 gpurun_out/r04p_t.log; exit 1; }
tail -1 gpurun_out/r04p_t.log
run() {
  DCAMD_LIB=data-compression_amd/$1/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 $2 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());k=d['kernels_ms'];print(*sys.argv[1:],d['value'],d['ms_per_step'],{a:b for a,b in k.items() if 'crc' in a})" $1 "$2"
}
for i in 1 2; do run lib "--ber 1e-6" && run lib_cs "--ber 1e-6" || exit 1; done
