# round-4: CRC-32 final combine with table-driven constant multiplies (lib) vs bit-serial (lib_a)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fullsize.py -m gpu -x -q -k "crc or config5 or ct9 or resend" --timeout 120 --timeout-method thread > gpurun_out/crc_t.log 2>&1 || { tail -30 gpurun_out/crc_t.log; exit 1; }
tail -1 gpurun_out/crc_t.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in lib lib_a; do
  rm -rf gpurun_out/crcprof_$v
  DCAMD_LIB=data-compression_amd/$v/libdcamd.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/crcprof_$v -o r -- python3 tools/crc_time.py > gpurun_out/crcprof_$v.log 2>&1 || { tail -5 gpurun_out/crcprof_$v.log; exit 1; }
  DCAMD_LIB=data-compression_amd/$v/libdcamd.so timeout -k 10 60 python3 tools/crc_time.py 2>&1 | grep -v amdgpu.ids
done
