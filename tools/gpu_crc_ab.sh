#!/bin/bash
# CRC-32 kernels: parity tests, the pass time, config 5's bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "crc or ct9 or config5" > gpurun_out/crc_t.log 2>&1 || { tail -30 gpurun_out/crc_t.log; exit 1; }
tail -1 gpurun_out/crc_t.log
timeout -k 10 120 python3 -u tools/crc_time.py 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu --ber 1e-6 > gpurun_out/crc_b$i.json 2> gpurun_out/crc_b$i.err || { tail -20 gpurun_out/crc_b$i.err; exit 1; }
  python3 tools/bench_summary.py gpurun_out/crc_b$i.json > gpurun_out/crc_b$i.txt; grep -E "^value|^kernels_ms" gpurun_out/crc_b$i.txt
done
