#!/bin/bash
# CRC pass grid A/B: the receiver pass time and config 5 at several workgroup caps (0 = one per 32 KiB block)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for gc in 4096 0 2048 1024; do
  echo "DC_CRC_GRID=$gc: $(DC_CRC_GRID=$gc timeout -k 10 120 python3 -u tools/crc_time.py 2>&1 | grep -v amdgpu.ids)"
done
for gc in 4096 0 2048; do
  DC_CRC_GRID=$gc timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu --ber 1e-6 > gpurun_out/cg_$gc.json 2> gpurun_out/cg_$gc.err || { tail -20 gpurun_out/cg_$gc.err; exit 1; }
  python3 tools/bench_summary.py gpurun_out/cg_$gc.json > gpurun_out/cg_$gc.txt; echo "grid $gc: $(grep -E '^value' gpurun_out/cg_$gc.txt)"; grep -E '^kernels_ms' gpurun_out/cg_$gc.txt
done
