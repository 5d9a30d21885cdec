#!/bin/bash
# fused3d_kernel (DC_FUSED3=2: static rounds by the parsing workgroup + dynamic tickets): its tests and the static
# fused tests, the A/B tool with stamps per static share, then the quick bench line on / off, alternating (one box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f3d_tests.log 2>&1 || { tail -30 gpurun_out/f3d_tests.log; exit 1; }
tail -1 gpurun_out/f3d_tests.log
for sq in 3 2 4 1; do
  echo "== DC_F3D_STATIC=$sq"
  DC_F3D_STATIC=$sq DC_FUSED3_STAMPS=1 timeout -k 10 120 python3 -u tools/experiments/fused3_ab.py 26 7 enc dyn seg20 > gpurun_out/f3d_stamps_$sq.txt 2>&1 || { tail -20 gpurun_out/f3d_stamps_$sq.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/f3d_stamps_$sq.txt
done
for i in 1 2; do
  for f in 2 0; do
    DC_FUSED3=$f timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > gpurun_out/f3d_${f}_$i.json 2> gpurun_out/f3d_${f}_$i.err || { tail -20 gpurun_out/f3d_${f}_$i.err; exit 1; }
    python3 tools/bench_summary.py gpurun_out/f3d_${f}_$i.json > gpurun_out/f3d_${f}_$i.txt
    echo "DC_FUSED3=$f run $i: $(grep -E '^value' gpurun_out/f3d_${f}_$i.txt)"
    grep -E "^kernels_ms" gpurun_out/f3d_${f}_$i.txt
  done
done
