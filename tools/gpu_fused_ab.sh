#!/bin/bash
# fused3 tests, SQ counters of both decoders (tools/experiments/fused3_ab.py under two --pmc passes), the
# phase stamps, then the quick bench line with the fused launch on / off, alternating (one box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f3_tests.log 2>&1 || { tail -30 gpurun_out/f3_tests.log; exit 1; }
tail -1 gpurun_out/f3_tests.log
bash tools/sq_profile_cmd.sh fused3 tools/experiments/fused3_ab.py 26 7 enc || exit 1
DC_FUSED3_STAMPS=1 timeout -k 10 120 python3 -u tools/experiments/fused3_ab.py 26 7 enc > gpurun_out/f3_stamps.txt 2>&1 || { tail -20 gpurun_out/f3_stamps.txt; exit 1; }
for i in 1 2 3; do
  for f in 1 0; do
    DC_FUSED3=$f timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > gpurun_out/fab_${f}_$i.json 2> gpurun_out/fab_${f}_$i.err || { tail -20 gpurun_out/fab_${f}_$i.err; exit 1; }
    python3 tools/bench_summary.py gpurun_out/fab_${f}_$i.json > gpurun_out/fab_${f}_$i.txt
    echo "DC_FUSED3=$f run $i: $(grep -E '^value' gpurun_out/fab_${f}_$i.txt)"
    grep -E "^kernels_ms" gpurun_out/fab_${f}_$i.txt
  done
done
