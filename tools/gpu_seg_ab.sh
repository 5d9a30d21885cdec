#!/bin/bash
# parse3 segment lengths: the decode3 segment tests, then the quick bench line at each forced length (one box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode3.py -x -q --timeout 120 --timeout-method thread -k "segment_lengths or maps or slow_sync" > gpurun_out/seg_t.log 2>&1 || { tail -30 gpurun_out/seg_t.log; exit 1; }
tail -1 gpurun_out/seg_t.log
for i in 1 2; do
  for sg in 16 20 24; do
    DC_DEC3_SEG=$sg timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > gpurun_out/sab_${sg}_$i.json 2> gpurun_out/sab_${sg}_$i.err || { tail -20 gpurun_out/sab_${sg}_$i.err; exit 1; }
    python3 tools/bench_summary.py gpurun_out/sab_${sg}_$i.json > gpurun_out/sab_${sg}_$i.txt
    echo "seg $sg run $i: $(grep -E '^value' gpurun_out/sab_${sg}_$i.txt) $(grep -E '^kernels_ms' gpurun_out/sab_${sg}_$i.txt)"
  done
done
