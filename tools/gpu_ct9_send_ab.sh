#!/bin/bash
# CT9 send without a copy pass: parity tests, then config 5's bench line in both modes, alternating (one box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "crc or ct9 or config5 or send" > gpurun_out/ct9s_t.log 2>&1 || { tail -30 gpurun_out/ct9s_t.log; exit 1; }
tail -1 gpurun_out/ct9s_t.log
for i in 1 2; do
  for m in send copy; do
    DC_CT9_MODE=$m timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu --ber 1e-6 > gpurun_out/ct9s_${m}_$i.json 2> gpurun_out/ct9s_${m}_$i.err || { tail -20 gpurun_out/ct9s_${m}_$i.err; exit 1; }
    python3 tools/bench_summary.py gpurun_out/ct9s_${m}_$i.json > gpurun_out/ct9s_${m}_$i.txt
    echo "$m run $i: $(grep -E '^value' gpurun_out/ct9s_${m}_$i.txt)"; grep -E '^kernels_ms' gpurun_out/ct9s_${m}_$i.txt
  done
done
timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > gpurun_out/ct9s_main.json 2> gpurun_out/ct9s_main.err || { tail -20 gpurun_out/ct9s_main.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/ct9s_main.json > gpurun_out/ct9s_main.txt; echo "headline: $(grep -E '^value' gpurun_out/ct9s_main.txt)"; grep -E '^kernels_ms' gpurun_out/ct9s_main.txt
