#!/bin/bash
# (r06) halo min-fold A/B (DC_HALO_MIN2=1: the separate min_final launch), then the evidence steps of tools/gpu_run.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "halo" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_halo_t.log 2>&1 || { tail -40 gpurun_out/${TAG}_halo_t.log; exit 1; }
tail -1 gpurun_out/${TAG}_halo_t.log
for r in 1 2; do for m in 0 1; do
  DC_HALO_MIN2=$m timeout -k 10 200 python3 -u bench.py --halo --steps 500 > gpurun_out/${TAG}_hm$m.json 2> gpurun_out/${TAG}_hm$m.err || { tail -20 gpurun_out/${TAG}_hm$m.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_hm$m.json').readline());print('min2=$m',d['value'],d['ms_per_step'],d['config']['exchange_check'])"
done; done
bash tools/gpu_run.sh $TAG "$@"
