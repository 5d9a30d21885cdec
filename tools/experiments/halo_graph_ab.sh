#!/bin/bash
# (r06) halo step as one HIP graph: the halo GPU tests, then bench.py --halo with DC_HALO_GRAPH=1 / 0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "halo or chunk_map_forced" --timeout 120 --timeout-method thread > gpurun_out/hg_t.log 2>&1 || { tail -40 gpurun_out/hg_t.log; exit 1; }
tail -1 gpurun_out/hg_t.log
for r in 1 2; do for g in 1 0; do for ep in 0 1; do
  DC_HALO_GRAPH=$g DC_HALO_EPAIR=$ep timeout -k 10 200 python3 -u bench.py --halo --steps 500 > gpurun_out/hg_${g}${ep}.json 2> gpurun_out/hg_${g}${ep}.err || { tail -20 gpurun_out/hg_${g}${ep}.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/hg_${g}${ep}.json').readline());print('graph=$g epair=$ep',d['value'],d['ms_per_step'],d['config']['exchange_check'],d['config']['launch'])"
done; done; done
