#!/bin/bash
# (r06) paired halo encode: the halo GPU tests, then bench.py --halo with DC_HALO_PAIR=1 and 0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 400 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "halo or chunk_map_forced" --timeout 120 --timeout-method thread > gpurun_out/h2_t.log 2>&1 || { tail -40 gpurun_out/h2_t.log; exit 1; }
tail -1 gpurun_out/h2_t.log
for pair in 1 0 1 0; do for ep in 1 0; do
  DC_HALO_EPAIR=$ep DC_HALO_PAIR=$pair timeout -k 10 200 python3 -u bench.py --halo --steps 200 > gpurun_out/h2_${pair}${ep}.json 2> gpurun_out/h2_${pair}${ep}.err || { tail -20 gpurun_out/h2_${pair}${ep}.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/h2_${pair}${ep}.json').readline());print('pair=$pair epair=$ep',d['value'],d['ms_per_step'])"
done; done
