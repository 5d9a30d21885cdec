#!/bin/bash
# (r06) halo decode with the scatter fused into the values kernel: halo tests, bench --halo (graph), kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q -k "halo or chunk_map_forced" --timeout 120 --timeout-method thread > gpurun_out/hs_t.log 2>&1 || { tail -40 gpurun_out/hs_t.log; exit 1; }
tail -1 gpurun_out/hs_t.log
for r in 1 2; do for g in 1 0; do
  DC_HALO_GRAPH=$g timeout -k 10 200 python3 -u bench.py --halo --steps 500 > gpurun_out/hs_$g.json 2> gpurun_out/hs_$g.err || { tail -20 gpurun_out/hs_$g.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/hs_$g.json').readline());print('graph=$g',d['value'],d['ms_per_step'],d['config']['exchange_check'],d['config']['launch'])"
done; done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hs -o run -- python3 bench.py --halo --steps 100 > gpurun_out/hs_prof.log 2>&1 || { tail -20 gpurun_out/hs_prof.log; exit 1; }
echo prof ok
