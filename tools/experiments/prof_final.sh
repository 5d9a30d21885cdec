#!/bin/bash
# (r06) final profiles: the bench command's kernel trace + PMC passes (tools/gpu_run.sh prof), then the halo step's
# kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1
bash tools/gpu_run.sh $TAG prof || exit 1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_halo_$TAG -o run -- python3 bench.py --halo --steps 100 > gpurun_out/halo_prof_$TAG.log 2>&1 || { tail -20 gpurun_out/halo_prof_$TAG.log; exit 1; }
echo halo prof ok
