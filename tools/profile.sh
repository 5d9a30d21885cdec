#!/bin/bash
# Profile bench.py on the GPU box: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes.  Summaries land in profiles/ (tracked); raw output in gpurun_out/ (scratch).
# usage: tools/profile.sh TAG [bench args...]
set -euo pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$TAG gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py "$@" --no-cpu --no-pipelined > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmcf_$TAG -o p -- python3 bench.py "$@" --no-cpu --no-pipelined > gpurun_out/pmcf_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/pmcw_$TAG -o p -- python3 bench.py "$@" --no-cpu --no-pipelined > gpurun_out/pmcw_$TAG.log 2>&1
# the box only hands back gpurun_out/: tools/collect_profile.sh TAG copies these into profiles/
python3 tools/pmc_to_json.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG 67108864 7 gpurun_out/${TAG}_pmc.json
