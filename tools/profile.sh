#!/bin/bash
# Profile bench.py on the GPU box: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes.  Summaries land in profiles/ (tracked); raw output in gpurun_out/ (scratch).
# usage: tools/profile.sh TAG [bench args...]
set -euo pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p profiles gpurun_out
rm -rf gpurun_out/prof_$TAG gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py "$@" --no-cpu > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/pmcf_$TAG -o p -- python3 bench.py "$@" --no-cpu > gpurun_out/pmcf_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/pmcw_$TAG -o p -- python3 bench.py "$@" --no-cpu > gpurun_out/pmcw_$TAG.log 2>&1
cp gpurun_out/prof_$TAG/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
python3 tools/pmc_to_json.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG 67108864 7 profiles/${TAG}_pmc.json
cp profiles/${TAG}_pmc.json profiles/pmc_latest.json
grep '^{' gpurun_out/bench_$TAG.log > profiles/${TAG}_bench_under_rocprof.json || true
