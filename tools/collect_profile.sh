#!/bin/bash
# Copy the summaries of a tools/profile.sh run (merged back into gpurun_out/) into profiles/.
set -euo pipefail
TAG=$1
cd "$(dirname "$0")/.."
cp gpurun_out/prof_$TAG/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
cp gpurun_out/prof_$TAG/run_domain_stats.csv profiles/${TAG}_domain_stats.csv
python3 tools/pmc_to_json.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG 67108864 7 profiles/${TAG}_pmc.json profiles/r04_fetch_calib.json > /dev/null
cp profiles/${TAG}_pmc.json profiles/pmc_latest.json
grep '^{' gpurun_out/bench_$TAG.log > profiles/${TAG}_bench_under_rocprof.json || true
python3 tools/kstats.py profiles/${TAG}_kernel_stats.csv > profiles/${TAG}_kernel_stats.txt
