# r03v: the Himeno halo step (config 4) and the 2^14 sweep point under a kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03v.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 200 python3 -u bench.py --halo --steps 20 > gpurun_out/v_halo.json 2> gpurun_out/v_halo.err || { tail -20 gpurun_out/v_halo.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/v_halo.json').readline());print(d['value'],d['ms_per_step'])"
rm -rf gpurun_out/v_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/v_prof -o run -- python3 bench.py --halo --steps 20 > gpurun_out/v_prof.log 2>&1 || exit $?
python3 tools/kstats.py gpurun_out/v_prof/run_kernel_stats.csv | head -25
