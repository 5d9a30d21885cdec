# r03r: the whole GPU suite + smoke + the full bench line (configs, sweep, cpu baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03r.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r.log 2>&1
rc=$?
tail -n 5 gpurun_out/t_r.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r_smoke.log 2>&1 || exit $?
cat gpurun_out/r_smoke.log
timeout -k 10 360 python3 -u bench.py > gpurun_out/r_bench.json 2> gpurun_out/r_bench.err || { tail -20 gpurun_out/r_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r_bench.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms']); print(json.dumps(d.get('configs'))[:2500])"
