# r03n: after re-entry: the whole GPU suite + smoke + the full bench line (configs, sweep, cpu baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03n.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_n.log 2>&1
rc=$?
tail -n 15 gpurun_out/t_n.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/n_smoke.log 2>&1 || exit $?
cat gpurun_out/n_smoke.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/n_bench.json 2> gpurun_out/n_bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/n_bench.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms']); print(json.dumps(d.get('configs'))[:3000])"
