# r03m: the whole GPU suite + a bench line (value timed without events)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03m.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_m.log 2>&1
rc=$?
tail -n 15 gpurun_out/t_m.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/m_bench.json 2> gpurun_out/m_bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/m_bench.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms'])"
