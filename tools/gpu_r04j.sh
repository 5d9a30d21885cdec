# round-4 evidence: the whole GPU suite + smoke, FETCH_SIZE calibration of the codec's read patterns,
# kernel trace + PMC passes of the bench (tools/profile.sh), the full bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_tall.log 2>&1 || { tail -40 gpurun_out/r04_tall.log; exit 1; }
tail -1 gpurun_out/r04_tall.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.log 2>&1 || { tail -20 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
rm -rf gpurun_out/calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/calib -o c -- ./tools/fetch_calib > gpurun_out/calib.txt 2>&1 || { tail -20 gpurun_out/calib.txt; exit 1; }
python3 tools/fetch_calib.py gpurun_out/calib gpurun_out/calib.txt gpurun_out/r04_fetch_calib.json
bash tools/profile.sh r04b --no-extra || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/r04b_bench_full.json 2> gpurun_out/r04b_bench_full.err || { tail -20 gpurun_out/r04b_bench_full.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04b_bench_full.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms']);print({k:(v['value'],v['ms_per_step']) for k,v in d.get('sweep',{}).items()});print({k:(v['value'],v['ms_per_step']) for k,v in d.get('configs',{}).items()})"
timeout -k 10 200 python3 -u bench.py --halo --steps 50 > gpurun_out/r04b_halo.json 2> gpurun_out/r04b_halo.err || { tail -20 gpurun_out/r04b_halo.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04b_halo.json').readline());print('halo',d['value'],d['ms_per_step'])"
