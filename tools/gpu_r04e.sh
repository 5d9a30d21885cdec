# round-4 closing evidence (r04e, after the segment-decoder robustness fixes): the whole GPU suite + smoke,
# kernel trace + PMC passes of the bench, the full bench line, the halo bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04e_tall.log 2>&1 || { tail -40 gpurun_out/r04e_tall.log; exit 1; }
tail -1 gpurun_out/r04e_tall.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04e_smoke.log 2>&1 || { tail -20 gpurun_out/r04e_smoke.log; exit 1; }
tail -1 gpurun_out/r04e_smoke.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile.sh r04e --no-extra || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/r04e_bench_full.json 2> gpurun_out/r04e_bench_full.err || { tail -20 gpurun_out/r04e_bench_full.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04e_bench_full.json').readline());print(d['value'],d['ms_per_step'],d['kernels_ms']);print({k:(v['value'],v['ms_per_step']) for k,v in d.get('sweep',{}).items()});print({k:(v['value'],v['ms_per_step']) for k,v in d.get('configs',{}).items()})"
timeout -k 10 200 python3 -u bench.py --halo --steps 50 > gpurun_out/r04e_halo.json 2> gpurun_out/r04e_halo.err || { tail -20 gpurun_out/r04e_halo.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04e_halo.json').readline());print('halo',d['value'],d['ms_per_step'])"
