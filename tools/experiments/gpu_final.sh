# final round-2 check: GPU suite + smoke, rocprof kernel stats + HBM PMC of the headline bench, full bench line
set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
bash tools/profile.sh ${1:-r02e} --no-extra --steps 20 --warmup 5 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?
tail -n 2 gpurun_out/gt.log
cat gpurun_out/smoke.log
exit $rc
