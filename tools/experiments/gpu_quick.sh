# GPU suite + a quick bench line (no sweep / configs)
set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?
tail -n 2 gpurun_out/gt.log
exit $rc
