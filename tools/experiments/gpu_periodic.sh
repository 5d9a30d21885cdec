# GPU suite, then the headline bench, the halo bench (config 4) and EQ 2^28 (config 3) with their status
set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err && \
DC_DEBUG_ERR=1 timeout -k 10 300 python -u bench.py --halo --ct 5 --steps 10 --warmup 3 --no-cpu > gpurun_out/halo.json 2> gpurun_out/halo.err && \
DC_DEBUG_ERR=1 timeout -k 10 400 python -u bench.py --input eq --log2n 28 --steps 5 --warmup 2 --no-cpu --no-pipelined --no-extra > gpurun_out/eq28.json 2> gpurun_out/eq28.err
rc=$?
tail -n 2 gpurun_out/gt.log
exit $rc
