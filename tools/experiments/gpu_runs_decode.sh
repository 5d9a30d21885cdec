# runs-mode decode (run stepping in phases A/B and the fix-up): GPU suite, then plane stamps, halo / EQ / U10 benches
set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
DC_DEBUG_STAMPS=1 timeout -k 10 120 python -u tools/stamps.py 16 plane 5 > gpurun_out/stamps_plane.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --halo --ct 5 --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_halo_plain.json 2>&1 && \
timeout -k 10 300 python3 bench.py --input eq --log2n 28 --steps 5 --warmup 2 --no-cpu --no-pipelined --no-extra > gpurun_out/bench_eq.json 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/bench_u10.json 2>&1
rc=$?
tail -n 3 gpurun_out/gt.log; cat gpurun_out/stamps_plane.txt | grep -v Warn
exit $rc
