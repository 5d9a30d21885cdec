# small-chunk decoder build: golden diagnostic, GPU suite, plane stamps, halo / 2^18 A/B / EQ / U10 benches
set -o pipefail
cd /root/repo
DC_DEBUG_ERR=1 timeout -k 10 200 python -u tools/dbg_small.py > gpurun_out/dbg_small.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
DC_DEBUG_STAMPS=1 timeout -k 10 120 python -u tools/stamps.py 16 plane 5 > gpurun_out/stamps_plane.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --halo --ct 5 --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_halo_plain.json 2>&1 && \
DC_SMALL_CHUNK_MAX_BYTES=0 timeout -k 10 200 python3 bench.py --halo --ct 5 --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_halo_big.json 2>&1 && \
timeout -k 10 200 python3 bench.py --log2n 18 --steps 50 --no-cpu --no-pipelined --no-extra > gpurun_out/bench_18.json 2>&1 && \
DC_SMALL_CHUNK_MAX_BYTES=0 timeout -k 10 200 python3 bench.py --log2n 18 --steps 50 --no-cpu --no-pipelined --no-extra > gpurun_out/bench_18_big.json 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/bench_u10.json 2>&1
rc=$?
grep -c MISMATCH gpurun_out/dbg_small.txt; tail -n 2 gpurun_out/dbg_small.txt; tail -n 3 gpurun_out/gt.log; grep -v Warn gpurun_out/stamps_plane.txt
exit $rc
