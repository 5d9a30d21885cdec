# decoder/encoder phase stamps (DC_DEBUG_STAMPS) + a short bench, for profiling the hot kernels
set -o pipefail
cd /root/repo
DC_DEBUG_STAMPS=1 timeout -k 10 120 python -u tools/stamps.py 26 > gpurun_out/stamps.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu --no-pipelined --steps 10 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
