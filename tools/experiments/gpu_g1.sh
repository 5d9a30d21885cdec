set -o pipefail
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/g1_bench.json 2> gpurun_out/g1_bench.err && \
DC_DEBUG_ERR=1 timeout -k 10 400 python -u bench.py --input eq --log2n 28 --steps 5 --warmup 2 --check --no-cpu --no-pipelined > gpurun_out/g1_eq28.json 2> gpurun_out/g1_eq28.err
echo done
