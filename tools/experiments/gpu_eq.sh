# config 3 (EQ 2^28) with the slow path timed inside the step, checked against the oracle
set -o pipefail
cd /root/repo
DC_DEBUG_ERR=1 timeout -k 10 400 python -u bench.py --input eq --log2n 28 --steps 5 --warmup 2 --check --no-cpu --no-pipelined --no-extra > gpurun_out/eq28.json 2> gpurun_out/eq28.err
