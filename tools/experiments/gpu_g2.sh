# bench.py restructure: default run (sweep + configs); stamps of the decoder phases
set -o pipefail
cd /root/repo
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/g2_bench.json 2> gpurun_out/g2_bench.err; echo "bench rc=$?"
DC_DEBUG_STAMPS=1 timeout -k 10 120 python -u tests/stamps.py 26 > gpurun_out/g2_stamps.txt 2>&1; echo "stamps rc=$?"
