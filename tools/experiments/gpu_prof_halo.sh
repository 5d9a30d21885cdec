# kernel trace of the halo bench (config 4) to see where its 1.8 ms per step goes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_halo -o run -- python3 bench.py --halo --ct 5 --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_halo.log 2>&1
