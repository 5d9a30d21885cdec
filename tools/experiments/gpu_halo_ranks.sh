# halo bench: one rank, then 2 and 3 gloo ranks on the one GPU (z-neighbour exchange inside the timed step)
set -o pipefail
cd /root/repo
timeout -k 10 200 python3 bench.py --halo --ct 5 --steps 50 --warmup 5 --no-cpu > gpurun_out/halo_1.json 2>&1 && \
DC_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --halo --ct 5 --gpus 2 --steps 30 --warmup 3 --no-cpu > gpurun_out/halo_2_gloo.json 2>&1 && \
DC_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --halo --ct 5 --gpus 3 --steps 30 --warmup 3 --no-cpu > gpurun_out/halo_3_gloo.json 2>&1
rc=$?; for f in halo_1 halo_2_gloo halo_3_gloo; do grep '^{' gpurun_out/$f.json | cut -c 1-400; done; tail -3 gpurun_out/halo_3_gloo.json; exit $rc
