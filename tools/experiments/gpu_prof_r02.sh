# round-2 profile of the headline bench: kernel stats + HBM PMC (tools/profile.sh), then a full bench line
set -o pipefail
cd /root/repo
bash tools/profile.sh r02b --no-extra --steps 20 --warmup 5 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
