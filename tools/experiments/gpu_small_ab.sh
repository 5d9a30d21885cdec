# A/B of the chunk size on U10 streams of 2^14 / 2^18 / 2^22 floats (bench lines; small = 256-bit chunks)
set -o pipefail
cd /root/repo
for k in 14 18 22; do
  for thr in 0 67108864; do
    DC_SMALL_CHUNK_MAX_BYTES=$thr timeout -k 10 200 python3 bench.py --log2n $k --steps 50 --no-cpu --no-pipelined --no-extra > gpurun_out/ab_${k}_${thr}.json 2>&1 || exit 1
  done
done
