# occupancy sensitivity of parse/decode (LDS padding variants)
set -o pipefail
cd /root/repo
for v in lib lib_v1 lib_v2 lib_v3; do
  DCAMD_LIB=$PWD/data-compression_amd/$v/libdcamd.so timeout -k 10 120 python -u bench.py --no-cpu --no-pipelined --steps 10 > gpurun_out/occ_$v.json 2>gpurun_out/occ_$v.err || exit 1
done
echo ok
