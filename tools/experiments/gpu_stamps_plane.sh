# decoder phase stamps (DC_DEBUG_STAMPS) on one Himeno halo plane (config 4 shape, CT5) and on U10 2^26
set -o pipefail
cd /root/repo
DC_DEBUG_STAMPS=1 timeout -k 10 120 python -u tools/stamps.py 16 plane 5 > gpurun_out/stamps_plane.txt 2>&1 && \
DC_DEBUG_STAMPS=1 timeout -k 10 120 python -u tools/stamps.py 26 u10 7 > gpurun_out/stamps_u10.txt 2>&1
rc=$?; cat gpurun_out/stamps_plane.txt gpurun_out/stamps_u10.txt; exit $rc
