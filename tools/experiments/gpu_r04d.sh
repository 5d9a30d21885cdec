set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in lib_k4 lib; do
DCAMD_LIB=data-compression_amd/$lib/libdcamd.so DC_DEBUG_STAMPS=1 timeout -k 10 120 python3 -u tools/fused_stamps.py > gpurun_out/fs_$lib.txt 2>&1 || { tail -20 gpurun_out/fs_$lib.txt; exit 1; }
echo "== $lib"; head -12 gpurun_out/fs_$lib.txt; sed -n 13,40p gpurun_out/fs_$lib.txt | awk 'NR%3==1'
done
