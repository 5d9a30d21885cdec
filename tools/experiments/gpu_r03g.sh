# r03g: section timing of the segment decoder (prof build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03g.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
DCAMD_LIB=data-compression_amd/lib_p/libdcamd.so timeout -k 10 200 python3 -u tools/dec3_prof.py 7 26 1e-3 > gpurun_out/prof3.txt 2>&1
rc=$?
cat gpurun_out/prof3.txt
exit $rc
