set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lg in 26 22; do
DCAMD_LIB=data-compression_amd/lib_p/libdcamd.so timeout -k 10 150 python3 -u tools/dec3_prof.py 7 $lg > gpurun_out/p3_$lg.txt 2>&1 || { tail -20 gpurun_out/p3_$lg.txt; exit 1; }
cat gpurun_out/p3_$lg.txt
done
