set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in lib; do
  echo "== $v"
  DBG_ORACLE=1 DCAMD_LIB=data-compression_amd/$v/libdcamd.so timeout -k 10 200 python -u tools/experiments/dbg_pipe.py 26 300 > gpurun_out/dbg_$v.txt 2>&1 || { tail -5 gpurun_out/dbg_$v.txt; exit 1; }
  grep -v "amdgpu.ids\|same" gpurun_out/dbg_$v.txt | head -20
done
