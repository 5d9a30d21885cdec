# decode3 parallel pending rounds + table-driven maps parse: parity, then slow-sync timings and a kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode3.py tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05d_t.log 2>&1 || { tail -30 gpurun_out/r05d_t.log; exit 1; }
tail -1 gpurun_out/r05d_t.log
O=gpurun_out/r05d_slow_sync.txt; : > $O
for a in "7 ramp 1e-3" "7 sine 1e-5" "11 normal 1e-3" "5 ramp 1e-3" "7 u10 1e-3"; do
  set -- $a
  timeout -k 10 120 python3 -u tools/seg_time.py 24 $1 16 $3 $2 2>&1 | grep -v amdgpu.ids >> $O || { tail -20 $O; exit 1; }
done
cat $O
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for k in ramp sine; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_maps_$k -o run -- python3 tools/seg_time.py 24 7 16 $([ $k = sine ] && echo 1e-5 || echo 1e-3) $k > gpurun_out/maps_prof_$k.log 2>&1 || exit 1
  python3 tools/kstats.py gpurun_out/prof_maps_$k/run_kernel_stats.csv | head -8
done
