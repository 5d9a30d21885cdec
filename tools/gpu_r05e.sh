# med_dataset rewrite (narrow window, one wave per chunk, LDS ring): parity, timing, kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_f64.py tests/test_gpu_dist.py -m gpu -x -q -k "med or global" --timeout 120 --timeout-method thread > gpurun_out/r05e_t.log 2>&1 || { tail -30 gpurun_out/r05e_t.log; exit 1; }
tail -1 gpurun_out/r05e_t.log
timeout -k 10 200 python3 -u tools/experiments/med_time.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_med2 -o run -- python3 tools/experiments/med_time.py 26 > gpurun_out/med_prof2.log 2>&1 || exit 1
python3 tools/kstats.py gpurun_out/prof_med2/run_kernel_stats.csv | head -8
DCAMD_LIB=data-compression_amd/lib_mp/libdcamd.so timeout -k 10 120 python3 tools/experiments/med_prof.py 26 2>&1 | grep -v amdgpu.ids
