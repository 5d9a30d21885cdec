# small-message step (2^14 / 2^18 U10 CT7): default three launches vs variants, plus a rocprof kernel trace at 2^14
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lg in 14 18; do
  for v in "" "DC_FUSED3=1"; do
    env $v timeout -k 10 120 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 50 --warmup 10 --log2n $lg > gpurun_out/sm.json 2> gpurun_out/sm.err || { tail -20 gpurun_out/sm.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/sm.json').readline());print(sys.argv[1],sys.argv[2],d['ms_per_step'],d['kernels_ms'])" $lg "${v:-default}" | tee -a gpurun_out/small_ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_small -o run -- python3 bench.py --no-cpu --no-pipelined --no-extra --steps 50 --warmup 10 --log2n 14 > gpurun_out/prof_small.log 2>&1 || exit 1
python3 tools/kstats.py $(find gpurun_out/prof_small -name "*kernel_stats.csv" | head -1) | head -12
