# kernel trace of config 3 (EQ 2^28) with the slow path timed: which kernels the decode spends its time in
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_eq -o eq -- python3 $R/bench.py --input eq --log2n 28 --steps 3 --warmup 1 --no-cpu --no-pipelined --no-extra > $R/gpurun_out/prof_eq.log 2>&1
rc=$?
f=$(find $R/gpurun_out/prof_eq -name "*kernel_stats.csv" | head -n 1)
cp "$f" $R/gpurun_out/eq_kernel_stats.csv
exit $rc
