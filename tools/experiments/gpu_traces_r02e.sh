# kernel traces of config 4 (Himeno halo planes) and config 3 (EQ 2^28) on the final round-2 code
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_halo -o halo -- python3 $R/bench.py --halo --ct 5 --steps 10 --warmup 3 --no-cpu > $R/gpurun_out/bench_halo.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_eq -o eq -- python3 $R/bench.py --input eq --log2n 28 --steps 3 --warmup 1 --no-cpu --no-pipelined --no-extra > $R/gpurun_out/prof_eq.log 2>&1 && \
timeout -k 10 200 python3 $R/bench.py --halo --ct 5 --steps 50 --warmup 5 --no-cpu > $R/gpurun_out/bench_halo_plain.json 2>&1
rc=$?
for t in halo eq; do f=$(find $R/gpurun_out/prof_$t -name "*kernel_stats.csv" | head -n 1); [ -n "$f" ] && cp "$f" $R/gpurun_out/${t}_kernel_stats.csv; done
exit $rc
