cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for i in 1 2; do for sg in 16 20; do
  DC_DEC3_SEG=$sg timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu --no-pipelined --ct 6 > gpurun_out/c6_${sg}_$i.json 2> gpurun_out/c6_${sg}_$i.err || { tail -20 gpurun_out/c6_${sg}_$i.err; exit 1; }
  python3 tools/bench_summary.py gpurun_out/c6_${sg}_$i.json > gpurun_out/c6_${sg}_$i.txt; echo "ct6 seg $sg run $i: $(grep -E '^value' gpurun_out/c6_${sg}_$i.txt) $(grep -E '^kernels_ms' gpurun_out/c6_${sg}_$i.txt)"
done; done
