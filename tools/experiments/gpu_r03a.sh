# r03a: ISA issue-cost microbenchmark, token-walk variants, a quick bench line of the r02 code
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03a.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 240 python3 -u tools/isa_bench.py > gpurun_out/isa_bench.txt 2>&1 && \
timeout -k 10 240 python3 -u tools/walk_bench.py > gpurun_out/walk_bench.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err
rc=$?
tail -n 3 gpurun_out/isa_bench.txt gpurun_out/walk_bench.txt
exit $rc
