# round-4: the small-stream decoder (tests, halo planes, 2^14 sweep point, --halo), CRC nibble tables
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_decode_runs.py tests/test_gpu_codec.py tests/test_gpu_decode3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l_t.log 2>&1 || { tail -40 gpurun_out/r04l_t.log; exit 1; }
tail -1 gpurun_out/r04l_t.log
timeout -k 10 200 python3 -u bench.py --halo --steps 50 > gpurun_out/halo.json 2> gpurun_out/halo.err || { tail -20 gpurun_out/halo.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/halo.json').readline());print('halo',d['value'],d['ms_per_step'],d['config']['stream_bytes'])"
for lg in 14 16; do
timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --log2n $lg --steps 50 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(sys.argv[1],d['value'],d['ms_per_step'],d['kernels_ms'])" $lg
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_halo -o run -- python3 bench.py --halo --steps 20 > gpurun_out/prof_halo.log 2>&1 || { tail -20 gpurun_out/prof_halo.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof_halo/run_kernel_stats.csv | head -20
