# r03h: ticket vs static job mapping; FETCH_SIZE of the segment decoder kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03h.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
B="--no-cpu --no-pipelined --no-extra --steps 10"
timeout -k 10 200 python3 -u bench.py $B > gpurun_out/h_base.json 2> gpurun_out/h_base.err || exit $?
DCAMD_LIB=data-compression_amd/lib_s1/libdcamd.so timeout -k 10 200 python3 -u bench.py $B > gpurun_out/h_s1.json 2> gpurun_out/h_s1.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/h_pmcf -o p -- python3 bench.py --no-cpu --no-pipelined --no-extra --steps 3 --warmup 1 > gpurun_out/h_pmcf.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/h_pmcw -o p -- python3 bench.py --no-cpu --no-pipelined --no-extra --steps 3 --warmup 1 > gpurun_out/h_pmcw.log 2>&1 || exit $?
for f in h_base h_s1; do python3 -c "import json;d=json.loads(open('gpurun_out/$f.json').readline());print('$f',d['value'],d['kernels_ms'])"; done
