# r03j: A/B of the non-temporal (streaming) x loads / stream and float stores
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03j.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
B="--no-cpu --no-pipelined --no-extra --steps 10"
timeout -k 10 200 python3 -u bench.py $B > gpurun_out/j_nt.json 2> gpurun_out/j_nt.err || exit $?
DCAMD_LIB=data-compression_amd/lib_v0/libdcamd.so timeout -k 10 200 python3 -u bench.py $B > gpurun_out/j_v0.json 2> gpurun_out/j_v0.err || exit $?
for f in j_nt j_v0; do python3 -c "import json;d=json.loads(open('gpurun_out/$f.json').readline());print('$f',d['value'],d['kernels_ms'])"; done
