# round-4: fused encoder at 8 workgroups per CU (64 VGPRs, 18 spilled) vs 7 (lib)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {
  DCAMD_LIB=data-compression_amd/$1/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 $2 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(*sys.argv[1:],d['value'],d['ms_per_step'],d['kernels_ms'])" $1 "$2"
}
for i in 1 2 3; do run lib && run lib_f8 || exit 1; done
