# round-4: look-back window variants (LIBS), then the CT9 config-5 line (--ber 1e-6)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in ${LIBS:-lib}; do
  DCAMD_LIB=data-compression_amd/$lib/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());print(sys.argv[1],d['value'],d['ms_per_step'],d['kernels_ms'])" $lib
done
DC_ENC_PASSES=2 timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 --ber 1e-6 > gpurun_out/ct9.json 2> gpurun_out/ct9.err || { tail -20 gpurun_out/ct9.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/ct9.json').readline());print('ct9',d['value'],d['ms_per_step'],d.get('kernels_sum_ms'),d['config'].get('detected_all'),d['kernels_ms'])"
