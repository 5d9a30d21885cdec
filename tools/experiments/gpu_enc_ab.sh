# round-4: single-pass encoder store rounds (lib: 4 words per thread per round; lib_a: 1; lib_b: 8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in lib lib_b; do
  DBG_ORACLE=1 DCAMD_LIB=data-compression_amd/$v/libdcamd.so timeout -k 10 200 python -u tools/experiments/dbg_pipe.py 26 20 > gpurun_out/dbg_$v.txt 2>&1 || { tail -5 gpurun_out/dbg_$v.txt; exit 1; }
  echo "$v: $(grep -c differ gpurun_out/dbg_$v.txt) bad reps of 20"
done
run() {
  env DCAMD_LIB=data-compression_amd/$1/libdcamd.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());k=d['kernels_ms'];print(*sys.argv[1:],d['value'],d['ms_per_step'],{a:b for a,b in k.items() if 'enc' in a})" $1
}
for i in 1 2 3; do for v in lib lib_a lib_b; do run $v || exit 1; done; done
for v in lib lib_a; do DCAMD_LIB=data-compression_amd/$v/libdcamd.so DC_DEBUG_STAMPS=1 timeout -k 10 100 python -u tools/fused_stamps.py 2>&1 | head -6; done
