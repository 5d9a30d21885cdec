# round-4: pipelined encoder variants (lib: tickets 4/CU; lib_a: static tiles 4/CU; lib_b: tickets 3/CU; lib_c: static 3/CU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in lib lib_a lib_b lib_c; do
  DBG_ORACLE=1 DCAMD_LIB=data-compression_amd/$v/libdcamd.so timeout -k 10 200 python -u tools/experiments/dbg_pipe.py 26 20 > gpurun_out/dbg_$v.txt 2>&1 || { tail -5 gpurun_out/dbg_$v.txt; exit 1; }
  echo "$v: $(grep -c differ gpurun_out/dbg_$v.txt) bad reps of 20"
done
run() {
  env DCAMD_LIB=data-compression_amd/$1/libdcamd.so $2 timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());k=d['kernels_ms'];print(*sys.argv[1:],d['value'],d['ms_per_step'],{a:b for a,b in k.items() if 'enc' in a})" $1 "$2"
}
for i in 1 2; do for v in lib lib_a lib_b lib_c; do run $v DC_ENC_PIPE=1 || exit 1; done; run lib DC_ENC_PIPE=0 || exit 1; done
