# small-message step: default vs the maps parse (DC_DEC3_MAPS=1) vs 8-chunk segments, 2^14 / 2^18 U10 CT7
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lg in 14 18; do
  for v in "DC_X=0" "DC_DEC3_MAPS=1" "DC_DEC3_SEG=8"; do
    env $v timeout -k 10 120 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 50 --warmup 10 --log2n $lg > gpurun_out/sm.json 2> gpurun_out/sm.err || { tail -20 gpurun_out/sm.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/sm.json').readline());print(sys.argv[1],sys.argv[2],d['ms_per_step'],d['self_check'],d['kernels_ms'])" $lg "$v" | tee -a gpurun_out/small_ab.txt
  done
done
