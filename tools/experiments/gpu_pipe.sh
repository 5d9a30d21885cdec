# round-4: persistent pipelined single-pass encoder (DC_ENC_PIPE=1, default) vs one tile per workgroup
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "back_to_back or shard or start_bit" --timeout 120 --timeout-method thread > gpurun_out/pipe_t0.log 2>&1 || { tail -30 gpurun_out/pipe_t0.log; exit 1; }
tail -1 gpurun_out/pipe_t0.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_t1.log 2>&1 || { tail -30 gpurun_out/pipe_t1.log; exit 1; }
tail -1 gpurun_out/pipe_t1.log
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; return 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.json').readline());k=d['kernels_ms'];print(*sys.argv[1:],d['value'],d['ms_per_step'],{a:b for a,b in k.items() if 'enc' in a})" "$1"
}
for i in 1 2; do run DC_ENC_PIPE=1 && run DC_ENC_PIPE=0 || exit 1; done
