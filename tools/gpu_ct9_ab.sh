# CT9 flow (config 5) A/B: separate CRC passes (default) vs the fused sender / 16 KiB-block receiver CRC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for f in 0 1; do
    DC_CT9_FUSED=$f timeout -k 10 300 python3 -u bench.py --ber 1e-6 --no-extra --no-cpu --no-pipelined --steps 20 > gpurun_out/ct9_$f.json 2> gpurun_out/ct9_$f.err || { tail -20 gpurun_out/ct9_$f.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(next(l for l in open(sys.argv[1]) if l.startswith('{')));c=d['config'];print('fused',sys.argv[2],d['value'],d['ms_per_step'],d['self_check'],c.get('detected_all'));print({k:round(v,4) for k,v in d['kernels_ms'].items()})" gpurun_out/ct9_$f.json $f | tee -a gpurun_out/ct9_ab.txt
  done
done
