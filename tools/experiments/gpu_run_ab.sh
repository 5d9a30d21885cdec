# A/B on the headline bench (default library vs lib_v0), then config 3 (EQ 2^28, checked) and the halo
# bench on the default library, then the GPU suite
set -o pipefail
cd /root/repo
V0=$PWD/data-compression_amd/lib_v0/libdcamd.so
timeout -k 10 300 python -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/ab_new.json 2> gpurun_out/ab_new.err && \
DCAMD_LIB=$V0 timeout -k 10 300 python -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/ab_old.json 2> gpurun_out/ab_old.err && \
DC_DEBUG_ERR=1 timeout -k 10 400 python -u bench.py --input eq --log2n 28 --steps 5 --warmup 2 --check --no-cpu --no-pipelined --no-extra > gpurun_out/eq28.json 2> gpurun_out/eq28.err && \
DC_DEBUG_ERR=1 timeout -k 10 300 python -u bench.py --halo --steps 20 --no-cpu > gpurun_out/halo.json 2> gpurun_out/halo.err && \
DCAMD_LIB=$V0 timeout -k 10 300 python -u bench.py --halo --steps 20 --no-cpu > gpurun_out/halo_old.json 2> gpurun_out/halo_old.err && \
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
tail -n 3 gpurun_out/gt.log
exit $rc
