# A/B: default library vs an experiment variant (lib_v0), then the GPU test suite on the default
set -o pipefail
cd /root/repo
timeout -k 10 300 python -u bench.py --no-cpu --no-pipelined --steps 10 > gpurun_out/ab_new.json 2> gpurun_out/ab_new.err && \
DCAMD_LIB=$PWD/data-compression_amd/lib_v0/libdcamd.so timeout -k 10 300 python -u bench.py --no-cpu --no-pipelined --steps 10 > gpurun_out/ab_old.json 2> gpurun_out/ab_old.err && \
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
tail -5 gpurun_out/gt.log
exit $rc
