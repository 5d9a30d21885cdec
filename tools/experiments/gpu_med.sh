# exact mean tests, then the GPU suite and a quick bench (med_dataset_s in phases_ms)
set -o pipefail
cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -v -m gpu -k med_exact --timeout 120 --timeout-method thread > gpurun_out/med.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?
tail -3 gpurun_out/med.log gpurun_out/gt.log
exit $rc
