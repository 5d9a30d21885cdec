# exact mean tests (float + double), then the GPU suite
set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_f64.py -x -v -m gpu -k "med_exact or med64_exact or prepasses" --timeout 120 --timeout-method thread > gpurun_out/med.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1
rc=$?
tail -n 3 gpurun_out/med.log gpurun_out/gt.log
exit $rc
