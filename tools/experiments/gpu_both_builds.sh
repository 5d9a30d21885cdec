set -o pipefail
cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -q -m gpu -k "both_decoder_builds or ragged or golden" --timeout 240 --timeout-method thread > gpurun_out/gt_both.log 2>&1
rc=$?; tail -n 4 gpurun_out/gt_both.log; exit $rc
