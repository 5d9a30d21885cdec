# the GPU test suite (as the driver runs it) + smoke
set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
tail -5 gpurun_out/gt.log
echo "tests rc=$rc"
[ $rc -eq 0 ] && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"
exit $rc
