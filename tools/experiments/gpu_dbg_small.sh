set -o pipefail
cd /root/repo
DC_DEBUG_ERR=1 timeout -k 10 200 python -u tools/dbg_small.py > gpurun_out/dbg_small.txt 2>&1
rc=$?; grep -v Warn gpurun_out/dbg_small.txt | tail -40; exit $rc
