#!/bin/bash
# One GPU-box evidence run: usage  tools/gpu_run.sh TAG STEP...   (run from gpurun; every GPU step under its
# own time limit, the first failure ends the run).  Steps:
#   tests     the whole GPU suite (-m gpu) + smoke()
#   bench     the full bench line (N=1: sweep, configs, cpu_baseline) -> gpurun_out/TAG_bench_full.json
#   quick     bench.py --no-extra --no-cpu -> gpurun_out/TAG_bench_quick.json
#   gloo2     the multi-rank path rehearsed on this one GPU: 2 ranks over gloo -> TAG_bench_2ranks_1gpu_gloo.json
#   gloo3     the same with 3 ranks
#   prof      rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the bench (tools/profile.sh TAG)
#   halo      bench.py --halo
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tall.log 2>&1 || { tail -40 gpurun_out/${TAG}_tall.log; exit 1; }
      tail -1 gpurun_out/${TAG}_tall.log
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -1 gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 600 python3 -u bench.py > gpurun_out/${TAG}_bench_full.json 2> gpurun_out/${TAG}_bench_full.err || { tail -20 gpurun_out/${TAG}_bench_full.err; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${TAG}_bench_full.json ;;
    quick)
      timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > gpurun_out/${TAG}_bench_quick.json 2> gpurun_out/${TAG}_bench_quick.err || { tail -20 gpurun_out/${TAG}_bench_quick.err; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${TAG}_bench_quick.json ;;
    gloo2|gloo3)
      N=${step#gloo}
      DC_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus $N --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_${N}ranks_1gpu_gloo.json 2> gpurun_out/${TAG}_bench_${N}ranks_1gpu_gloo.err || { tail -30 gpurun_out/${TAG}_bench_${N}ranks_1gpu_gloo.err; exit 1; }
      python3 tools/bench_summary.py gpurun_out/${TAG}_bench_${N}ranks_1gpu_gloo.json ;;
    prof)
      cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
      bash tools/profile.sh ${TAG} --no-extra || exit 1 ;;
    halo)
      timeout -k 10 200 python3 -u bench.py --halo --steps 50 > gpurun_out/${TAG}_halo.json 2> gpurun_out/${TAG}_halo.err || { tail -20 gpurun_out/${TAG}_halo.err; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_halo.json').readline());print('halo',d['value'],d['ms_per_step'])" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
