#!/bin/bash
# SQ issue/stall counters per kernel for one short bench run (two --pmc passes, kernel trace only).
# usage: tools/sq_profile.sh TAG [bench args...]; output gpurun_out/sq_TAG/*.csv
set -euo pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -rf gpurun_out/sq1_$TAG gpurun_out/sq2_$TAG
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -f csv -d gpurun_out/sq1_$TAG -o p -- python3 bench.py "$@" --no-cpu > gpurun_out/sq1_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA -f csv -d gpurun_out/sq2_$TAG -o p -- python3 bench.py "$@" --no-cpu > gpurun_out/sq2_$TAG.log 2>&1
python3 tools/sq_summary.py gpurun_out/sq1_$TAG gpurun_out/sq2_$TAG > gpurun_out/sq_$TAG.txt
