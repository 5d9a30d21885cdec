#!/bin/bash
# SQ issue/stall counters per kernel for any short python command (two --pmc passes, kernel trace only).
# usage: tools/sq_profile_cmd.sh TAG script.py [args...]; output gpurun_out/sq_TAG.txt
set -euo pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -rf gpurun_out/sq1_$TAG gpurun_out/sq2_$TAG
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -f csv -d gpurun_out/sq1_$TAG -o p -- python3 "$@" > gpurun_out/sq1_$TAG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA -f csv -d gpurun_out/sq2_$TAG -o p -- python3 "$@" > gpurun_out/sq2_$TAG.log 2>&1
python3 tools/sq_summary.py gpurun_out/sq1_$TAG gpurun_out/sq2_$TAG > gpurun_out/sq_$TAG.txt
