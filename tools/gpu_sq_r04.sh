set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/sq_profile.sh r04 --no-extra --no-pipelined --steps 5 --warmup 2 || exit 1
cat gpurun_out/sq_r04.txt
