set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for ct in 5 7; do timeout -k 10 120 python3 -u tools/dbg_runs.py $ct || exit 1; done
