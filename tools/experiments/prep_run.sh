set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_prep.py tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prep or encode_sub or med or to_small or roundtrip" > gpurun_out/prep_t.log 2>&1 || { tail -40 gpurun_out/prep_t.log; exit 1; }
tail -2 gpurun_out/prep_t.log
timeout -k 10 200 python3 -u tools/prep_chain_time.py 20 24 26 2>&1 | grep -v amdgpu.ids | tee gpurun_out/prep_chain.txt
