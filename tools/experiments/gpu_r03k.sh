# r03k: parity + bench + decoder section timing + FETCH/WRITE per kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03k.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_codec.py tests/test_gpu_decode3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_k.log 2>&1 || { tail -30 gpurun_out/t_k.log; exit 1; }
tail -2 gpurun_out/t_k.log
timeout -k 10 300 python3 -u bench.py --no-cpu --no-pipelined --no-extra --steps 10 > gpurun_out/k_bench.json 2> gpurun_out/k_bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/k_bench.json').readline());print(d['value'],d['kernels_ms'])"
DCAMD_LIB=data-compression_amd/lib_p/libdcamd.so timeout -k 10 200 python3 -u tools/dec3_prof.py 7 26 1e-3 > gpurun_out/k_prof3.txt 2>&1 || exit $?
cat gpurun_out/k_prof3.txt
rm -rf gpurun_out/k_pmcf gpurun_out/k_pmcw
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/k_pmcf -o p -- python3 bench.py --no-cpu --no-pipelined --no-extra --steps 3 --warmup 1 > gpurun_out/k_pmcf.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/k_pmcw -o p -- python3 bench.py --no-cpu --no-pipelined --no-extra --steps 3 --warmup 1 > gpurun_out/k_pmcw.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections, glob
for d, c in (("gpurun_out/k_pmcf", "FETCH_SIZE"), ("gpurun_out/k_pmcw", "WRITE_SIZE")):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "dc::" in k and ("encode" in k or "3_kernel" in k):
            agg[k.split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(c, k, len(v), round(sum(v) / len(v) / 1024, 1), "MiB (raw KiB units / 1024)")
PY
