# r03l: SQ counters of the codec kernels (separate --pmc passes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "tools/gpu_r03l.sh $(date -u +%FT%TZ)" >> gpurun_out/script_log.txt
B="--no-cpu --no-pipelined --no-extra --steps 3 --warmup 1"
rm -rf gpurun_out/l_sq1 gpurun_out/l_sq2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY -f csv -d gpurun_out/l_sq1 -o p -- python3 bench.py $B > gpurun_out/l_sq1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_WAVE32_LDS GRBM_GUI_ACTIVE -f csv -d gpurun_out/l_sq2 -o p -- python3 bench.py $B > gpurun_out/l_sq2.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections, glob
for d in ("gpurun_out/l_sq1", "gpurun_out/l_sq2"):
    fs = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not fs:
        print("no csv in", d); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"]
        if "dc::" in k and ("encode" in k or "3_kernel" in k):
            agg[k.split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        print(k, {c: round(sum(v) / len(v)) for c, v in cs.items()})
PY
