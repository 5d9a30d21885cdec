"""Per-kernel averages of SQ counters from rocprofv3 --pmc passes (tools/sq_profile.sh).

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over waves; WAIT_ANY +
WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots).
usage: sq_summary.py DIR [DIR ...]
"""
import collections, csv, glob, os, sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dc::", "")
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    c = {n: sum(v) / len(v) for n, v in vals[k].items()}
    print(k)
    for n in sorted(c):
        print(f"  {n:24s} {c[n]:16.0f}")
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA"):
            if n in c:
                print(f"  {n + ' / WAVE_CYCLES':40s} {c[n] / wc:.3f}")
    if c.get("SQ_WAVES"):
        w = c["SQ_WAVES"]
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES"):
            if n in c:
                print(f"  {n + ' per wave':40s} {c[n] / w:.1f}")
