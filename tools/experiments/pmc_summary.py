"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (diagnostic helper).
usage: pmc_summary.py DIR [DIR ...]   (each DIR holds one pass' *counter_collection.csv)"""
import collections, csv, glob, os, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, {c: round(sum(x) / len(x)) for c, x in sorted(v.items())})
