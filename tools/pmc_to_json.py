"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into profiles/pmc_latest.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (both reported in KiB): on gfx950 FETCH_SIZE counts
64 B per 128-B request of a wide streaming read, so it is doubled (MI355X_MICROARCH.md, HBM section).
usage: pmc_to_json.py FETCH_DIR WRITE_DIR N CT OUT.json
"""
import collections, csv, glob, json, os, sys


def load(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dc::", "").replace("dc64::", "")
                vals[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
n, ct = int(sys.argv[3]), int(sys.argv[4])
out = {"n": n, "ct": ct, "note": "HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KiB->B), rocprofv3 --pmc, "
       "separate passes", "fetch_bytes": {}, "write_bytes": {}, "hbm_bytes_per_launch": {}}
names = {"tile_fix_kernel": None, "tile_scan_kernel": None}
for k in sorted(set(fetch) | set(write)):
    f, w = 2.0 * fetch.get(k, 0.0), write.get(k, 0.0)
    out["fetch_bytes"][k] = round(f)
    out["write_bytes"][k] = round(w)
    out["hbm_bytes_per_launch"][k] = round(f + w)
json.dump(out, open(sys.argv[5], "w"), indent=1, sort_keys=True)
print(json.dumps(out["hbm_bytes_per_launch"], indent=1))
