"""FETCH_SIZE calibration factors from a `rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib` run.

usage: fetch_calib.py PMC_DIR BYTES_JSON_LINE_FILE OUT.json
Factor = bytes the kernel read / FETCH_SIZE bytes (KiB x 1024) of its last dispatch.  The guide's
calibrated case (16 B per lane, consecutive) should read 2.0 on gfx950; pmc_to_json.py applies each
codec kernel's own pattern factor instead of the blanket 2."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, bfile, out = sys.argv[1], sys.argv[2], sys.argv[3]
    last = {}
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        rows = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE":
                name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
                rows[name].append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"]) * 1024.0))
        for k, v in rows.items():
            last[k] = sorted(v)[-1][1]
    bytes_ = None
    for line in open(bfile):
        if line.startswith("{"):
            bytes_ = json.loads(line)["bytes"]
    res = {"source": "tools/fetch_calib.hip under rocprofv3 --pmc FETCH_SIZE (1 GiB, every byte read once)",
           "fetch_bytes": {k: round(v) for k, v in last.items()}, "bytes": bytes_, "factor": {}}
    for k, b in bytes_.items():
        if last.get(k):
            res["factor"][k] = round(b / last[k], 4)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res["factor"]))


if __name__ == "__main__":
    main()
