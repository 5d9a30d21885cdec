"""Diagnostic (not a test): every golden case through the library vs the oracle; prints mismatches."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch
torch.zeros(1, device="cuda")
import dcamd
from conftest import BOUNDS, CASES, golden
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0)
orc = Oracle()
bad = 0
for bound in BOUNDS:
    g = golden(bound)
    L.set_bound(bound)
    for case in CASES:
        for ct in [5, 6, 7, 11]:
            s = g[f"{case}/ct{ct}/stream"]; n = g[f"{case}/input"].size
            t, m17 = int(g[f"{case}/type"]), int(g[f"{case}/mask17"])
            out = L.decompress(ct, s, n, t, m17)
            spec, got = orc.decompress(ct, s, n, bound, t, m17)
            d = np.nonzero(out.view(np.uint32) != spec.view(np.uint32))[0]
            if d.size:
                bad += 1
                print(f"MISMATCH {bound} {case} ct{ct} n={n} bytes={s.size} first={d[0]} count={d.size} last={d[-1]}",
                      out[d[0]:d[0]+4], spec[d[0]:d[0]+4], flush=True)
print("bad", bad)
