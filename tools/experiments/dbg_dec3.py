"""Debug one golden case through the segment decoder (diagnostic)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
torch.zeros(1, device="cuda")
import dcamd
from pyoracle import Oracle
from conftest import golden
L = dcamd.Lib(); L.init(0); O = Oracle()
bound = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-6
case = sys.argv[2] if len(sys.argv) > 2 else "u10_16k"
ct = int(sys.argv[3]) if len(sys.argv) > 3 else 7
g = golden(bound)
L.set_bound(bound)
s = g[f"{case}/ct{ct}/stream"]; n = g[f"{case}/input"].size
t, m17 = int(g[f"{case}/type"]), int(g[f"{case}/mask17"])
spec, got = O.decompress(ct, s, n, bound, t, m17)
for thr in (-1, 0):
    L.set_decode3_min_bytes(thr)
    out = L.decompress(ct, s, n, t, m17)
    bad = np.nonzero(out.view(np.uint32) != spec.view(np.uint32))[0]
    print(f"thr {thr}: v3={L.last_decode_was_v3()} nbytes={s.size} n={n} type={t} m17={m17:#x} mismatches={bad.size}",
          "first:", bad[:10], "last:", bad[-5:] if bad.size else [])
    if bad.size:
        for i in bad[:6]:
            print(f"  [{i}] got {out.view(np.uint32)[i]:#010x} want {spec.view(np.uint32)[i]:#010x}")
