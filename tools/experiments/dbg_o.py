"""r03o debug: which decline bit does the segment decoder set on u10 100003 (CT5, 1e-3)?"""
import os, sys
os.environ["DC_DEBUG_ERR"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import dcamd
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0); O = Oracle()
L.set_decode3_min_bytes(0)
for n in (1 << 20, 100003, 65537, 262143):
    for ct in (5, 7):
        L.set_bound(1e-3)
        x = O.gen_u10(n)
        _, xs = O.to_small(x)
        t, m17 = O.type_mask(xs)
        s, nb, pos = L.compress(ct, xs, t, m17)
        out = L.decompress(ct, s, n, t, m17)
        print(n, ct, "v3" if L.last_decode_was_v3() else "declined", flush=True)
