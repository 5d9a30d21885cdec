"""Large-input parity sweep of the double codecs (GPU vs oracle): inputs with many pending prefixes
(ramp: '110' chains, runs: '101' copies) and mixed data, 2^log2n doubles, CT 5/6/7/11."""
import os, sys, time, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import dcamd
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0); O = Oracle()
n = 1 << int(sys.argv[1]); bound = 1e-3
L.set_bound(bound)
rs = np.random.RandomState(2)
cases = {"ramp": 0.37 * np.arange(n, dtype=np.float64),
         "runs": np.repeat(rs.rand(n // 1000 + 1) * 7.0, 1000)[:n],
         "mixed": np.concatenate([O.gen_u10_64(n // 4), np.full(n // 4, 2.5), np.arange(n // 4) * 1e-4, rs.rand(n - 3 * (n // 4)) * 1e9])}
bad = 0
for name, x in cases.items():
    mn, xs = O.to_small64(x); mean, t = O.med64(xs); m20 = O.mask20(mean)
    for ct in (5, 6, 7, 11):
        t0 = time.time()
        s, nb, pos = L.compress64(ct, xs, t, m20)
        d = L.decompress64(ct, s, n, t, m20)
        fl = int(L.L.dc64_last_decode_flags())
        so, nbo, _ = O.compress64(ct, xs, bound, t, m20)
        ref, _ = O.decompress64(ct, so, n, bound, t, m20)
        ok = nb == nbo and np.array_equal(s, so) and np.array_equal(d.view(np.uint64), ref.view(np.uint64))
        bad += not ok
        print(f"{name} ct{ct} n={n} bytes={nb} flags={fl} ok={ok} ({time.time() - t0:.1f}s)", flush=True)
print("BAD", bad)
sys.exit(1 if bad else 0)
