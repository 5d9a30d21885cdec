"""Diagnostic (not a test): back-to-back encodes of 2^26 U10 CT7, where do repeats differ from the first."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd
L = dcamd.Lib(); L.init(0); L.set_bound(1e-3)
n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
if os.environ.get("DBG_ORACLE"):
    sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
    from pyoracle import Oracle
    from test_gpu_fullsize import _u10
    O = Oracle()
    _, xs = O.to_small(_u10(O, n))
    x = torch.from_numpy(xs).cuda()
else:
    x = torch.from_numpy(dcamd.gen_u10(n)).cuda()
cap = L.stream_capacity(n)
first = torch.zeros(cap, dtype=torch.uint8, device="cuda")
st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
mean, t = L.med_device(x.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
L.encode_device(7, x.data_ptr(), n, first.data_ptr(), type_=t, mask17=m17)
nb0 = L.encode_result()
print("first bits", nb0, "status", L.encode_status(), flush=True)
f = first.cpu().numpy()
nrep = int(sys.argv[2]) if len(sys.argv) > 2 else 24
for rep in range(nrep):
    st.zero_()
    torch.cuda.synchronize()
    L.encode_device(7, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
    L.synchronize()
    nb = nb0
    if torch.equal(st[:(nb0 + 7) // 8], first[:(nb0 + 7) // 8]):
        if rep % 50 == 0:
            print(f"rep {rep}: same", flush=True)
        continue
    s = st.cpu().numpy()
    nbyte = (nb0 + 7) // 8
    d = np.nonzero(s[:nbyte] != f[:nbyte])[0]
    if d.size:
        w = d // 4
        brk = np.nonzero(np.diff(d) > 64)[0]
        runs = [(int(d[0]), int(d[brk[0]] if brk.size else d[-1]))]
        for q in range(len(brk)):
            runs.append((int(d[brk[q] + 1]), int(d[brk[q + 1]] if q + 1 < len(brk) else d[-1])))
        print(f"rep {rep}: status {L.encode_status()} differ {d.size} bytes in {len(runs)} runs {runs[:8]}, "
              f"zero-bytes-in-diff {int((s[d] == 0).sum())}", flush=True)
        for (a0, a1) in runs[:4]:
            hb = a0 * 8
            lo, hi = 0, (n + 4095) // 4096          # prefix bits of tiles [0, k): the encode of x[:4096 k]
            pb = lambda k: 0 if k == 0 else L.encode_bits(7, x.data_ptr(), 4096 * k, 0, t, m17)
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if pb(mid) <= hb:
                    lo = mid
                else:
                    hi = mid
            b0, b1 = pb(lo), pb(lo + 1)
            print(f"   hole bytes {a0}..{a1}: tile {lo}, tile bits [{b0}, {b1}) = {(b1 - b0) / 32:.1f} words, "
                  f"hole at word {(hb - b0) / 32:.1f} .. {((a1 + 1) * 8 - b0) / 32:.1f} of the tile", flush=True)
    elif rep % 10 == 0:
        print(f"rep {rep}: same", flush=True)
