"""Debug: the halo M-size plane (ct 5, k = 128) through the small-stream decoder vs the oracle."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, "..", "data-compression_amd"))
import dcamd  # noqa: E402
from pyoracle import Oracle  # noqa: E402

dc = dcamd.Lib()
dc.init(0)
O = Oracle()
dc.set_bound(1e-3)
ct = int(sys.argv[1]) if len(sys.argv) > 1 else 5
mi, mj, mk = 129, 129, 131
imax, jmax, kmax = 128, 128, 130
ijk, v = 3, 128
ii = np.arange(mi, dtype=np.float32)[:, None, None]
rs = np.random.RandomState(ijk * 1000 + v)
p = (ii * ii / np.float32((imax - 1) * (imax - 1)) + np.zeros((mi, mj, mk), np.float32)).astype(np.float32)
p += (rs.rand(mi, mj, mk).astype(np.float32) * np.float32(0.01))
A, B = imax, jmax
a, b = np.meshgrid(np.arange(A), np.arange(B), indexing="ij")
plane = p[(a, b, v)].reshape(-1).copy()
mn, xs = O.to_small(plane)
t, m17 = O.type_mask(xs)
s, nb, pos = O.compress(ct, xs, 1e-3, t, m17)
n = xs.size
spec, _ = O.decompress(ct, s, n, 1e-3, t, m17)
print("n", n, "bytes", nb, "chunks", (nb * 8 + 255) // 256)
for label, rmax in (("runs", 1 << 30), ("default", -2)):
    old = dc.set_runs_max_bytes(rmax)
    ds = torch.from_numpy(np.concatenate([s, np.zeros(64, np.uint8)])).cuda()
    out = torch.zeros(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    dc.decode_device(ct, ds.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17)
    st = dc.decode_status()
    dc.decode_finish()
    got = out.cpu().numpy()
    bad = np.flatnonzero(got.view(np.uint32) != spec.view(np.uint32))
    print(label, "runs" if dc.last_decode_was_runs() else "", "status", hex(st), "mismatches", bad.size, bad[:20])
    if bad.size:
        k = bad[0]
        print("  got ", got[max(k - 4, 0):k + 6])
        print("  want", spec[max(k - 4, 0):k + 6])
    dc.set_runs_max_bytes(old)
