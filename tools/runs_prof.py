"""Section stamps of runs_scan_kernel (DC_RUNS_PROF build), for the Himeno plane stream and 2^12 U10."""
import ctypes
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
dc.set_runs_max_bytes(1 << 30)
rd = dc.L.dc_runs_prof_read
rd.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 16)()
for name, x in (("himeno", np.tile(O.gen_himeno_plane(256, 256), 1)), ("u10 2^12", O.gen_u10(1 << 12)),
                ("u10 2^14", O.gen_u10(1 << 14))):
    _, xs = O.to_small(x)
    t, m17 = O.type_mask(xs)
    ct = 5
    s, nb, pos = O.compress(ct, xs, 1e-3, t, m17)
    ds = torch.from_numpy(np.concatenate([s, np.zeros(64, np.uint8)])).cuda()
    out = torch.zeros(xs.size, dtype=torch.float32, device="cuda")
    for _ in range(3):
        dc.decode_device(ct, ds.data_ptr(), nb, xs.size, out.data_ptr(), type_=t, mask17=m17)
        dc.decode_finish()
    assert rd(ctypes.addressof(buf)) == 0
    st = [buf[k] for k in range(7)]
    d = [(st[k + 1] - st[k]) / 100.0 for k in range(6)]     # s_memrealtime: 100 MHz -> us
    print(f"{name}: bytes {nb} runs {dc.last_decode_was_runs()} sections (us): maps {d[0]:.2f} mapscan {d[1]:.2f} "
          f"stage {d[2]:.2f} entries+counts {d[3]:.2f} pass1 {d[4]:.2f} carryscan {d[5]:.2f} total {(st[6]-st[0])/100:.2f}")
