"""Phase stamps of the one-workgroup decoder (a DC_TY_STAMPS build: DCAMD_LIB=...), 2^14 U10 CT7 @1e-3: start, stream
loaded, walked, linked (rounds), scanned, values, pending (rounds), stored -- s_memrealtime (100 MHz)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch, dcamd
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0); L.set_bound(1e-3); O = Oracle()
n = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 14
xs = O.to_small(O.gen_u10(n))[1]
t, m17 = O.type_mask(xs)
s, nb, pos = L.compress(7, xs, t, m17)
st = torch.zeros(L.stream_capacity(n), dtype=torch.uint8, device="cuda")
st[:nb] = torch.from_numpy(s).cuda()
out = torch.empty(n, dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
for rep in range(5):
    L.check(L.L.dc_decode_device(7, ctypes.c_void_p(st.data_ptr()), ctypes.c_longlong(nb), None,
                                 ctypes.c_longlong(L.stream_capacity(n)), ctypes.c_longlong(n), t, m17,
                                 ctypes.c_void_p(out.data_ptr())), "decode")
    L.check(L.L.dc_decode_finish(), "finish")
    h = (ctypes.c_ulonglong * 16)()
    L.L.dc_tiny_stamps(h)
    a = np.array(h[:16], np.int64)
    d = (a[1:7] - a[0:6]) / 100.0
    print("tiny:", dict(zip(["load", "walk", "links", "scan", "values", "pend+store"], d.round(2))),
          "link rounds", a[10], "pending rounds", a[11], "total us", (a[6] - a[0]) / 100.0,
          "was_tiny", L.L.dc_last_decode_was_tiny(), flush=True)
