"""The bitmask chain's pre-passes + encode on the device (impl/pingpong.c:148-209: toSmallDataset_float,
med_dataset_float of data_small, the mask, myCompress_bitwise_mask of data_small), 2^k U10 floats already in HBM:
  separate -- dc_to_small_device (min + x - min written) + dc_med_device + dc_encode_device
  fused    -- dc_prep_device (min and the mean of x - min, x - min never written) + dc_encode_sub_device
wall time per chain (each call synchronous as the library makes it, the encode waited for), both streams compared
with each other and the minimum / mean / stream with the CPU oracle's.  usage: prep_chain_time.py [lg...]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch, dcamd
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0); L.set_bound(1e-3); O = Oracle()
for lg in [int(a) for a in (sys.argv[1:] or ["26"])]:
    n = 1 << lg
    xh = dcamd.gen_u10(n) - np.float32(3.5)
    x = torch.from_numpy(xh).cuda()
    y = torch.empty_like(x)
    cap = L.stream_capacity(n)
    s1 = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    s2 = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def separate():
        mn = L.to_small_device(x.data_ptr(), n, y.data_ptr())
        mean, t = L.med_device(y.data_ptr(), n)
        m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
        L.encode_device(7, y.data_ptr(), n, s1.data_ptr(), type_=t, mask17=m17)
        return mn, mean, t, L.encode_result()

    def fused():
        mn, mean, t = L.prep_device(x.data_ptr(), n)
        m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
        L.encode_sub_device(7, x.data_ptr(), n, mn, s2.data_ptr(), type_=t, mask17=m17)
        return mn, mean, t, L.encode_result()

    res = {}
    for name, f in (("separate", separate), ("fused", fused)):
        for _ in range(3):
            r = f()
        K = 10
        t0 = time.perf_counter()
        for _ in range(K):
            r = f()
        res[name] = ((time.perf_counter() - t0) / K * 1e3, r)
    (ts, rs), (tf, rf) = res["separate"], res["fused"]
    nb = (rs[3] + 7) // 8
    same = rs == rf and torch.equal(s1[:nb], s2[:nb])
    line = f"2^{lg}: separate {ts:.3f} ms, fused {tf:.3f} ms per chain (min + mean + encode); streams equal {same}"
    if lg <= 24:
        omn, oxs = O.to_small(xh)
        om, ot = O.med(oxs)
        so, nbo, _ = O.compress(7, oxs, 1e-3, ot, O.mask17(om))
        line += f"; oracle equal {bool(rf[0] == omn and rf[1] == om and rf[2] == ot and nbo == nb and np.array_equal(s2[:nb].cpu().numpy(), so))}"
    print(line, flush=True)
