"""med_dataset_float on the device (dcamd.Lib.med_device: chunk sums, scan, transducers, compose) at 2^k U10
after toSmallDataset: wall time per call (synchronous), and the result against the CPU oracle's serial sum."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch, dcamd
from pyoracle import Oracle
L = dcamd.Lib(); L.init(0); O = Oracle()
for lg in [int(a) for a in (sys.argv[1:] or ["20", "24", "26"])]:
    n = 1 << lg
    _, xs = O.to_small(dcamd.gen_u10(n))
    ref_mean, ref_t = O.med(xs)
    x = torch.from_numpy(xs).cuda()
    torch.cuda.synchronize()
    for _ in range(3):
        mean, t = L.med_device(x.data_ptr(), n)
    K = 10
    t0 = time.perf_counter()
    for _ in range(K):
        mean, t = L.med_device(x.data_ptr(), n)
    dt = (time.perf_counter() - t0) / K
    ok = np.float32(mean).view(np.uint32) == np.float32(ref_mean).view(np.uint32) and t == ref_t
    print(f"2^{lg}: med_dataset_float {dt * 1e3:.3f} ms per call (synchronous), exact {ok}", flush=True)
