"""Debug: a shard whose first tokens are predictions, decoded by the segment decoder in shard mode."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch, dcamd
from pyoracle import Oracle
dc = dcamd.Lib(); dc.init(0); O = Oracle()
dc.set_bound(1e-3)
for ct in (5, 7):
    n = 1 << 16
    x = O.gen_u10(2 * n)
    x[n - 40:n + 40] = x[n - 41]
    _, xs = O.to_small(x)
    t, m17 = O.type_mask(xs)
    buf = torch.zeros(n + 4, dtype=torch.float32, device="cuda")
    buf[1:4] = torch.from_numpy(xs[n - 3:n].copy()); buf[4:] = torch.from_numpy(xs[n:].copy())
    cap = dc.stream_capacity(n)
    local = torch.zeros(cap + 64, dtype=torch.uint8, device="cuda")
    d_count = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    dc.encode_device(ct, buf[4:].data_ptr(), n, local.data_ptr(), idx0=n, type_=t, mask17=m17, start_bit=0, total_ptr=d_count.data_ptr())
    nb = dc.encode_result()
    print("ct", ct, "bits", nb, "first bytes", local[:16].cpu().numpy())
    s_all, _, _ = O.compress(ct, xs, 1e-3, t, m17)
    dec_all, _ = O.decompress(ct, s_all, 2 * n, 1e-3, t, m17)
    mb = (cap + 64) // 16 * 16
    dc.decode_status_clear()
    dc.decode_shard3_device(ct, local.data_ptr(), d_count.data_ptr(), mb, n, out.data_ptr(), t, m17, has_history=1)
    dc.synchronize()
    print(" after shard3 decode: status", hex(dc.decode_status()), "out[:6]", out[:6].cpu().numpy().view(np.uint32))
    hin = torch.from_numpy(dec_all[n - 3:n][::-1].copy()).cuda()
    torch.cuda.synchronize()
    dc.decode_shard3_fix(hin.data_ptr())
    dc.synchronize()
    o = out.cpu().numpy()
    bad = np.nonzero(o.view(np.uint32) != dec_all[n:].view(np.uint32))[0]
    print(" after fix: status", hex(dc.decode_status()), "mismatches", bad.size, bad[:10], "out", o[:4].view(np.uint32), "ref", dec_all[n:n+4].view(np.uint32))
    # the plain (non-shard) path for comparison
    dc.decode_status_clear()
