"""Back-to-back encodes of 2^26 U10 CT7 (the bench's stream) with the encoder's helping instantiation
(DC_ENC_HELP=1; a DC_HELP_POLLS=0 build helps at every unpublished state): where does a stream differ from the
first?  Prints the first differing word, its tile (by the first stream's tile offsets from dc_encode_bits... the
word index * 32 / ~80k bits per tile) and how many words differ."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd
L = dcamd.Lib(); L.init(0); L.set_bound(1e-3)
L.L.dc_set_encode_help(1)
n = 1 << 26
xh = dcamd.gen_u10(n); xh = xh - xh.min()
x = torch.from_numpy(np.ascontiguousarray(xh, np.float32)).cuda()
cap = L.stream_capacity(n)
first = torch.zeros(cap, dtype=torch.uint8, device="cuda")
st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
mean, t = L.med_device(x.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
L.encode_device(7, x.data_ptr(), n, first.data_ptr(), type_=t, mask17=m17)
nbits = L.encode_result(); nb = (nbits + 7) // 8
bad = 0
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 48):
    st.zero_(); torch.cuda.synchronize()
    L.encode_device(7, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
    L.synchronize()
    nb2 = L.encode_result()
    a = first[:nb].view(torch.int32) if nb % 4 == 0 else first[:nb // 4 * 4].view(torch.int32)
    b = st[:a.numel() * 4].view(torch.int32)
    d = (a != b).nonzero().flatten()
    if d.numel() or nb2 != nbits:
        bad += 1
        w = int(d[0]) if d.numel() else -1
        print(f"rep {r}: nbits {nb2} vs {nbits}; {d.numel()} words differ, first at word {w} (bit {32 * w}, "
              f"~tile {32 * w * 4096 // nbits * n // 4096 // n if w >= 0 else -1}); words around: "
              f"{[hex(int(v) & 0xFFFFFFFF) for v in a[max(w - 1, 0):w + 2].cpu()]} vs "
              f"{[hex(int(v) & 0xFFFFFFFF) for v in b[max(w - 1, 0):w + 2].cpu()]}", flush=True)
print(f"{bad} of the reps differ; status {L.encode_status()}", flush=True)
