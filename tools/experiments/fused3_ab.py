"""The single-launch parse + decode (fused3_kernel, DC_FUSED3) against parse3 + decode3 on the bench's workload
(CT7, U10 2^k after toSmallDataset, med mask, bound 1e-3): decode time per step (HIP events on the library
stream, 20 back-to-back decodes), bit-exactness against the two-launch output, and the fused kernel's phase
stamps (DC_FUSED3_STAMPS=1 must be set in the environment): per fused job the parse, prefix wait and decode
times, and when the jobs' phases run on the device's timeline.

usage: DC_FUSED3_STAMPS=1 python3 tools/experiments/fused3_ab.py [lg=26] [ct=7] [enc]   (enc: an encode before
every decode, as the bench's step)"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd

L = dcamd.Lib(); L.init(0)
L.set_bound(1e-3)
lg = int(sys.argv[1]) if len(sys.argv) > 1 else 26
ct = int(sys.argv[2]) if len(sys.argv) > 2 else 7
n = 1 << lg
xh = dcamd.gen_u10(n)
xh = xh - xh.min()
x = torch.from_numpy(np.ascontiguousarray(xh, np.float32)).cuda()
cap = L.stream_capacity(n)
st = torch.zeros(cap, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
mean, t = L.med_device(x.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
L.encode_device(ct, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
nbits = L.encode_result()
nb = (nbits + 7) // 8
ls = torch.cuda.ExternalStream(L.L.dc_get_stream())
L.set_decode3_seg(16)


ENC = "enc" in sys.argv[3:]          # re-encode before every decode (the bench's step: the stream fresh)
MODE = 2 if "dyn" in sys.argv[3:] else 1   # dyn: fused3d_kernel (dynamic decode jobs)
if "seg20" in sys.argv[3:]:
    L.set_decode3_seg(20)


def run(fused, K=20):
    L.set_fused3(fused)
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    for _ in range(3):
        L.decode_device(ct, st.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
        L.decode_finish()
    torch.cuda.synchronize()
    L.decode_status_clear()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for k in range(K):
        if ENC:
            L.encode_device(ct, x.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17)
        ev[k][0].record(ls)
        L.decode_device(ct, st.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
        ev[k][1].record(ls)
    torch.cuda.synchronize()
    e0, e1 = ev[0][0], ev[-1][1]
    per = float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1000
    stv = L.decode_status()
    L.decode_status_clear()
    out.fill_(-7.0)
    torch.cuda.synchronize()
    L.decode_device(ct, st.data_ptr(), nb, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
    L.decode_finish()
    torch.cuda.synchronize()
    return per, stv, L.L.dc_last_decode_was_v3(), out


us2, s2, v2, ref = run(0)
print(f"2^{lg} ct{ct}: parse3 + decode3 {us2:.1f} us per decode, status 0x{s2:x}, v3 {v2}", flush=True)
us1, s1, v1, out = run(MODE)
print(f"2^{lg} ct{ct}: {'fused3d_kernel' if MODE == 2 else 'fused3_kernel'}   {us1:.1f} us per decode, status 0x{s1:x}, v3 {v1}, "
      f"bit-exact vs two launches {bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))}", flush=True)
us2b, _, _, _ = run(0)
print(f"2^{lg} ct{ct}: parse3 + decode3 again {us2b:.1f} us", flush=True)
nfj = 1 << 20
L.set_fused3(MODE)
L.decode_device(ct, st.data_ptr(), nb, n, ref.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
L.decode_finish()
S = L.fused3_stamps(nfj).astype(np.int64)
L.set_fused3(0)
print(f"fused segment length {L.L.dc_fused3_last_seg()} chunks", flush=True)
if MODE == 2:                                     # per wave: start, parse end, decode end
    S = S[S[:, 2] > 0]
    t0 = S[:, 0].min()
    par, dec, end = (S[:, 1] - S[:, 0]) * 0.01, (S[:, 2] - S[:, 1]) * 0.01, (S[:, 2] - t0) * 0.01
    print(f"waves {len(S)}: parse {par.mean():.1f} us (min {par.min():.1f}, max {par.max():.1f}), decode "
          f"{dec.mean():.1f} (min {dec.min():.1f}, max {dec.max():.1f}); wave end min {end.min():.1f} "
          f"median {np.median(end):.1f} max {end.max():.1f} us", flush=True)
    sys.exit(0)
used = S[:, 3] > 0
S = S[used]
if len(S):
    t0 = S[:, 0].min()
    us = lambda v: v * 0.01                                   # 100 MHz ticks -> us
    par, pre, dec = us(S[:, 1] - S[:, 0]), us(S[:, 2] - S[:, 1]), us(S[:, 3] - S[:, 2])
    print(f"fused jobs {len(S)}: parse {par.mean():.1f} us (min {par.min():.1f}, max {par.max():.1f}), "
          f"prefix wait {pre.mean():.2f} (max {pre.max():.1f}), decode {dec.mean():.1f} (min {dec.min():.1f}, "
          f"max {dec.max():.1f})", flush=True)
    end = us(S[:, 3] - t0)
    start = us(S[:, 0] - t0)
    print(f"timeline: last job start {start.max():.1f} us, first job end {end.min():.1f}, last end {end.max():.1f}; "
          f"jobs starting after 10 us: {(start > 10).sum()}", flush=True)
    # how much of the timeline had parse and decode phases running together
    edges = np.linspace(0, end.max(), 21)
    rows = []
    for a, b in zip(edges[:-1], edges[1:]):
        np_ = ((us(S[:, 0] - t0) < b) & (us(S[:, 1] - t0) > a)).sum()
        nd_ = ((us(S[:, 2] - t0) < b) & (us(S[:, 3] - t0) > a)).sum()
        rows.append(f"{a:6.1f}-{b:6.1f} us: parsing {np_:5d} decoding {nd_:5d}")
    print("jobs in each phase over the launch (workgroups):\n  " + "\n  ".join(rows), flush=True)
