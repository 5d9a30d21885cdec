"""Section timing of the segment decoder (DC_DEC3_PROF build): where do parse3/decode3 spend their cycles?
Usage on the GPU box: DCAMD_LIB=data-compression_amd/lib_p/libdcamd.so python3 tools/dec3_prof.py [ct] [log2n] [bound]
[kind: u10 | ramp | sine | normal (the slowly-synchronising streams of tools/experiments/sync_kinds.py)] [maps]"""
import ctypes
import os
import sys
import time
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "data-compression_amd"))
import bench  # noqa: E402
import dcamd  # noqa: E402


def main():
    ct = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    log2n = int(sys.argv[2]) if len(sys.argv) > 2 else 26
    bound = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-3
    reps = 10
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    L = dcamd.Lib()
    L.init(0)
    C = types.SimpleNamespace(L=L, dev=dev, rank=0, dist=None, dcamd=dcamd)
    kind = sys.argv[4] if len(sys.argv) > 4 else "u10"
    if len(sys.argv) > 5 and sys.argv[5] == "maps":
        L.L.dc_set_decode3_maps(1)
    if kind == "u10":
        W = bench.prepare(C, ct, "u10", log2n, bound)
    else:
        n = 1 << log2n
        i = np.arange(n, dtype=np.float64)
        xh = {"sine": lambda: np.sin(i * 1e-3) * 50.0 + np.sin(i * 0.37) * 0.5,
              "normal": lambda: np.random.default_rng(1).standard_normal(n),
              "ramp": lambda: i * 1e-4 + np.random.default_rng(2).random(n) * 1e-2}[kind]().astype(np.float32)
        xs = torch.from_numpy(xh - xh.min()).to(dev)
        L.set_bound(bound)
        mean, t = L.med_device(xs.data_ptr(), n)
        W = {"n": n, "xs": xs, "type": t, "mask17": int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)}
    n = W["n"]
    cap = L.stream_capacity(n)
    stream = torch.empty(cap, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    d_nbits = torch.zeros(1, dtype=torch.int64, device=dev)
    L.encode_device(ct, W["xs"].data_ptr(), n, stream.data_ptr(), type_=W["type"], mask17=W["mask17"],
                    total_ptr=d_nbits.data_ptr())
    rd = L.L.dc_dec3_prof_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 32)()

    def dec():
        L.decode_device(ct, stream.data_ptr(), -1, n, out.data_ptr(), type_=W["type"], mask17=W["mask17"],
                        d_nbits=d_nbits.data_ptr(), max_bytes=cap)
        L.decode_finish()

    dec()
    assert rd(buf, 1) == 0, "not a DC_DEC3_PROF build"
    L.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dec()
    L.synchronize()
    wall = (time.perf_counter() - t0) / reps
    assert rd(buf, 1) == 0
    p = [v / reps for v in buf]
    nbits = int(d_nbits.item())
    print(f"ct {ct} n 2^{log2n} bound {bound} stream {nbits / 8e6:.1f} MB ({nbits / n:.2f} bits/value) "
          f"v3 {L.last_decode_was_v3()} maps {L.L.dc_last_decode_used_maps()} wall {wall * 1e3:.3f} ms/decode")
    pj, dj = max(p[5], 1), max(p[13], 1)
    print(f"parse: jobs {p[5]:.0f} tokens {p[4]:.0f} repair rounds {p[3]:.0f}")
    print(f"  per job (kcycles): main {p[0] / pj / 1e3:.1f} link wait {p[1] / pj / 1e3:.1f} repair {p[2] / pj / 1e3:.1f}")
    print(f"  per token per lane-walk (cycles): {p[0] / max(p[4] / 64, 1):.1f}")
    print(f"  repair walks: {p[6] / max(p[3], 1) / 1e3:.1f} kcycles and {p[7] / max(p[3], 1):.2f} lines per round; "
          f"max per job over {reps} decodes (kcycles): "
          f"total {buf[16] / 1e3:.1f} main {buf[17] / 1e3:.1f} links {buf[18] / 1e3:.1f}")
    print(f"decode: jobs {p[13]:.0f} tokens {p[15]:.0f} pending lanes {p[14]:.0f}")
    print(f"  per job (kcycles): claim {p[8] / dj / 1e3:.2f} stage {p[9] / dj / 1e3:.2f} walk {p[10] / dj / 1e3:.2f} "
          f"pend {p[11] / dj / 1e3:.2f} store {p[12] / dj / 1e3:.2f}")
    print(f"  walk cycles per token step: {p[10] / max(p[15] / 64, 1):.1f}")
    spec = np.array([v for v in out[:8].cpu().numpy()])
    print("first values", spec)


if __name__ == "__main__":
    main()
