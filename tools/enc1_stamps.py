"""Phase stamps of the encoder pack kernel (DC_DEBUG_STAMPS=1): per-phase durations and start spread.
Usage on the GPU box: DC_DEBUG_STAMPS=1 python3 tools/enc1_stamps.py [ct] [log2n]"""
import ctypes
import os
import sys
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
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    L = dcamd.Lib()
    L.init(0)
    C = types.SimpleNamespace(L=L, dev=dev, rank=0, dist=None, dcamd=dcamd)
    W = bench.prepare(C, ct, "u10", log2n, 1e-3)
    n = W["n"]
    stream = torch.empty(L.stream_capacity(n), dtype=torch.uint8, device=dev)
    nb = torch.zeros(1, dtype=torch.int64, device=dev)
    for _ in range(3):
        L.encode_device(ct, W["xs"].data_ptr(), n, stream.data_ptr(), type_=W["type"], mask17=W["mask17"],
                        total_ptr=nb.data_ptr())
    L.synchronize()
    buf = (ctypes.c_ulonglong * (8192 * 8))()
    assert L.L.dc_debug_enc_stamps(buf, 8192 * 8) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8).astype(np.int64)
    nt = min(8192, (n + 4095) // 4096)
    a = a[:nt, :5]
    t0 = a[:, 0].min()
    d = np.diff(a, axis=1) * 10.0 / 1000.0     # 100 MHz ticks -> us
    names = ["load+lengths", "scan+pack", "merge+sync", "store"]
    for i, nm in enumerate(names):
        print(f"{nm:12s} mean {d[:, i].mean():7.2f} us  p50 {np.median(d[:, i]):7.2f}  p99 {np.percentile(d[:, i], 99):7.2f}  max {d[:, i].max():7.2f}")
    st = (a[:, 0] - t0) * 0.01
    en = (a[:, 4] - t0) * 0.01
    print(f"tiles {nt}: start span {st.max():.1f} us, end span {en.max():.1f} us, mean tile {(en - st).mean():.2f} us")
    for q in range(0, nt, nt // 16):
        print(f"  tile {q:5d}: start {st[q]:7.1f} end {en[q]:7.1f}")


if __name__ == "__main__":
    main()
