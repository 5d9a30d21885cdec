"""Benchmark: CT7 (bitmask bit-wise) compress+decompress of U10 float32 at absErrorBound=1e-3.

Metric (BASELINE.json): GB/s of input float bytes, 4N / (t_compress + t_decompress), whole job over all
ranks (weak scaling: every rank owns a contiguous 2^26-float block of one global U10 array and runs the
hot path on it; inputs are resident in HBM before the timed region).  `--gpus N` without a launcher
starts N ranks under torch.distributed.run itself.

A step = dc_encode_device (count / scan / write kernels) + dc_decode_device (parse / tile fix / tile scan /
decode kernels) of the rank's block, on the library's HIP stream.  The decoder's fast-path status word
is read after the timed steps; a nonzero status (some step needed an exact slow path, which is not in
the timed region) makes the run exit non-zero.  Rank 0 prints ONE JSON line with:
  roofline      the dominant kernel: algorithmic bytes / its average HIP-event duration on the library
                stream; traffic = PMC HBM bytes from profiles/pmc_latest.json (labelled, not this run)
  pipelined     the same K steps with encode k+1 on its own HIP stream overlapping decode k (beside value)
  end_to_end    N>1: + bit-count all-gather, shard placement, RCCL all-gather of the shard streams into the
                single global stream and the per-rank shard decode with the 12-byte history exchange
  sweep/configs N=1: the north_star size sweep (2^14..2^28) and BASELINE configs 2 / 3 / 5, few steps each
  cpu_baseline  N=1: the reference's own impl/dataCompression.c (oracle/_ref, else the C restatement)
                on one host core, on a bounded sample of the same workload
`--check` compares the GPU stream with the oracle's stream and the GPU decode with the oracle's decode.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
GOLDEN_HASHES = os.path.join(ROOT, "tests", "golden", "bench_hashes.json")


def golden_entry(ct, kind, log2n, bound, world):
    """The oracle's hashes for this workload (tests/golden/make_bench_hashes.py), or None."""
    try:
        g = json.load(open(GOLDEN_HASHES))
    except (OSError, ValueError):
        return None
    return g.get(f"ct{ct}_{kind}_2^{log2n}_{bound:g}_w{world}")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--log2n", type=int, default=26, help="floats per GPU (2^log2n)")
    ap.add_argument("--ct", type=int, default=7)
    ap.add_argument("--bound", type=float, default=1e-3)
    ap.add_argument("--input", default="u10", choices=["u10", "eq"])
    ap.add_argument("--cpu-log2n", type=int, default=24, help="cpu_baseline sample size (2^k floats, ~10 s of CPU)")
    ap.add_argument("--no-extra", action="store_true", help="skip the size sweep and the other BASELINE configs (N=1)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end multi-GPU curve (N>1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify the round trip against the oracle")
    ap.add_argument("--halo", action="store_true",
                    help="BASELINE configs[3]: Himeno L-size z-halo planes (256x256 of p[257][257][k]) per rank, "
                         "fused device halo encode + decode, CT from --ct (config: 5)")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the second pass that times the same K steps pipelined (encode of step k+1 on its own "
                         "HIP stream while step k decodes), reported under 'pipelined'; value is always the "
                         "back-to-back number")
    ap.add_argument("--f64", action="store_true",
                    help="the double codecs (myCompress/myDecompress_bitwise_double*, k-means/mm/lu payloads): "
                         "compress+decompress of 2^log2n U10 doubles per GPU, CT from --ct")
    ap.add_argument("--ber", type=float, default=0.0,
                    help="CT9 flow (BASELINE configs[4]): CRC-32 of the CT7 stream, floor(bits*BER) real bit flips on "
                         "the received copy, CRC check, resend, decode -- all inside the timed step")
    return ap.parse_args()


def gen_input(kind, n, offset):
    import dcamd
    if kind == "u10":
        return dcamd.gen_u10(n, 42, offset)
    return np.full(n, np.float32(0.123456789), np.float32)


def cpu_baseline(ct, bound, n, kind):
    """Time the reference CPU codec on a bounded sample (1 host core, single-threaded)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    x = gen_input(kind, n, 0)
    O = pyoracle.Oracle()
    mn, xs = O.to_small(x)
    mean, t = O.med(xs)
    m17 = O.mask17(mean)
    try:
        R = pyoracle.RefLib(bound)
        t0 = time.perf_counter()
        s, nb, pos = R.compress(ct, xs, t, m17)
        t1 = time.perf_counter()
        R.decompress(ct, s, n, t, m17)
        t2 = time.perf_counter()
        kind_s = "reference"
    except (FileNotFoundError, OSError):
        t0 = time.perf_counter()
        s, nb, pos = O.compress(ct, xs, bound, t, m17)
        t1 = time.perf_counter()
        O.decompress(ct, s, n, bound, t, m17)
        t2 = time.perf_counter()
        kind_s = "port"
    gbs = 4.0 * n / (t2 - t0) / 1e9
    return {"value": round(gbs, 6), "unit": "GB/s", "cores": 1, "kind": kind_s,
            "sample": f"{kind.upper()} 2^{int(np.log2(n))} floats CT{ct} @{bound:g}: compress {t1 - t0:.3f} s + "
                      f"decompress {t2 - t1:.3f} s, single-threaded impl/dataCompression.c"
                      + (" (compiled reference)" if kind_s == "reference" else " restatement (oracle)")}


def halo_bench(args):
    """Himeno halo exchange payload (impl/himenoBMTxps.c:644-706): every Jacobi iteration each rank
    compresses its two z-halo planes (k = 1 and k = kmax - 2 of p[257][257][kk], 65,536 floats each)
    and decompresses the two it receives.  Here a step = encode + decode of both planes on this
    rank's GPU through the fused device path (no MPI; the planes are independent streams)."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        # RCCL over xGMI; DC_BENCH_BACKEND=gloo rehearses the multi-rank path with several ranks per GPU
        dist.init_process_group(os.environ.get("DC_BENCH_BACKEND", "nccl"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import dcamd
    L = dcamd.Lib()
    L.init(local)
    L.set_bound(args.bound)
    mi, mj, mk = 257, 257, 8                       # L-size i/j extent; a thin z slab per rank
    imax, jmax, kmax = 256, 256, 7
    ii = torch.arange(mi, dtype=torch.float32, device=dev).view(mi, 1, 1)
    kk3 = torch.arange(mk, dtype=torch.float32, device=dev).view(1, 1, mk)

    def field(r):
        # initmt's p = i^2 / (imax-1)^2 (it = 0), offset per rank and plane so that a swapped direction
        # or a wrong plane in the exchange cannot pass the check below
        return (ii * ii / float((imax - 1) * (imax - 1)) + 0.25 * r + 0.01 * kk3).expand(mi, mj, mk).contiguous()

    p = field(rank)
    q = torch.zeros_like(p)
    n = imax * jmax
    cap = L.stream_capacity(n)
    st = [torch.zeros(cap, dtype=torch.uint8, device=dev) for _ in range(2)]
    bits = torch.zeros(2, dtype=torch.int64, device=dev)
    mins = torch.zeros(2, dtype=torch.float32, device=dev)
    ct = args.ct if args.ct != 7 else 5
    planes = [1, kmax - 2]

    # several ranks: a non-periodic line of z-slabs (MPI_Cart as himenoBMTxps.c); each rank sends plane k = 1
    # down and k = kmax - 2 up, and decodes what it receives into k = kmax - 1 (from up) and k = 0 (from down)
    down = rank - 1 if rank > 0 else None
    up = rank + 1 if rank + 1 < world else None
    rmins = torch.zeros(2, dtype=torch.float32, device=dev)
    xfer = [0, 0]                                   # stream bytes this rank received, per step
    last = [None]                                   # the last step's received (stream, bits, min) per side

    # no host read inside a step: the planes' decoder status is read after the timed steps
    L.L.dc_set_halo_async(1)

    pair = os.environ.get("DC_HALO_PAIR", "1") != "0"            # decode both planes at once
    # one rank: the step recorded once into a HIP graph and replayed (DC_HALO_GRAPH=0: call by call); the planes
    # encoded at once on two streams (DC_HALO_EPAIR) pays inside the graph, not call by call
    use_graph = dist is None and os.environ.get("DC_HALO_GRAPH", "1") != "0"
    epair = os.environ.get("DC_HALO_EPAIR", "1" if use_graph else "0") == "1"

    def step():
        if epair:                                   # both planes at once (two streams)
            L.halo_encode2_device(ct, p.data_ptr(), (mi, mj, mk), 3, planes[0], planes[1], (imax, jmax, kmax),
                                  st[0].data_ptr(), st[1].data_ptr(), bits.data_ptr(), bits.data_ptr() + 8,
                                  mins.data_ptr(), mins.data_ptr() + 4)
        else:
            for h, v in enumerate(planes):
                L.halo_encode_device(ct, p.data_ptr(), (mi, mj, mk), 3, v, (imax, jmax, kmax), st[h].data_ptr(),
                                     bits.data_ptr() + 8 * h, mins.data_ptr() + 4 * h)
        if dist is None:
            # both planes at once (each on its own stream: the decoders are one-workgroup scans); DC_HALO_PAIR=0
            # decodes them one after the other
            if pair:
                L.halo_decode2_device(ct, st[0].data_ptr(), st[1].data_ptr(), bits.data_ptr(), bits.data_ptr() + 8, 0, 0,
                                      mins.data_ptr(), mins.data_ptr() + 4, q.data_ptr(), (mi, mj, mk), 3, planes[0],
                                      planes[1], (imax, jmax, kmax))
                return
            for h, v in enumerate(planes):
                L.halo_decode_device(ct, st[h].data_ptr(), -1, bits.data_ptr() + 8 * h, 0, 0, mins.data_ptr() + 4 * h,
                                     q.data_ptr(), (mi, mj, mk), 3, v, (imax, jmax, kmax))
            return
        L.synchronize()                             # the sizes leave first (impl/himenoBMTxps.c:648-670)
        nb, mn = bits.cpu().tolist(), mins.cpu().tolist()
        got = dcamd.halo_exchange(st, nb, mn, down, up)
        last[0] = (got, nb, mn)
        for i, rec in enumerate(got):
            if rec is not None:
                rmins[i] = rec[2]
        torch.cuda.synchronize()                    # received bytes / minima land on torch's streams, the
        for i, (rec, kk) in enumerate(zip(got, (kmax - 1, 0))):   # decoder runs on the library's own
            if rec is None:
                continue
            rs, rb, rmn = rec
            xfer[i] = (rb + 7) // 8
            L.halo_decode_device(ct, rs.data_ptr(), (rb + 7) // 8, 0, 0, 0, rmins.data_ptr() + 4 * i,
                                 q.data_ptr(), (mi, mj, mk), 3, kk, (imax, jmax, kmax))

    torch.cuda.synchronize()                        # (the fills above run on torch's stream)
    for _ in range(max(args.warmup, 1)):
        step()
    L.synchronize()
    graph = None
    if use_graph:
        L.capture_begin()
        step()
        graph = L.capture_end()
        for _ in range(max(args.warmup, 1)):
            L.graph_launch(graph)
        L.synchronize()
    run = (lambda: L.graph_launch(graph)) if graph is not None else step
    nbytes = [(int(b) + 7) // 8 for b in bits.cpu()]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    L.synchronize()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dstat = L.decode_status()
    estat = L.encode_status()
    L.L.dc_set_halo_async(0)
    if graph is not None:
        L.graph_destroy(graph)
    if dstat != 0 or estat != 0:
        print(f"bench.py: halo decoder status 0x{dstat:x}, encoder status 0x{estat:x} after the timed steps",
              file=sys.stderr)
        sys.exit(1)
    xcheck = None
    if dist is None:                                # the last (replayed) step's output = the calls issued directly
        got = (bits.clone(), mins.clone(), [s.clone() for s in st], q[:, :, planes].clone())
        L.L.dc_set_halo_async(1)
        step()
        L.synchronize()
        L.L.dc_set_halo_async(0)
        xcheck = (torch.equal(got[0], bits) and torch.equal(got[1].view(torch.int32), mins.view(torch.int32)) and
                  all(torch.equal(a, b) for a, b in zip(got[2], st)) and
                  torch.equal(got[3].view(torch.int32), q[:, :, planes].view(torch.int32)))
    if dist is not None:
        # the plane received from up must be up's plane k = 1 and the one from down down's plane
        # k = kmax - 2 (each rank's field differs): encoded here from the neighbour's field, the same
        # bits, min and stream bytes, and the received halo decodes to the same plane
        got, nb, mn = last[0]
        q2 = torch.zeros_like(q)
        xcheck = True
        for rec, kk, src, h in zip(got, (kmax - 1, 0), (up, down), (0, 1)):
            if rec is None:
                continue
            rs, rb, rmn = rec
            pn = field(src)
            sn = torch.zeros(cap, dtype=torch.uint8, device=dev)
            bn = torch.zeros(1, dtype=torch.int64, device=dev)
            mnn = torch.zeros(1, dtype=torch.float32, device=dev)
            torch.cuda.synchronize()
            L.halo_encode_device(ct, pn.data_ptr(), (mi, mj, mk), 3, planes[h], (imax, jmax, kmax), sn.data_ptr(),
                                 bn.data_ptr(), mnn.data_ptr())
            L.synchronize()
            k = (rb + 7) // 8
            xcheck &= rb == int(bn.item()) and rmn == float(mnn.item()) and bool(torch.equal(rs[:k].cpu(), sn[:k].cpu()))
            L.halo_decode_device(ct, sn.data_ptr(), -1, bn.data_ptr(), 0, 0, mnn.data_ptr(),
                                 q2.data_ptr(), (mi, mj, mk), 3, kk, (imax, jmax, kmax))
            L.synchronize()
            xcheck &= bool(torch.equal(q[:imax, :jmax, kk], q2[:imax, :jmax, kk]))
    planes_cd = 2.0 * world                        # (encodes + decodes) / 2 per step, all ranks
    if dist is not None:
        w = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w[0])
        u = torch.tensor([(2 + (down is not None) + (up is not None)) / 2.0], dtype=torch.float64, device=dev)
        dist.all_reduce(u)                         # the end ranks of the line decode one plane
        planes_cd = float(u[0])
        c = torch.tensor([1.0 if xcheck else 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.MIN)
        xcheck = bool(c[0] > 0.5)
    res = {"metric": f"GB/s (halo plane float bytes) compress+decompress, Himeno L z-halos, CT={ct} "
                     f"absErrorBound={args.bound:g}",
           "value": round(planes_cd * 4.0 * n / (wall / args.steps) / 1e9, 4), "unit": "GB/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic Himeno initmt pressure field (p = i^2/(imax-1)^2, it = 0)",
           "config": {"workload": "Himeno L-size z-halo planes, 2 x 256x256 floats per rank per step, fused device "
                                  "plane gather + toSmallDataset + encode, decode + min scatter", "ct": ct,
                      "plane_floats": n, "stream_bytes": nbytes, "ratio": round(4.0 * n / max(nbytes[0], 1), 3),
                      "parallelism": f"dp{world}",
                      "launch": "one HIP graph per step" if graph is not None else "call by call",
                      "exchange": ("none (one rank: each plane decoded locally)" if dist is None else
                                   "z-neighbour exchange inside the timed step: sizes + min, then the stream bytes "
                                   f"(torch.distributed P2P, {dist.get_backend()}); rank 0 received {xfer} bytes"),
                      "exchange_check": xcheck}}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if xcheck is False:
        sys.exit("halo exchange check failed: a received plane differs from its sender's by more than the bound")


def f64_bench(args):
    """Double codecs (dc_f64.hip): a step = dc64_encode_device + dc64_decode_device of the rank's block of
    2^log2n U10 doubles already in HBM; toSmallDataset_double / med_dataset_double run once before."""
    import ctypes
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("DC_BENCH_BACKEND", "nccl"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import dcamd
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    L = dcamd.Lib()
    L.init(local)
    L.set_bound(args.bound)
    n = 1 << args.log2n
    ct = args.ct
    from pyoracle import Oracle
    O = Oracle()
    x = torch.from_numpy(O.gen_u10_64(n, 42, rank * n)).to(dev)
    xs = torch.empty_like(x)
    mn = ctypes.c_double(0)
    L.check(L.L.dc64_to_small_device(ctypes.c_void_p(x.data_ptr()), n, ctypes.c_void_p(xs.data_ptr()), ctypes.byref(mn)),
            "dc64_to_small_device")
    mean, typ = ctypes.c_double(0), ctypes.c_int(0)
    t_med0 = time.perf_counter()
    L.check(L.L.dc64_med_device(ctypes.c_void_p(xs.data_ptr()), n, ctypes.byref(mean), ctypes.byref(typ)), "dc64_med_device")
    t_med = time.perf_counter() - t_med0
    typ = typ.value
    mask20 = int(np.array([mean.value], np.float64).view(np.uint64)[0] >> 44)
    cap = int(L.L.dc64_stream_capacity(n))
    stream = torch.empty(cap, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.float64, device=dev)
    d_nbits = torch.zeros(1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ext = torch.cuda.ExternalStream(L.L.dc_get_stream())

    def step(ev=None):
        if ev:
            ev[0].record(ext)
        L.encode64_device(ct, xs.data_ptr(), n, stream.data_ptr(), typ, mask20, total_ptr=d_nbits.data_ptr())
        if ev:
            ev[1].record(ext)
        L.decode64_device(ct, stream.data_ptr(), -1, n, out.data_ptr(), typ, mask20, d_nbits=d_nbits.data_ptr(),
                          max_bytes=cap)
        if ev:
            ev[2].record(ext)

    for _ in range(max(args.warmup, 1)):
        step()
    flags = L.decode64_finish()
    nbytes = (L.encode64_result() + 7) // 8
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    L.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    L.synchronize()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    flags |= L.decode64_finish()
    if dist is not None:
        w = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w[0])
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    ok = None
    if args.check and rank == 0:
        s_h = stream[:nbytes].cpu().numpy()
        so, nbo, _ = O.compress64(ct, xs.cpu().numpy(), args.bound, typ, mask20)
        ref, _ = O.decompress64(ct, so, n, args.bound, typ, mask20)
        ok = bool(nbo == nbytes and np.array_equal(s_h, so) and
                  np.array_equal(out.cpu().numpy().view(np.uint64), ref.view(np.uint64)))
    res = {"metric": f"GB/s (input double bytes) compress+decompress, double CT={ct} absErrorBound={args.bound:g}",
           "value": round(world * 8.0 * n / (wall / args.steps) / 1e9, 3), "unit": "GB/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic U10 doubles (counter-based splitmix64, 53-bit uniform [0,10), seed 42), generated per rank",
           "config": {"workload": f"double CT{ct} bit-wise compress+decompress, U10 2^{args.log2n} float64 per GPU, "
                                  f"absErrorBound={args.bound:g}", "doubles_per_gpu": n, "ct": ct,
                      "stream_bytes": int(nbytes), "ratio": round(8.0 * n / nbytes, 4), "type": typ,
                      "mask20": f"{mask20:05x}", "parallelism": f"dp{world}", "exact_fallback": bool(flags & 1)},
           "phases_ms": {"encode": round(enc_ms, 4), "decode": round(dec_ms, 4), "med_dataset_double_s": round(t_med, 4)}}
    # roofline of the dominant phase (decode: stream in, doubles out), HIP events on the library stream
    dbytes = float(nbytes) + 8.0 * n
    dach = dbytes / (dec_ms * 1e-3) / 1e9 if dec_ms > 0 else 0.0
    res["roofline"] = {"bound": "hbm", "kernel": "double decode (all launches of dc64_decode_device)",
                       "achieved": round(dach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(dach / HBM_PEAK_GBS, 4), "traffic": None,
                       "algorithmic_bytes_per_launch": int(dbytes), "avg_launch_ms": round(dec_ms, 4)}
    if ok is not None:
        res["check_vs_oracle"] = ok
    if rank == 0 and not args.no_cpu:
        R = None
        try:
            from pyoracle import RefLib
            R = RefLib(args.bound)
        except (FileNotFoundError, OSError):
            pass
        m = 1 << args.cpu_log2n
        xh = np.ascontiguousarray(xs[:m].cpu().numpy())
        t0 = time.perf_counter()
        s, nb, _ = R.compress64(ct, xh, typ, mask20) if R else O.compress64(ct, xh, args.bound, typ, mask20)
        t1 = time.perf_counter()
        R.decompress64(ct, s, m, typ, mask20) if R else O.decompress64(ct, s, m, args.bound, typ, mask20)
        t2 = time.perf_counter()
        res["cpu_baseline"] = {"value": round(8.0 * m / (t2 - t0) / 1e9, 6), "unit": "GB/s", "cores": 1,
                               "kind": "reference" if R else "port",
                               "sample": f"U10 2^{args.cpu_log2n} doubles CT{ct}: compress {t1 - t0:.3f} s + decompress "
                                         f"{t2 - t1:.3f} s, single-threaded impl/dataCompression.c"
                                         + (" (compiled reference)" if R else " restatement (oracle)")}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def spawn_ranks(args):
    """`bench.py --gpus N` outside a launcher: start N ranks under torch.distributed.run as a child
    process (this process touches no GPU, so no exec after GPU initialisation) and exit with its code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


class Ctx:
    """Per-process state of a float-codec run: torch device, library, optional process group."""

    def __init__(self):
        import torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
        # several ranks on one GPU (the gloo rehearsal).  Until r05 they encoded with the wait-free three-launch
        # variant: a single-pass tile could wait past its bound for a predecessor left undispatched behind another
        # process's waiting waves.  Since r06 a tile computes a late predecessor's count itself (dc_encode.hip
        # enc_lookback's help: the helping instantiation, selected below), so every rank keeps the single pass
        # (DC_ENC_PASSES still selects another)
        self.shared_gpu = self.world > max(torch.cuda.device_count(), 1)
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            torch.cuda.set_device(self.local)
            # RCCL over xGMI; DC_BENCH_BACKEND=gloo rehearses the multi-rank path with several ranks per GPU
            dist.init_process_group(os.environ.get("DC_BENCH_BACKEND", "nccl"))
            self.dist = dist
        self.dev = torch.device("cuda", self.local)
        torch.cuda.set_device(self.dev)
        import dcamd
        self.dcamd = dcamd
        self.L = dcamd.Lib()
        self.L.init(self.local)
        if self.shared_gpu:             # ranks share a GPU: the encoder's helping instantiation
            self.L.L.dc_set_encode_help(1)

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, v):
        if self.dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])


def prepare(C, ct, kind, log2n, bound):
    """This rank's contiguous block of one global array (+3-float predictor halo) in HBM, toSmallDataset
    over the global array and the CT7 type / mask from the exact global sequential mean (all outside
    the timed region, like the reference apps' pre-passes, impl/pingpong.c:128-209)."""
    import ctypes
    import torch
    L, dev, rank = C.L, C.dev, C.rank
    L.set_bound(bound)
    n = 1 << log2n
    xh = gen_input(kind, n + 3, rank * n - 3) if rank > 0 else np.concatenate(
        [np.zeros(3, np.float32), gen_input(kind, n, 0)])
    x_all = torch.from_numpy(xh).to(dev)
    del xh
    xs_all = torch.empty(n + 4, dtype=torch.float32, device=dev)
    xs = xs_all[4:]                                  # 16-byte aligned shard start
    mnc = ctypes.c_float(0)
    L.check(L.L.dc_to_small_device(ctypes.c_void_p(x_all[3:].data_ptr()), n, ctypes.c_void_p(xs.data_ptr()),
                                   ctypes.byref(mnc)), "to_small")
    L.synchronize()
    if C.dist is not None:      # toSmallDataset over the global array: global min, then x - min (halo too)
        gm = torch.tensor([mnc.value], dtype=torch.float32, device=dev)
        C.dist.all_reduce(gm, op=C.dist.ReduceOp.MIN)
        torch.sub(x_all, gm[0], out=xs_all[1:])
        torch.cuda.synchronize()
    del x_all
    t_med0 = time.perf_counter()
    if C.dist is None:
        mean, typ = L.med_device(xs.data_ptr(), n)
    else:
        mean, typ = C.dcamd.global_med(L, xs.data_ptr(), n, dev)
    t_med = time.perf_counter() - t_med0
    mask17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
    return {"n": n, "xs": xs, "xs_all": xs_all, "type": typ, "mask17": mask17, "t_med": t_med, "ct": ct,
            "kind": kind, "log2n": log2n, "bound": bound}


def run_codec(C, W, steps, warmup, pipelined=False, ber=0.0, check=False):
    """Time `steps` back-to-back steps (encode + decode of the rank's block on the library stream).
    The decoder's fast-path status word is read after the timed steps (it is OR-ed over every decode):
    a nonzero value means some step left the fast path, whose exact slow paths are not in the timed
    region -- reported as fast_path: false (the main metric exits non-zero on it)."""
    import ctypes
    import torch
    L, dev = C.L, C.dev
    n, ct, typ, mask17, xs = W["n"], W["ct"], W["type"], W["mask17"], W["xs"]
    cap = L.stream_capacity(n)
    stream = torch.empty(cap, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    d_nbits = torch.zeros(1, dtype=torch.int64, device=dev)
    ext = torch.cuda.ExternalStream(L.L.dc_get_stream())
    idx0 = C.rank * n

    slow = [False]                # the stream needs the decoder's exact slow path: finish inside the step

    def step(ev=None):
        if ev:
            ev[0].record(ext)
        L.encode_device(ct, xs.data_ptr(), n, stream.data_ptr(), idx0=idx0, type_=typ, mask17=mask17,
                        total_ptr=d_nbits.data_ptr())
        if ev:
            ev[1].record(ext)
        L.decode_device(ct, stream.data_ptr(), -1, n, out.data_ptr(), type_=typ, mask17=mask17,
                        d_nbits=d_nbits.data_ptr(), max_bytes=cap)
        if slow[0]:
            L.decode_finish()                         # the exact slow path, timed (host-synchronised)
        if ev:
            ev[2].record(ext)

    torch.cuda.synchronize()
    warm_status = 0
    for _ in range(max(warmup, 1)):
        step()
        warm_status |= L.decode_status()
        L.decode_finish()                             # completes a slow path if one was needed
    slow[0] = warm_status != 0
    nbits = L.encode_result()
    nbytes = (nbits + 7) // 8

    # CT9 flow (--ber): sender CRC, channel copy with floor(bits*BER) flipped bits, receiver CRC check, resend
    # of the clean stream on a mismatch, CRC check of the resent copy, decode of the received copy.  The
    # sender's CRC comes out of the encoder (dc_encode_crc_device: its tiles CRC the words they store), the
    # receiver's check of the resent copy out of the resend copy itself (dc_crc_resend_crc_device): one CRC
    # pass per step, the receiver's check of the damaged copy.  Checks and resend run on the device (no host
    # round trip inside the step); the host reads each step's counters (resends, mismatches left)
    # asynchronously as the protocol's ack and checks them after the loop.  The stream length is the
    # warm-up's (same input every step).
    resends = [0]
    ct9 = {}
    if ber > 0:
        rcv = torch.empty(cap, dtype=torch.uint8, device=dev)
        d_crc = torch.zeros(2, dtype=torch.int32, device=dev)
        d_cnt = torch.zeros(2, dtype=torch.int32, device=dev)
        nflip = int(nbits * ber)
        seed = [1]
        acks = []
        ack_buf = torch.zeros((max(steps, warmup) + 1, 2), dtype=torch.int32, pin_memory=True)
        # DC_CT9_MODE: "copy" (default) the send as a copy pass that CRCs what it sends (dc_crc32_copy_device) and
        # a receiver pass; "send" the encoder writes its stream into the receiver's buffer as well (the channel,
        # dc_encode_send_device) and one pass CRCs both copies after the damage (dc_crc32_pair_device);
        # "fused" (or DC_CT9_FUSED=1) the sender's CRC inside the encoder's tiles (slower).
        # Each phase carries its algorithmic bytes in stream sizes: a copy pass reads and writes the stream (2),
        # a CRC pass reads it (1), the pair pass reads both copies (2), flips and launch gaps move nothing (0)
        ct9_mode = "fused" if os.environ.get("DC_CT9_FUSED", "0") == "1" else os.environ.get("DC_CT9_MODE", "copy")
        CT9_PHASES = {
            "fused": [("crcf_final_kernel (sender CRC: combine of the encoder's block CRCs)", 0), ("channel copy", 2),
                      ("flip_bits_kernel", 0), ("crcf_blocks + crcf_final (receiver CRC, damaged copy)", 1),
                      ("crc_blocks<copy> + crc_final2 (resend copy with its CRC + check)", 2)],
            "copy": [("(encode call beyond its kernel)", 0),
                     ("crc_blocks<copy> + crc_final2 (send: channel copy + sender CRC)", 2),
                     ("flip_bits_kernel", 0), ("crc_blocks + crc_final2 (receiver CRC, damaged copy)", 1),
                     ("crc_blocks<copy> + crc_final2 (resend copy with its CRC + check)", 2)],
            "send": [("(encode call beyond its kernel: the encoder also writes the receiver's copy)", 0),
                     ("(no send pass)", 0), ("flip_bits_kernel", 0),
                     ("crc_blocks x2 + crc_final2 x2 (sender's and receiver's CRC, one pass)", 2),
                     ("crc_blocks<copy> + crc_final2 (resend copy with its CRC + check)", 2)]}[ct9_mode]
        CT9_STREAMS = dict(CT9_PHASES)
        CT9_PHASES = [nm for nm, _ in CT9_PHASES]

        # Default: the send copies the stream into the receiver's buffer and CRCs the bytes it sends in one pass
        # (dc_crc32_copy_device), the receiver CRCs what arrived (dc_crc32_device_async), the resend copies and
        # CRCs in one pass (dc_crc_resend_crc_device).  DC_CT9_FUSED=1: the sender's CRC inside the encoder's
        # tiles and the receiver's by the 16 KiB-block kernels (dc_encode_crc_device, dc_crc32_stream_device),
        # which measured slower.
        fused_crc = ct9_mode == "fused"
        send_mode = ct9_mode == "send"

        def step(ev=None, ph=None):                          # noqa: F811 -- the CT9 variant of the step
            def mark(i):
                if ph is not None:
                    ph[i].record(ext)
            if ev:
                ev[0].record(ext)
            if fused_crc:
                L.encode_crc_device(ct, xs.data_ptr(), n, stream.data_ptr(), d_nbits.data_ptr(), d_crc.data_ptr(),
                                    idx0=idx0, type_=typ, mask17=mask17)
                mark(0)
                with torch.cuda.stream(ext):
                    rcv[:nbytes].copy_(stream[:nbytes])
            elif send_mode:
                # the send: the encoder writes the stream into the receiver's buffer too (no copy pass)
                L.encode_send_device(ct, xs.data_ptr(), n, stream.data_ptr(), rcv.data_ptr(), d_nbits.data_ptr(),
                                     idx0=idx0, type_=typ, mask17=mask17)
                mark(0)
            else:
                L.encode_device(ct, xs.data_ptr(), n, stream.data_ptr(), idx0=idx0, type_=typ, mask17=mask17,
                                total_ptr=d_nbits.data_ptr())
                mark(0)
                # the send: the channel copy, the sender's CRC of the bytes it sends computed in the same pass
                L.crc32_copy_device(stream.data_ptr(), rcv.data_ptr(), nbytes, d_crc.data_ptr())
            mark(1)
            L.flip_bits_device(rcv.data_ptr(), nbits, nflip, seed[0])
            seed[0] += nflip
            mark(2)
            if fused_crc:
                L.crc32_stream_device(rcv.data_ptr(), nbytes, d_crc.data_ptr() + 4)
            elif send_mode:                                  # the sender's CRC and the receiver's, one pass
                L.crc32_pair_device(stream.data_ptr(), rcv.data_ptr(), nbytes, d_crc.data_ptr(), d_crc.data_ptr() + 4)
            else:
                L.crc32_device_async(rcv.data_ptr(), nbytes, d_crc.data_ptr() + 4)
            mark(3)
            L.crc_resend_crc_device(d_crc.data_ptr(), stream.data_ptr(), rcv.data_ptr(), nbytes, d_cnt.data_ptr())
            mark(4)
            if ev:
                ev[1].record(ext)
            L.decode_device(ct, rcv.data_ptr(), nbytes, n, out.data_ptr(), type_=typ, mask17=mask17, max_bytes=cap)
            if ev:
                ev[2].record(ext)
            with torch.cuda.stream(ext):                     # the ack: this step's counters, copied async
                a = ack_buf[len(acks) % ack_buf.shape[0]]
                a.copy_(d_cnt, non_blocking=True)
                acks.append(a)

        for _ in range(warmup):
            step()
            L.decode_finish()
        L.synchronize()
        d_cnt.zero_()
        acks.clear()
        ct9 = {"d_cnt": d_cnt, "acks": acks, "phases": CT9_PHASES, "streams": CT9_STREAMS, "nflip": nflip}

    # ---- timed region: barrier + sync on both sides, max over ranks, nothing but the steps (an event
    # record between launches costs a few microseconds of dispatch gap)
    C.barrier()
    torch.cuda.synchronize()
    L.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step()
    L.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    C.barrier()
    enc_status = L.encode_status()                    # the encoder's error word over all timed encodes
    if enc_status:
        print(f"bench.py: encoder error word 0x{enc_status:x} after the timed steps", file=sys.stderr)
        sys.exit(1)
    status = L.decode_status()                        # OR over all timed decodes, no slow path run
    try:
        L.decode_finish()
    except C.dcamd.DCError:
        if status == 0:
            raise
    wall = C.max_over_ranks(t1 - t0)
    timed_resends = resends[0]
    if ber > 0:                                       # every step's ack: one resend (its damaged copy detected),
        acks = [a.numpy().copy() for a in ct9["acks"]]   # no mismatch left after it
        timed_resends = int(acks[-1][0]) if acks else 0
        ct9["acks_ok"] = all(int(a[0]) == k + 1 and int(a[1]) == 0 for k, a in enumerate(acks)) and len(acks) == steps
        ct9["d_cnt"].zero_()
        ct9["acks"].clear()
    # ---- the same steps again with per-kernel HIP events, recorded by the library on its own stream
    # (dc_timing_enable, one event set per step): the kernel table and the roofline's launch duration
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    phs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(steps)] if ber > 0 else None
    L.L.dc_timing_enable(steps)
    torch.cuda.synchronize()
    L.synchronize()
    for k in range(steps):
        if ber > 0:
            step(evs[k], phs[k])
        else:
            step(evs[k])
    L.synchronize()
    torch.cuda.synchronize()
    st2 = L.decode_status()
    try:
        L.decode_finish()
    except C.dcamd.DCError:
        if st2 == 0:
            raise
    status |= st2
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    kms = np.zeros((steps, 11), np.float32)
    for k in range(steps):
        buf = (ctypes.c_float * 11)()
        if L.L.dc_timing_read_all(k, buf) == 0:
            kms[k] = np.frombuffer(buf, np.float32)
    L.L.dc_timing_enable(0)
    kavg = kms.mean(axis=0)
    if ber > 0:                                       # the CT9 launches between encode and decode, per step
        ct9["phase_ms"] = {nm: float(np.mean([p[i - 1].elapsed_time(p[i]) for p in phs]))
                           for i, nm in enumerate(ct9["phases"]) if i > 0}
        # the sender's combine: the encode call's span less the encoder kernel's own (library event slot)
        ct9["phase_ms"][ct9["phases"][0]] = max(0.0, float(np.mean([e[0].elapsed_time(p[0]) for e, p in zip(evs, phs)]))
                                                - float(kavg[0]))
    # ---- self-check: poison the stream and the output, run one more step, and compare device hashes of
    # both with the oracle's (tests/golden/bench_hashes.json): a step that skipped work would leave poison
    stream.fill_(0xA5)
    out.view(torch.int32).fill_(-1)
    if ber > 0:
        rcv.fill_(0x5A)
    torch.cuda.synchronize()
    step()
    L.synchronize()
    chk_bits = L.encode_result()
    if L.decode_status():
        L.decode_finish()
    torch.cuda.synchronize()
    chk_bytes = (chk_bits + 7) // 8
    sc = {"stream_hash": f"{L.hash_device(stream.data_ptr(), chk_bytes):016x}",
          "out_hash": f"{L.hash_device(out.data_ptr(), 4 * n):016x}", "nbits": int(chk_bits)}
    if ber > 0:
        sc["received_hash"] = f"{L.hash_device(rcv.data_ptr(), chk_bytes):016x}"
    g = golden_entry(ct, W["kind"], W["log2n"], W["bound"], C.world)
    if g is not None and C.world > 1:
        g = dict(g["ranks"][C.rank], type=g["type"], mask17=g["mask17"])
    if g is None:
        sc["ok"] = None
        sc["golden"] = "none for this workload (tests/golden/make_bench_hashes.py)"
    else:
        ok = (int(g["nbits"]) == chk_bits and int(g["stream"]) == int(sc["stream_hash"], 16) and
              int(g["out"]) == int(sc["out_hash"], 16) and g["type"] == typ and g["mask17"] == f"{mask17:05x}")
        if ber > 0:
            ok &= int(g["stream"]) == int(sc["received_hash"], 16)
        sc["ok"] = bool(ok)
        sc["golden"] = ("tests/golden/bench_hashes.json: the oracle's stream and decode of this workload"
                        + (f" (rank {C.rank}'s shard)" if C.world > 1 else ""))
    res = {"nbits": int(nbits), "nbytes": int(nbytes), "wall": wall, "enc_ms": enc_ms, "dec_ms": dec_ms, "self_check": sc,
           "kavg": kavg, "status": int(status | warm_status), "warm_status": int(warm_status), "resends": timed_resends,
           "slow_path_timed": slow[0], "v3": bool(L.L.dc_last_decode_launched_v3()),
           "runs": bool(L.L.dc_last_decode_launched_runs()), "fused": bool(L.L.dc_decode3_last_fused()),
           "tiny": bool(L.L.dc_last_decode_launched_tiny()),
           "fused_seg": int(L.L.dc_fused3_last_seg()),
           "enc_mode": int(L.L.dc_encode_mode()), "ct9": {k: v for k, v in ct9.items() if k in ("phase_ms", "acks_ok", "nflip", "streams")}}

    if pipelined and ber <= 0:
        # the same K steps pipelined (encode k+1 || decode k, two stream buffers), reported beside value
        es = torch.cuda.Stream(device=dev)
        stream2 = [stream, torch.empty(cap, dtype=torch.uint8, device=dev)]
        nb2 = [d_nbits, torch.zeros(1, dtype=torch.int64, device=dev)]
        enc_done = [torch.cuda.Event() for _ in range(steps)]
        dec_done = [torch.cuda.Event() for _ in range(steps)]

        def enc(k):
            b = k & 1
            if k >= 2:
                es.wait_event(dec_done[k - 2])
            L.encode_device(ct, xs.data_ptr(), n, stream2[b].data_ptr(), idx0=idx0, type_=typ, mask17=mask17,
                            total_ptr=nb2[b].data_ptr())
            enc_done[k].record(es)

        def dec(k):
            b = k & 1
            ext.wait_event(enc_done[k])
            L.decode_device(ct, stream2[b].data_ptr(), -1, n, out.data_ptr(), type_=typ, mask17=mask17,
                            d_nbits=nb2[b].data_ptr(), max_bytes=cap)
            dec_done[k].record(ext)

        L.synchronize()
        torch.cuda.synchronize()
        C.barrier()
        L.check(L.L.dc_set_encode_stream(ctypes.c_void_p(es.cuda_stream)), "dc_set_encode_stream")
        p0 = time.perf_counter()
        enc(0)
        for k in range(steps):
            if k + 1 < steps:
                enc(k + 1)
            dec(k)
        L.synchronize()
        torch.cuda.synchronize()
        pw = C.max_over_ranks(time.perf_counter() - p0)
        L.L.dc_set_encode_stream(None)
        pst = L.decode_status()
        try:
            L.decode_finish()
        except C.dcamd.DCError:
            if pst == 0:
                raise
        res["pipelined"] = {"value": round(C.world * 4.0 * n / (pw / steps) / 1e9, 3),
                            "ms_per_step": round(pw / steps * 1e3, 4), "fast_path": pst == 0, "decoder_status": pst,
                            "encoder_status": int(L.encode_status()),
                            "how": "encode of step k+1 on its own HIP stream overlaps the decode of step k (two "
                                   "stream buffers); every step encodes and decodes the whole block"}
    if check and C.rank == 0:
        # the GPU stream against the oracle's stream (bytes, length, pos) and the GPU decode of it against
        # the oracle's decode, bit for bit
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from pyoracle import Oracle
        O = Oracle()
        s_h = stream[:nbytes].cpu().numpy()
        xh = xs.cpu().numpy() if C.world == 1 else None
        ok_s = None
        if xh is not None:
            so, nbo, poso = O.compress(ct, xh, W["bound"], typ, mask17)
            ok_s = bool(nbo == nbytes and np.array_equal(s_h, so))
            del so, xh
        ref, _ = O.decompress(ct, s_h, n, W["bound"], typ, mask17)
        ok_d = bool(np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32)))
        res["check"] = {"stream_vs_oracle": ok_s, "decode_vs_oracle": ok_d}
    del stream, out
    return res


COPY_VARIANTS = ["4 x 16 B per lane in flight, default policy", "4 x 16 B per lane, nontemporal",
                 "8 x 16 B per lane, default policy", "8 x 16 B per lane, nontemporal"]


def copy_bandwidth(L, dev, n, reps=10):
    """Achievable HBM rate on this GPU: the best of four hand-written streaming copies (dc_copy_rate_device:
    16-byte buffer loads and stores, the guide's float4 copy) of n floats, read + written bytes over the
    average HIP-event launch time on the library stream."""
    import torch
    a = torch.ones(n, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    torch.cuda.synchronize()
    gbs, v = L.copy_rate(a.data_ptr(), b.data_ptr(), 4 * n, reps)
    del a, b
    return gbs, COPY_VARIANTS[v]


def kernel_table(ct, n, nbytes, kavg, v3=True, enc_mode=1, runs=False, fused=False, tiny=False):
    """The timed launches of a step (library timing slots, HIP events on the library stream) and their
    algorithmic bytes: the encoder's count and pack launches (the pack's workgroup 0 scans the tile
    offsets), then the decoder's -- the segment decoder (parse3, whose jobs check the
    link into them, and decode3, which sums the parse jobs' totals itself: no scan launch) or the
    chunk-map decoder (parse, tile fix + scan, decode) -- and, when the first decoder handed the stream
    over inside the step (dc_decode_finish), the chunk-map decoder's launches and the runs-mode resolve
    and resolved decode.  The decode bytes go to the launch whose values were kept."""
    k = [float(v) for v in kavg]
    fin = any(v > 0 for v in k[6:11])
    res = k[9] > 0
    dec_b = nbytes + 4.0 * n
    if enc_mode == 1:     # the single-pass encoder: one launch reads x once and writes the stream
        kernels = {f"encode_fused_kernel<{ct}>": (k[0], 4.0 * n + nbytes)}
    else:
        kernels = {   # name: (avg ms, algorithmic bytes per launch)
            f"encode_count_kernel<{ct}>": (k[0], 4.0 * n),
            f"encode_pack_kernel<{ct}>": (k[2], 4.0 * n + nbytes),
        }
    if tiny:              # the one-workgroup decoder of small streams: the stream read once, the floats written
        kernels.update({f"tiny_decode_kernel<{ct}>": (k[3] + k[5], 0.0 if fin else dec_b)})
    elif runs:            # the small-stream decoder: chunk maps + one-workgroup scans, then the values
        kernels.update({f"runs_map_kernel<{ct}>+runs_scan_kernel<{ct}>": (k[3], 0.0 if fin else float(nbytes)),
                        f"runs_values_kernel<{ct}>": (k[5], 0.0 if fin else dec_b)})
    elif v3 and fused:    # the single-launch parse + decode: the stream read once, the floats written
        kernels.update({f"fused3_kernel<{ct}>": (k[3] + k[5], 0.0 if fin else dec_b)})
    elif v3:
        kernels.update({f"parse3_kernel<{ct}>": (k[3], 0.0 if fin else float(nbytes)),
                        f"decode3_kernel<{ct}>": (k[5], 0.0 if fin else dec_b)})
    else:
        kernels.update({f"parse_kernel<{ct}>": (k[3], 0.0 if fin else float(nbytes)),
                        "tile_fix_kernel+tile_scan_kernel": (k[4], 0.0),
                        f"decode_kernel_fast<{ct}>": (k[5], 0.0 if fin else dec_b)})
    if fin:
        kernels.update({f"parse_kernel<{ct}> (finish)": (k[6], float(nbytes)),
                        "tile_fix_kernel+tile_scan_kernel (finish)": (k[7], 0.0),
                        f"decode_kernel_fast<{ct}> (finish)": (k[8], 0.0 if res else dec_b)})
    if res:
        kernels.update({"resolve_kernel": (k[9], 0.0),
                        f"decode_kernel_fast<{ct}> (resolved)": (k[10], dec_b)})
    return kernels


def ct9_bytes(name, nbytes, streams):
    """Algorithmic bytes of a CT9 phase: its stream count (CT9_PHASES: a copy pass 2, a CRC pass 1, the pair pass
    2, the flips and the launch gaps 0) times the stream's bytes."""
    return float(streams.get(name, 0)) * nbytes


def line_for(C, W, R, steps):
    """Summary of one configuration: value (GB/s of input floats, all ranks), roofline of the dominant
    kernel (algorithmic bytes / its HIP-event duration on the library stream) and of the whole step."""
    n, nbytes = W["n"], R["nbytes"]
    ms = R["wall"] / steps * 1e3
    kernels = kernel_table(W["ct"], n, nbytes, R["kavg"], R["v3"], R.get("enc_mode", 1), R.get("runs", False),
                           R.get("fused", False), R.get("tiny", False))
    for nm, ms_ in R.get("ct9", {}).get("phase_ms", {}).items():   # CT9: every launch of the step
        kernels[nm] = (ms_, ct9_bytes(nm, nbytes, R["ct9"].get("streams", {})))
    dname = max(kernels, key=lambda k: kernels[k][0])
    dms, dbytes = kernels[dname]
    ach = dbytes / (dms * 1e-3) / 1e9 if dms > 0 else 0.0
    step_bytes = 8.0 * n + 2 * nbytes
    return {"value": round(C.world * 4.0 * n / (ms * 1e-3) / 1e9, 3), "ms_per_step": round(ms, 4),
            "stream_bytes": int(nbytes), "ratio": round(4.0 * n / max(nbytes, 1), 4), "fast_path": R["status"] == 0,
            "decoder_status": R["status"],
            **({"fused_segment_chunks": R["fused_seg"]} if R.get("fused") else {}),
            "slow_path_in_timed_step": bool(R.get("slow_path_timed", False)),
            "dominant": {"kernel": dname, "avg_launch_ms": round(dms, 4), "achieved_GBs": round(ach, 1),
                         "frac": round(ach / HBM_PEAK_GBS, 4)},
            "kernels_sum_ms": round(sum(v[0] for v in kernels.values()), 4),
            "step_roofline_frac": round(step_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "kernels_ms": {k: round(v[0], 4) for k, v in kernels.items()}}


def prepass_chain(C, log2n, bound, reps=5):
    """The bitmask chain's pre-passes + encode (impl/pingpong.c:148-209: toSmallDataset_float, med_dataset_float of
    data_small, the mask, myCompress_bitwise_mask of data_small) on the raw U10 input in HBM, wall time per chain
    (outside the bench's timed step, like the reference apps' pre-passes): `separate` = dc_to_small_device (x - min
    written) + dc_med_device + dc_encode_device, `fused` = dc_prep_device (x - min never written) +
    dc_encode_sub_device.  The fused chain's stream hash is checked against the oracle's for the main workload."""
    import torch
    L, dev = C.L, C.dev
    L.set_bound(bound)
    n = 1 << log2n
    x = torch.from_numpy(gen_input("u10", n, 0)).to(dev)
    y = torch.empty_like(x)
    cap = L.stream_capacity(n)
    s1 = torch.zeros(cap, dtype=torch.uint8, device=dev)
    s2 = torch.zeros(cap, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def mask(mean):
        return int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)

    def separate():
        mn = L.to_small_device(x.data_ptr(), n, y.data_ptr())
        mean, t = L.med_device(y.data_ptr(), n)
        L.encode_device(7, y.data_ptr(), n, s1.data_ptr(), type_=t, mask17=mask(mean))
        return float(mn), float(mean), t, L.encode_result()

    def fused():
        mn, mean, t = L.prep_device(x.data_ptr(), n)
        L.encode_sub_device(7, x.data_ptr(), n, mn, s2.data_ptr(), type_=t, mask17=mask(mean))
        return float(mn), float(mean), t, L.encode_result()

    out = {}
    for name, f in (("separate", separate), ("fused", fused)):
        f()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = f()
        out[name] = (round((time.perf_counter() - t0) / reps * 1e3, 4), r)
    bits = out["fused"][1][3]
    g = golden_entry(7, "u10", log2n, bound, 1)
    sh = L.hash_device(s2.data_ptr(), (bits + 7) // 8)
    res = {"separate_ms": out["separate"][0], "fused_ms": out["fused"][0],
           "same_results": out["separate"][1] == out["fused"][1] and bool(torch.equal(s1[:(bits + 7) // 8], s2[:(bits + 7) // 8])),
           "self_check": None if g is None else (int(g["nbits"]) == bits and int(g["stream"]) == sh),
           "workload": f"CT7 U10 2^{log2n} raw input, bound {bound:g}: min + mean of x - min + mask + encode"}
    del x, y, s1, s2
    torch.cuda.empty_cache()
    return res


def side_config(C, ct, kind, log2n, steps, warmup, bound, ber=0.0):
    """A BASELINE config / sweep point on this GPU (N=1): prepared, timed, summarised, freed."""
    import torch
    W = prepare(C, ct, kind, log2n, bound)
    R = run_codec(C, W, steps, warmup, ber=ber)
    out = line_for(C, W, R, steps)
    out.update({"ct": ct, "input": kind, "floats": W["n"], "type": W["type"], "mask17": f"{W['mask17']:05x}",
                "self_check": R["self_check"]["ok"]})
    if ber > 0:
        out.update({"ber": ber, "flips_per_step": int(R["nbits"] * ber), "resends": R["resends"],
                    "detected_all": R["resends"] == steps and bool(R["ct9"].get("acks_ok"))})
    del W
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    if args.halo:
        return halo_bench(args)
    if args.f64:
        return f64_bench(args)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        sys.exit(2)
    C = Ctx()
    ct = args.ct
    W = prepare(C, ct, args.input, args.log2n, args.bound)
    R = run_codec(C, W, args.steps, args.warmup, pipelined=not args.no_pipelined, ber=args.ber, check=args.check)
    n, nbytes = W["n"], R["nbytes"]
    main_line = line_for(C, W, R, args.steps)
    if R["status"] != 0 and not R["slow_path_timed"]:
        # a timed step left the decoder's fast path: its exact slow path ran outside the timed region,
        # so the time is not the codec's -- refuse to report it (streams that need the slow path from the
        # warm-up on run it inside every timed step and are reported with fast_path false)
        print(f"bench.py: decoder status 0x{R['status']:x} in the timed steps (slow path not timed)", file=sys.stderr)
        sys.exit(1)
    kernels = kernel_table(ct, n, nbytes, R["kavg"], R["v3"], R.get("enc_mode", 1), R.get("runs", False),
                           R.get("fused", False), R.get("tiny", False))
    for nm, ms_ in R.get("ct9", {}).get("phase_ms", {}).items():   # (as line_for: the CT9 launches too)
        kernels[nm] = (ms_, ct9_bytes(nm, nbytes, R["ct9"].get("streams", {})))
    dname = main_line["dominant"]["kernel"]
    achievable, copy_how = copy_bandwidth(C.L, C.dev, n)
    traffic, traffic_src, ktraffic = None, None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            if pj.get("n") == n and pj.get("ct") == ct and pj.get("input", "u10") == args.input:
                hb = pj.get("hbm_bytes_per_launch", {})

                def pmc_bytes(name):       # table "parse3_kernel<7>" = rocprof "parse3_kernel<7, 16>"
                    if name in hb:
                        return hb[name]
                    stem = name[:-1] if name.endswith(">") else name
                    hits = [v for k, v in hb.items() if k.startswith(stem) and k[len(stem):len(stem) + 1] in (",", ">")]
                    return hits[0] if len(hits) == 1 else None
                traffic = pmc_bytes(dname)
                ktraffic = {}
                for kn, (_, ab) in kernels.items():
                    tb = pmc_bytes(kn)
                    if tb is not None and ab > 0:
                        ktraffic[kn] = {"hbm_bytes": int(tb), "algorithmic_bytes": int(ab), "ratio": round(tb / ab, 3)}
                traffic_src = (f"profiles/pmc_latest.json: rocprofv3 --pmc FETCH_SIZE (x the kernel's calibrated "
                               f"read-pattern factor, {pj.get('fetch_calibration', 'x2 gfx950')}) + WRITE_SIZE of this "
                               f"bench command, separate passes ({pj.get('source', 'tools/profile.sh')}); not measured "
                               f"in this run") if traffic is not None else None
        except Exception:
            traffic = None
    res = {
        "metric": "GB/s (input float bytes) compress+decompress, CT=7 absErrorBound=1e-3, 1/2/4/8 GPUs",
        "value": main_line["value"],
        "unit": "GB/s",
        "n_gpus": C.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main_line["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic {args.input.upper()} ("
                + ("counter-based splitmix64 uniform [0,10), seed 42" if args.input == "u10" else
                   "every value 0.123456789, tools/float_eq_262144.txt tiled") + "), generated per rank",
        "config": {"workload": f"CT{ct} bit-wise compress+decompress, {args.input.upper()} 2^{args.log2n} float32 per GPU, "
                               f"absErrorBound={args.bound:g}", "floats_per_gpu": n, "ct": ct,
                   "stream_bytes": int(nbytes), "ratio": main_line["ratio"], "type": W["type"],
                   "mask17": f"{W['mask17']:05x}", "parallelism": f"dp{C.world}",
                   "encoder": {1: "single pass", 2: "count + pack", 3: "three-launch"}.get(R.get("enc_mode", 1), "?")
                              + (" (ranks share a GPU)" if C.shared_gpu else "")},
        "roofline": {"bound": "hbm", "kernel": dname, "achieved": main_line["dominant"]["achieved_GBs"],
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": main_line["dominant"]["frac"],
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": int(kernels[dname][1]),
                     "avg_launch_ms": main_line["dominant"]["avg_launch_ms"],
                     "achievable": round(achievable, 1),
                     "achievable_source": f"hand-written streaming copy of 2^{args.log2n} floats (dc_copy_rate_device, best "
                                          f"variant: {copy_how}), read + written bytes",
                     "frac_of_achievable": round(main_line["dominant"]["achieved_GBs"] / achievable, 4)},
        "kernels_ms": main_line["kernels_ms"],
        "kernels_traffic": ktraffic,
        "phases_ms": {"encode": round(R["enc_ms"], 4), "decode": round(R["dec_ms"], 4),
                      "med_dataset_s": round(W["t_med"], 4)},
        "pipeline_roofline_frac": round((8.0 * n + 2 * nbytes) / ((R["enc_ms"] + R["dec_ms"]) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "decoder_fast_path": R["status"] == 0,
        "slow_path_in_timed_step": bool(R["slow_path_timed"]),
        "self_check": all_ranks_ok(C, R["self_check"]["ok"]),
        "self_check_detail": R["self_check"],
    }
    if "pipelined" in R:
        res["pipelined"] = R["pipelined"]
    if "check" in R:
        res["check_vs_oracle"] = R["check"]
    if args.ber > 0:
        res["metric"] = "GB/s (input float bytes) CT=9 flow: CT7 encode + CRC-32 + BER bit flips + CRC check + resend + decode"
        res["config"]["workload"] = (f"CT9 (CT7 stream + CRC-32) at BER={args.ber:g} with real bit flips, "
                                     f"{args.input.upper()} 2^{args.log2n} float32 per GPU, absErrorBound={args.bound:g}")
        res["config"].update({"ber": args.ber, "flips_per_step": int(R["nbits"] * args.ber), "resends": R["resends"],
                              "detected_all": R["resends"] == args.steps and bool(R["ct9"].get("acks_ok"))})
    if C.world > 1 and args.ber > 0:
        # config 5 across GPUs: the CT9 stream travels to the partner rank and back (the headline of --ber at N > 1);
        # the per-rank flow with a local channel copy stays beside it
        res["local_channel"] = {"value": res["value"], "ms_per_step": res["ms_per_step"]}
        X = ct9_pairs_run(C, W, args.steps, args.warmup, args.ber)
        res["ct9_exchange"] = X
        res["value"], res["ms_per_step"] = X["value"], X["ms_per_step"]
        res["config"]["detected_all"] = bool(X["detected_all"])
        res["config"]["parallelism"] = f"pairs{C.world}"
    elif C.world > 1 and not args.no_e2e:
        res["end_to_end"] = e2e_run(C, W, args.steps, args.warmup)
    del W
    if C.world == 1 and not args.no_extra and args.ber <= 0:
        import torch
        torch.cuda.empty_cache()
        # the size sweep of north_star (2^14..2^28 U10, CT7) and the other BASELINE configs, few steps each
        res["sweep"] = {}
        for lg in (14, 18, 22, 28):
            res["sweep"][f"2^{lg}"] = side_config(C, 7, "u10", lg, max(5, args.steps // 4), 2, args.bound)
        res["prepass_chain"] = prepass_chain(C, 26, args.bound)
        res["configs"] = {
            "config2_ct6_u10_2^26": side_config(C, 6, "u10", 26, max(5, args.steps // 4), 2, args.bound),
            "config3_ct7_eq_2^28": side_config(C, 7, "eq", 28, max(5, args.steps // 4), 2, args.bound),
            "config5_ct9_ber1e-6_u10_2^26": side_config(C, 7, "u10", 26, 5, 1, args.bound, ber=1e-6),
        }
    if C.world == 1 and not args.no_cpu:           # rank 0 at N=1 only (the contract's cpu_baseline leg)
        res["cpu_baseline"] = cpu_baseline(ct, args.bound, 1 << args.cpu_log2n, args.input)
    if C.rank == 0:
        print(json.dumps(res), flush=True)
    bad = [nm for nm, ok in [("main", res["self_check"])] + [(f"sweep {k}", v.get("self_check")) for k, v in
                                                               res.get("sweep", {}).items()]
           + [(k, v.get("self_check")) for k, v in res.get("configs", {}).items()]
           + [("prepass_chain", res.get("prepass_chain", {}).get("self_check"))]
           + [("end_to_end", res.get("end_to_end", {}).get("self_check")),
              ("ct9_exchange", res.get("ct9_exchange", {}).get("self_check"))] if ok is False]
    if C.dist is not None:
        C.dist.destroy_process_group()
    if bad:
        sys.exit(f"bench.py: self-check failed ({', '.join(bad)}): the hashes of the last step's stream / decode "
                 f"differ from the oracle's (tests/golden/bench_hashes.json)")


def all_ranks_ok(C, ok):
    """True / False / None (no golden) over every rank: False if any rank failed."""
    if C.dist is None:
        return ok
    import torch
    t = torch.tensor([2.0 if ok is None else (1.0 if ok else 0.0)], dtype=torch.float64, device=C.dev)
    C.dist.all_reduce(t, op=C.dist.ReduceOp.MIN)
    v = float(t[0])
    return False if v < 0.5 else (True if v < 1.5 else None)


def ct9_pairs_run(C, W, steps, warmup, ber):
    """BASELINE config 5 across GPUs (CT9 = CT7 stream + CRC-32 at a bit-error rate): the
    ranks pair up (dcamd.ct9_partner: 0-1, 2-3, ...) and every step each rank encodes its shard, CRCs its
    stream and sends stream + [CRC, bits] to its partner over torch.distributed point-to-point (RCCL over xGMI
    on device tensors), while receiving the partner's; the channel flips floor(bits * BER) bits of what
    arrived, the receiver CRCs it and answers with an ack; a rejected stream is sent again and checked again
    (impl/pingpong.c:280-289 sender, :408-447 receiver); then each rank decodes the copy it RECEIVED.  The acks
    are read on the host every round (the reference's blocking MPI_Recv of crc_ok).  value = all ranks'
    floats / max-over-ranks step time (each rank encodes n floats and decodes n)."""
    import torch
    L, dev, dcamd = C.L, C.dev, C.dcamd
    n, ct, typ, mask17, xs = W["n"], W["ct"], W["type"], W["mask17"], W["xs"]
    cap = L.stream_capacity(n)
    stream = torch.zeros(cap, dtype=torch.uint8, device=dev)
    rcv = torch.zeros(cap, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    d_nbits = torch.zeros(1, dtype=torch.int64, device=dev)
    idx0 = C.rank * n
    partner = dcamd.ct9_partner(C.rank, C.world)
    ops = dcamd.LibCT9(L)
    torch.cuda.synchronize()
    L.encode_device(ct, xs.data_ptr(), n, stream.data_ptr(), idx0=idx0, type_=typ, mask17=mask17,
                    total_ptr=d_nbits.data_ptr())
    nbits = L.encode_result()
    nbytes = (nbits + 7) // 8
    nbits_rx = dcamd.ct9_sizes(nbits, partner, dev)
    nbytes_rx = (nbits_rx + 7) // 8
    meta_tx = torch.zeros(2, dtype=torch.int64, device=dev)
    meta_tx[1] = nbits
    meta_rx = torch.zeros(2, dtype=torch.int64, device=dev)
    crc_rx = torch.zeros(1, dtype=torch.int64, device=dev)
    ack = torch.zeros(2, dtype=torch.int64, device=dev)
    nflip = int(nbits_rx * ber)
    seed = [1 + 1000003 * C.rank]
    log = []

    def step():
        L.encode_device(ct, xs.data_ptr(), n, stream.data_ptr(), idx0=idx0, type_=typ, mask17=mask17,
                        total_ptr=d_nbits.data_ptr())
        r = dcamd.ct9_exchange(ops, stream, nbytes, meta_tx, rcv, nbytes_rx, nbits_rx, meta_rx, crc_rx, ack, partner,
                               nflip, seed[0])
        seed[0] += nflip
        L.decode_device(ct, rcv.data_ptr(), nbytes_rx, n, out.data_ptr(), type_=typ, mask17=mask17, max_bytes=cap)
        log.append(r)

    for _ in range(max(warmup, 1)):
        step()
        L.decode_finish()
    L.synchronize()
    log.clear()
    C.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    L.synchronize()
    torch.cuda.synchronize()
    wall = C.max_over_ranks(time.perf_counter() - t0)
    st = {"encode": L.encode_status(), "decode": L.decode_status()}
    if any(st.values()):
        print(f"bench.py: CT9 exchange status words {st} after the timed steps", file=sys.stderr)
        sys.exit(1)
    # every round detected its damaged copy (nflip > 0: the first check fails, the resent copy passes)
    detected = all(ok and (rx == 1 if nflip > 0 else rx == 0) and rounds == (2 if nflip > 0 else 1)
                   for rounds, _, rx, ok in log) and len(log) == steps
    detected = all_ranks_ok(C, detected)
    # self-check: the received copy and its decode, poisoned first, against the oracle's stream and decode of
    # the PARTNER's shard
    rcv.fill_(0x5A)
    out.view(torch.int32).fill_(-1)
    torch.cuda.synchronize()
    step()
    L.synchronize()
    if L.decode_status():
        L.decode_finish()
    torch.cuda.synchronize()
    rh = L.hash_device(rcv.data_ptr(), nbytes_rx)
    oh = L.hash_device(out.data_ptr(), 4 * n)
    g = golden_entry(ct, W["kind"], W["log2n"], W["bound"], C.world)
    if g is not None and C.world > 1:
        g = g["ranks"][partner]
    ok = None if g is None else (int(g["nbits"]) == nbits_rx and int(g["stream"]) == rh and int(g["out"]) == oh)
    ok = all_ranks_ok(C, ok)
    return {"value": round(C.world * 4.0 * n / (wall / steps) / 1e9, 3), "ms_per_step": round(wall / steps * 1e3, 4),
            "partner": partner, "stream_bytes_sent": int(nbytes), "flips_per_step": nflip,
            "resends_per_step": float(np.mean([r[2] for r in log])) if log else 0.0, "detected_all": detected,
            "self_check": ok, "received_hash": f"{rh:016x}",
            "self_check_golden": ("tests/golden/bench_hashes.json: the oracle's stream and decode of the partner's "
                                  "shard" if g is not None else "none for this workload"),
            "how": "pairs (0-1, 2-3, ...): encode + CRC-32 of the own stream, stream + [CRC, bits] to the partner and "
                   "the partner's received (torch.distributed P2P: RCCL over xGMI), BER flips on the received copy, "
                   "receiver CRC + ack back, the rejected stream resent and re-checked, decode of the received "
                   "copy; acks read on the host each round"}


def e2e_run(C, W, steps, warmup):
    """End-to-end multi-GPU step, device-side: each rank encodes its shard at start bit 0 with
    its global index (bit count left on the device), the bit counts and the shards are all-gathered (RCCL
    over xGMI; slots sized from the warm-up's largest shard), one merge kernel scans the counts and lays
    the shards into the single global stream on every rank, and each rank cuts its shard out of that
    received stream and decodes it with the segment decoder, its first predictions fixed after a 12-byte
    all-gather of the previous shard's last values.  No host read inside the timed steps; the status words are checked after them."""
    import torch
    L, dev, dcamd = C.L, C.dev, C.dcamd
    n, ct, typ, mask17, xs = W["n"], W["ct"], W["type"], W["mask17"], W["xs"]
    cap = L.stream_capacity(n)
    local = torch.zeros(cap + 64, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    glob = torch.zeros((C.world * cap + 64) // 4 * 4, dtype=torch.uint8, device=dev)
    d_count = torch.zeros(1, dtype=torch.int64, device=dev)
    d_total = torch.zeros(1, dtype=torch.int64, device=dev)
    recv = torch.zeros(cap + 64, dtype=torch.uint8, device=dev)       # this rank's shard cut out of the received
    d_rbits = torch.zeros(1, dtype=torch.int64, device=dev)           # global stream
    idx0 = C.rank * n
    slot = [(cap + 8 + 3) // 4 * 4]

    dbg = [bool(os.environ.get("DC_BENCH_DEBUG"))]

    def show(what):
        if dbg[0]:
            L.synchronize()
            torch.cuda.synchronize()
            print(f"e2e rank {C.rank} {what}: count {int(d_count.item())} total {int(d_total.item())} enc "
                  f"{L.encode_status()} dec {L.decode_status()}", file=sys.stderr, flush=True)

    def step():
        L.encode_device(ct, xs.data_ptr(), n, local.data_ptr(), idx0=idx0, type_=typ, mask17=mask17, start_bit=0,
                        total_ptr=d_count.data_ptr())
        show("after encode")
        counts = dcamd.gather_stream_device(L, local, d_count, slot[0], glob, d_total)
        show("after gather")
        dcamd.decode_sharded_device(L, ct, local, d_count, (cap + 64) // 16 * 16, n, out, typ, mask17,
                                    received=(glob, counts, recv, d_rbits))
        show("after decode")

    # the zero fills above are queued on torch's stream, the steps on the library's: without this a fill
    # could land after the first encode wrote its bit count (seen with two ranks sharing one GPU)
    torch.cuda.synchronize()
    for _ in range(max(warmup, 1)):
        step()
    dbg[0] = False
    L.synchronize()
    torch.cuda.synchronize()
    # the slot for the timed steps: the warm-up's largest shard (a real run takes the previous step's)
    mx = torch.tensor([int(d_count.item())], dtype=torch.int64, device=dev)
    C.dist.all_reduce(mx, op=C.dist.ReduceOp.MAX)
    slot[0] = min((int(mx.item()) + 7) // 8 + 64 + 3, cap + 8 + 3) // 4 * 4
    for _ in range(max(warmup, 1)):
        step()
    C.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    L.synchronize()
    torch.cuda.synchronize()
    wall = C.max_over_ranks(time.perf_counter() - t0)
    st = {"encode": L.encode_status(), "merge": L.merge_status(), "decode": L.decode_status()}
    if any(st.values()):
        print(f"bench.py: end-to-end status words {st} after the timed steps", file=sys.stderr)
        sys.exit(1)
    # self-check: poison the merged global stream and the decoded shard, one more step, device hashes against
    # the oracle's global stream and its decode's slice for this rank (tests/golden/bench_hashes.json)
    glob.fill_(0xA5)
    recv.fill_(0x5A)
    out.view(torch.int32).fill_(-1)
    torch.cuda.synchronize()
    step()
    L.synchronize()
    torch.cuda.synchronize()
    total = int(d_total.item())
    gh = L.hash_device(glob.data_ptr(), (total + 7) // 8)
    oh = L.hash_device(out.data_ptr(), 4 * n)
    g = golden_entry(ct, W["kind"], W["log2n"], W["bound"], C.world)
    ok = None if g is None else (int(g["nbits"]) == total and int(g["stream"]) == gh and int(g["e2e_outs"][C.rank]) == oh)
    ok = all_ranks_ok(C, ok)
    return {"value": round(C.world * 4.0 * n / (wall / steps) / 1e9, 3), "ms_per_step": round(wall / steps * 1e3, 4),
            "global_stream_bytes": (total + 7) // 8, "slot_bytes": slot[0],
            "self_check": ok, "global_stream_hash": f"{gh:016x}",
            "self_check_golden": ("tests/golden/bench_hashes.json: the oracle's stream of the whole global array and "
                                  "its decode, every rank's slice" if g is not None else "none for this workload"),
            "how": "encode at start bit 0 (device bit count) + all-gather of the bit counts and of the shards "
                   "(slots from the warm-up's largest) + one merge kernel (device exscan, shifted shards, "
                   "OR-ed shared words) into the single global stream on every rank + each rank's shard cut "
                   "out of that received stream (extract kernel) and decoded by the segment decoder with a "
                   "12-byte all-gather of the previous shard's last values and a one-wave prefix fix; no host "
                   "read inside the timed steps"}


if __name__ == "__main__":
    main()
