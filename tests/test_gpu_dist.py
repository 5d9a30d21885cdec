"""GPU multi-process test of the sharded path (bench.py's end-to-end step): two gloo ranks
share cuda:0.  Every rank counts its shard's bits (dc_encode_bits_device), the counts are all-gathered into
global start bits, each rank encodes its shard at (start mod 8) with its global index and predictor halo,
the shards are gathered into the single global stream (dcamd.gather_stream) and each rank decodes its
shard of that stream (dcamd.decode_sharded: deferred history, 12-byte exchange, prefix fix).  The
gathered stream must equal the oracle's single-stream encode of the whole array (oracle/dc_oracle.c, the
restatement pinned to the compiled reference), and every rank's values the oracle decode's slice, bit
for bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))

pytestmark = pytest.mark.gpu


def _bits_of(nbytes, pos):
    return nbytes * 8 if pos == 8 else (nbytes - 1) * 8 + (8 - pos)


def _worker(rank, world, port, ct, n, kind, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcamd
        from pyoracle import Oracle
        L = dcamd.Lib()
        L.init(0)
        L.set_bound(1e-3)
        O = Oracle()
        N = world * n
        x = O.gen_u10(N)
        if kind == "chain":                   # a constant run across every cut: a prediction chain enters
            for r in range(1, world):         # the next shard, whose first values wait for the exchange
                x[r * n - 700:r * n + 900] = x[r * n - 701]
        _, xs = O.to_small(x)
        t, m17 = O.type_mask(xs)
        dev = torch.device("cuda", 0)
        lo = rank * n
        buf = torch.zeros(n + 4, dtype=torch.float32, device=dev)      # [halo | shard], shard 16-B aligned
        halo = xs[max(lo - 3, 0):lo]
        if halo.size:
            buf[4 - halo.size:4] = torch.from_numpy(halo.copy())
        buf[4:] = torch.from_numpy(xs[lo:lo + n].copy())
        xd = buf[4:]
        bits = L.encode_bits(ct, xd.data_ptr(), n, lo, t, m17)
        meta = torch.tensor([bits], dtype=torch.int64)
        parts = [torch.zeros_like(meta) for _ in range(world)]
        dist.all_gather(parts, meta)
        starts, total = dcamd.shard_offsets([int(p[0]) for p in parts])
        sb = starts[rank] % 8
        local = torch.zeros(L.stream_capacity(n) + 8, dtype=torch.uint8, device=dev)
        L.encode_device(ct, xd.data_ptr(), n, local.data_ptr(), idx0=lo, type_=t, mask17=m17, start_bit=sb)
        L.synchronize()
        glob, tot = dcamd.gather_stream(local[:(sb + bits + 7) // 8], sb, sb + bits)
        out = torch.empty(n, dtype=torch.float32, device=dev)
        dcamd.decode_sharded(L, ct, glob, glob.numel(), starts[rank], bits, n, out, t, m17)
        torch.cuda.synchronize()
        s_all, nb_all, pos_all = O.compress(ct, xs, 1e-3, t, m17)       # the oracle's single stream
        dec_all, _ = O.decompress(ct, s_all, N, 1e-3, t, m17)            # and its decode of it
        ok_stream = bool(tot == _bits_of(nb_all, pos_all) and np.array_equal(glob.cpu().numpy(), s_all))
        ok_dec = bool(np.array_equal(out.cpu().numpy().view(np.uint32), dec_all[lo:lo + n].view(np.uint32)))
        q.put((rank, ok_stream, ok_dec))
    except Exception as e:                    # report, do not hang the parent
        q.put((rank, False, repr(e)))
    finally:
        dist.destroy_process_group()


def _worker_device(rank, world, port, ct, n, kind, q, backend="gloo", received=True):
    """The device-side step (bench.py e2e): encode at start bit 0 with the global index, device bit count;
    gather_stream_device (all-gathered counts and shards, one merge kernel); decode_sharded_device (the
    segment decoder on the rank's shard -- cut out of the received global stream when `received`, else its
    own encode -- 12-byte exchange, one-wave prefix fix).  No host read until the checks.  A shard the
    segment decoder declines (a prediction chain through its whole first chunk) is decoded again on the
    host-synchronised path from the gathered stream.  backend "nccl" (world 1 on the one GPU of a box):
    the collectives run through RCCL on device tensors, the branch the driver's multi-GPU bench takes."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        import dcamd
        from pyoracle import Oracle
        L = dcamd.Lib()
        L.init(0)
        L.set_bound(1e-3)
        O = Oracle()
        N = world * n
        x = O.gen_u10(N)
        if kind == "chain":
            for r in range(1, world):
                x[r * n - 700:r * n + 900] = x[r * n - 701]
        _, xs = O.to_small(x)
        t, m17 = O.type_mask(xs)
        dev = torch.device("cuda", 0)
        lo = rank * n
        buf = torch.zeros(n + 4, dtype=torch.float32, device=dev)
        halo = xs[max(lo - 3, 0):lo]
        if halo.size:
            buf[4 - halo.size:4] = torch.from_numpy(halo.copy())
        buf[4:] = torch.from_numpy(xs[lo:lo + n].copy())
        xd = buf[4:]
        cap = L.stream_capacity(n)
        local = torch.zeros(cap + 64, dtype=torch.uint8, device=dev)
        d_count = torch.zeros(1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        L.encode_device(ct, xd.data_ptr(), n, local.data_ptr(), idx0=lo, type_=t, mask17=m17, start_bit=0,
                        total_ptr=d_count.data_ptr())
        slot = (cap + 8 + 3) // 4 * 4
        glob = torch.zeros((world * cap + 64) // 4 * 4, dtype=torch.uint8, device=dev)
        d_total = torch.zeros(1, dtype=torch.int64, device=dev)
        counts_d = dcamd.gather_stream_device(L, local, d_count, slot, glob, d_total)
        out = torch.empty(n, dtype=torch.float32, device=dev)
        rx = None
        if received:                           # decode the received bytes: poison the rank's own encode first
            L.synchronize()
            local.fill_(0xA5)
            torch.cuda.synchronize()
            rx = (glob, counts_d, torch.zeros(cap + 64, dtype=torch.uint8, device=dev),
                  torch.zeros(1, dtype=torch.int64, device=dev))
        dcamd.decode_sharded_device(L, ct, local, d_count, (cap + 64) // 16 * 16, n, out, t, m17, received=rx)
        L.synchronize()
        torch.cuda.synchronize()
        if received:
            assert int(rx[3].item()) == int(d_count.item()), (int(rx[3].item()), int(d_count.item()))
        st_enc, st_merge, st_dec = L.encode_status(), L.merge_status(reset=True), L.decode_status()
        tot = int(d_total.item())
        fallback = st_dec != 0
        if fallback:                           # the host-synchronised shard path, from the gathered stream
            L.decode_status_clear()
            bits = int(d_count.item())
            counts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(counts, torch.tensor([bits], dtype=torch.int64))
            starts, _ = dcamd.shard_offsets([int(c[0]) for c in counts])
            g = glob[:(tot + 7) // 8]
            if world == 1:
                L.decode_device(ct, g.data_ptr(), g.numel(), n, out.data_ptr(), t, m17)
                L.decode_finish()
            else:
                dcamd.decode_sharded(L, ct, g, g.numel(), starts[rank], bits, n, out, t, m17)
            torch.cuda.synchronize()
        s_all, nb_all, pos_all = O.compress(ct, xs, 1e-3, t, m17)
        dec_all, _ = O.decompress(ct, s_all, N, 1e-3, t, m17)
        nb = (tot + 7) // 8
        ok_stream = bool(st_enc == 0 and st_merge == 0 and tot == _bits_of(nb_all, pos_all) and
                         np.array_equal(glob[:nb].cpu().numpy(), s_all) and not glob[nb:nb + 16].cpu().numpy().any())
        ok_dec = bool(np.array_equal(out.cpu().numpy().view(np.uint32), dec_all[lo:lo + n].view(np.uint32)))
        q.put((rank, ok_stream, ok_dec, fallback))
    except Exception as e:
        q.put((rank, False, repr(e), None))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("ct,n,kind", [(7, (1 << 18) + 5, "u10"), (5, 100003, "chain"), (6, 65536, "u10"),
                                       (11, 40001, "chain"), (7, 300007, "chain")])
def test_sharded_encode_gather_decode_world2(ct, n, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ct, n, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True and r[2] is True for r in res), res


@pytest.mark.parametrize("ct,n,kind,received", [(7, (1 << 18) + 5, "u10", True), (5, 100003, "chain", True),
                                                (6, 65536, "u10", True), (11, 40001, "u10", True),
                                                (7, 300007, "chain", True), (7, 1 << 20, "u10", True),
                                                (7, (1 << 18) + 5, "u10", False)])
def test_device_step_world2(ct, n, kind, received):
    """The device-side multi-GPU step against the oracle's single stream and its decode; ordinary shards
    stay on the device path (no fallback).  received: every rank decodes its shard cut out of the merged
    global stream, its own encode poisoned before the decode (the step must decode what
    arrived)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_device, args=(r, 2, port, ct, n, kind, q, "gloo", received))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True and r[2] is True for r in res), res
    if kind == "u10":
        assert not any(r[3] for r in res), res


@pytest.mark.parametrize("ct,n,kind", [(7, (1 << 20) + 3, "u10"), (5, 100003, "chain"), (6, 65536, "u10")])
def test_device_step_rccl_world1(ct, n, kind):
    """The RCCL branch of the device-side step, executed (it had only ever run as gloo on host
    copies): a world-size-1 `nccl` process group on the box's one GPU, so gather_stream_device's two
    all_gather_into_tensor calls, the merge, the extract of the received shard, decode_sharded_device and
    exchange_history's all_gather all run on device tensors through RCCL; stream and decode against the
    oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    p = ctx.Process(target=_worker_device, args=(0, 1, port, ct, n, kind, q, "nccl", True))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[1] is True and res[2] is True, res
    if kind == "u10":
        assert not res[3], res


def _shard_stream(O, xs, r, n, ct, t, m17):
    """The oracle's stream of shard r (its elements' tokens with the 3 values before it as history): the
    stream of xs[r n - 3, (r+1) n) without its first three tokens (tests/golden/make_bench_hashes.py)."""
    if r == 0:
        s, nb, pos = O.compress(ct, xs[:n], 1e-3, t, m17)
        return s, _bits_of(nb, pos)
    full, fb, fp = O.compress(ct, xs[r * n - 3:(r + 1) * n], 1e-3, t, m17)
    _, hb, hp = O.compress(ct, xs[r * n - 3:r * n], 1e-3, t, m17)
    b, m = _bits_of(hb, hp), _bits_of(fb, fp) - _bits_of(hb, hp)
    bits = np.unpackbits(full[b // 8:(b + m + 7) // 8])[b % 8:b % 8 + m]
    return np.packbits(bits), m


def _worker_ct9(rank, world, port, n, ber, q):
    """Config 5 across ranks on the device (bench.py ct9_pairs_run's round): encode the shard, CRC-32, stream +
    [CRC, bits] to the partner, the channel's flips on what arrived, receiver CRC + ack, resend, decode of
    the RECEIVED copy -- against the oracle's stream and decode of the partner's shard."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcamd
        from pyoracle import Oracle
        L = dcamd.Lib()
        L.init(0)
        L.set_bound(1e-3)
        O = Oracle()
        ct = 7
        x = O.gen_u10(world * n)
        _, xs = O.to_small(x)
        t, m17 = O.type_mask(xs)
        dev = torch.device("cuda", 0)
        lo = rank * n
        buf = torch.zeros(n + 4, dtype=torch.float32, device=dev)
        halo = xs[max(lo - 3, 0):lo]
        if halo.size:
            buf[4 - halo.size:4] = torch.from_numpy(halo.copy())
        buf[4:] = torch.from_numpy(xs[lo:lo + n].copy())
        xd = buf[4:]
        cap = L.stream_capacity(n)
        stream = torch.zeros(cap, dtype=torch.uint8, device=dev)
        rcv = torch.zeros(cap, dtype=torch.uint8, device=dev)
        out = torch.empty(n, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        L.encode_device(ct, xd.data_ptr(), n, stream.data_ptr(), idx0=lo, type_=t, mask17=m17)
        nbits = L.encode_result()
        partner = dcamd.ct9_partner(rank, world)
        nbits_rx = dcamd.ct9_sizes(nbits, partner, dev)
        meta_tx = torch.zeros(2, dtype=torch.int64, device=dev)
        meta_tx[1] = nbits
        meta_rx, crc_rx, ack = (torch.zeros(2, dtype=torch.int64, device=dev), torch.zeros(1, dtype=torch.int64, device=dev),
                                torch.zeros(2, dtype=torch.int64, device=dev))
        nflip = int(nbits_rx * ber)
        res = dcamd.ct9_exchange(dcamd.LibCT9(L), stream, (nbits + 7) // 8, meta_tx, rcv, (nbits_rx + 7) // 8, nbits_rx,
                                 meta_rx, crc_rx, ack, partner, nflip, 11 + rank)
        L.decode_device(ct, rcv.data_ptr(), (nbits_rx + 7) // 8, n, out.data_ptr(), type_=t, mask17=m17, max_bytes=cap)
        L.decode_finish()
        torch.cuda.synchronize()
        sp, mp_ = _shard_stream(O, xs, partner, n, ct, t, m17)
        dp, _ = O.decompress(ct, sp, n, 1e-3, t, m17)
        nb = (nbits_rx + 7) // 8
        ok_stream = bool(mp_ == nbits_rx and np.array_equal(rcv[:nb].cpu().numpy(), sp[:nb]))
        ok_dec = bool(np.array_equal(out.cpu().numpy().view(np.uint32), dp.view(np.uint32)))
        q.put((rank, ok_stream, ok_dec, res, nflip))
    except Exception as e:
        q.put((rank, False, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,ber", [(2, (1 << 20) + 5, 1e-6), (2, 300007, 1e-4), (3, 100003, 1e-5)])
def test_ct9_exchange_device(world, n, ber):
    """BASELINE config 5 across ranks, on the GPU (ranks share cuda:0 over gloo): every received copy is
    damaged, detected by the CRC-32 check, resent, and the received stream and its decode equal the oracle's
    for the partner's shard bit for bit (an odd world's last rank keeps a local channel)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_ct9, args=(r, world, port, n, ber, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_s, ok_d, r, nflip in res:
        assert ok_s is True and ok_d is True, res
        assert nflip > 0 and r[3] and r[0] == 2 and r[2] == 1, res


def _worker_med(rank, world, port, kind, n, q):
    """dcamd.global_med on device shards (dc_med_shard_stats / dc_med_shard_trans / dc_med_sum_device)
    against the oracle's med_dataset_float of the whole array."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcamd
        from pyoracle import Oracle
        from test_med_dist import _case
        xs = _case(kind, world, n)
        L = dcamd.Lib()
        L.init(0)
        calls = [0]
        exact = L.med_sum_device

        def counted(*a):
            calls[0] += 1
            return exact(*a)
        L.med_sum_device = counted
        dev = torch.device("cuda", 0)
        xd = torch.from_numpy(xs[rank * n:(rank + 1) * n].copy()).to(dev)
        mean, typ = dcamd.global_med(L, xd.data_ptr(), n, dev)
        m_ref, t_ref = Oracle().med(xs)
        ok = bool(np.array([mean], np.float32).view(np.uint32)[0] == np.array([m_ref], np.float32).view(np.uint32)[0]
                  and typ == t_ref)
        q.put((rank, ok, calls[0], float(mean), float(m_ref)))
    except Exception as e:
        q.put((rank, False, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,n", [("u10", 4, 1 << 20), ("u10", 2, (1 << 21) + 5), ("neg", 2, 100000),
                                          ("nan_cut", 2, 65536), ("zeros_head", 3, 50000)])
def test_global_med_exscan_device(kind, world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_med, args=(r, world, port, kind, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True for r in res), res
    if kind == "u10" and world == 4:
        assert sum(r[2] for r in res) < world, res


@pytest.mark.parametrize("ct", [5, 7, 11])
def test_shard3_first_shard_declines_early_prediction(dc, oracle, ct):
    """dc_decode_shard3_device(has_history=0) is the first shard: a prediction among its first three tokens
    (possible only in a stream that is not a real start, e.g. a damaged one) declines it as it declines a
    whole stream, instead of decoding from zero history.  With has_history=1 the same shard
    decodes its pending prefix once the previous values arrive and equals the oracle's slice."""
    dc.set_bound(1e-3)
    n = 1 << 16
    x = oracle.gen_u10(2 * n)
    x[n - 40:n + 40] = x[n - 41]                  # a copy run across the cut: the shard starts with '101' codes
    _, xs = oracle.to_small(x)
    t, m17 = oracle.type_mask(xs)
    buf = torch.zeros(n + 4, dtype=torch.float32, device="cuda")
    buf[1:4] = torch.from_numpy(xs[n - 3:n].copy())
    buf[4:] = torch.from_numpy(xs[n:].copy())
    cap = dc.stream_capacity(n)
    local = torch.zeros(cap + 64, dtype=torch.uint8, device="cuda")
    d_count = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    dc.encode_device(ct, buf[4:].data_ptr(), n, local.data_ptr(), idx0=n, type_=t, mask17=m17, start_bit=0,
                     total_ptr=d_count.data_ptr())
    dc.encode_result()
    mb = (cap + 64) // 16 * 16
    dc.decode_status_clear()
    dc.decode_shard3_device(ct, local.data_ptr(), d_count.data_ptr(), mb, n, out.data_ptr(), t, m17, has_history=0)
    dc.synchronize()
    st = dc.decode_status()
    assert st & 512 and st & 16384, hex(st)
    dc.decode_status_clear()
    dc.decode_shard3_device(ct, local.data_ptr(), d_count.data_ptr(), mb, n, out.data_ptr(), t, m17, has_history=1)
    s_all, _, _ = oracle.compress(ct, xs, 1e-3, t, m17)
    dec_all, _ = oracle.decompress(ct, s_all, 2 * n, 1e-3, t, m17)
    hin = torch.from_numpy(dec_all[n - 3:n][::-1].copy()).cuda()
    torch.cuda.synchronize()
    dc.decode_shard3_fix(hin.data_ptr())
    dc.synchronize()
    assert dc.decode_status() == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint32), dec_all[n:].view(np.uint32))
    dc.decode_status_clear()
