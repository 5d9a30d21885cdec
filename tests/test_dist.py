"""Multi-process (gloo, world_size 2, CPU) tests of the sharded path: per-rank shard streams are
stitched into the single-stream bytes by an all-gather (dcamd.gather_stream), as the RCCL path does
on GPUs.  Shard streams come from the oracle (test infrastructure): the first k tokens of a stream
depend only on x[:k] (encoder history = original inputs), so a shard's bits are the global stream's
bits between the two shard boundaries."""
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


def _bits_of(nbytes, pos):
    return nbytes * 8 if pos == 8 else (nbytes - 1) * 8 + (8 - pos)


def _extract(stream, b0, b1):
    """bits [b0, b1) of stream, re-packed so that they start at bit b0 % 8 of byte 0."""
    bits = np.unpackbits(stream)
    lead = b0 % 8
    sub = np.concatenate([np.zeros(lead, np.uint8), bits[b0:b1]])
    return np.packbits(sub)


def _worker(rank, world, port, ct, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcamd
        from pyoracle import Oracle
        O = Oracle()
        x = O.gen_u10(n)
        _, xs = O.to_small(x)
        t, m17 = O.type_mask(xs)
        s, nb, pos = O.compress(ct, xs, 1e-3, t, m17)
        cut = [n * r // world for r in range(world + 1)]
        offs = []
        for c in cut:
            if c == 0:
                offs.append(0)
            else:
                _, nbc, posc = O.compress(ct, xs[:c], 1e-3, t, m17)
                offs.append(_bits_of(nbc, posc))
        b0, b1 = offs[rank], offs[rank + 1]
        local = torch.from_numpy(_extract(s, b0, b1))
        out, total = dcamd.gather_stream(local, b0 % 8, b0 % 8 + (b1 - b0))
        q.put((rank, total == _bits_of(nb, pos), bool(np.array_equal(out.numpy(), s))))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("ct,n", [(7, 20001), (6, 4099), (5, 777)])
def test_gather_stream_world2(ct, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ct, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] and r[2] for r in res), res


def test_shard_offsets():
    import dcamd
    assert dcamd.shard_offsets([5, 0, 7]) == ([0, 5, 5], 12)


def _settle_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcamd
        # every shard is one prediction chain: its last values are its incoming values + 1, so rank r
        # ends at r only after the exchange has run r rounds
        state = {"last": torch.zeros(3) if rank == 0 else torch.full((3,), -1.0)}

        def tail3():
            return state["last"].clone()

        def fix(hin):
            state["last"] = hin + 1.0
            return tail3()

        out = dcamd.settle_history(tail3, fix)
        q.put((rank, out.tolist()))
    finally:
        dist.destroy_process_group()


def test_settle_history_world3():
    """The sharded decode's 12-byte exchange converges even when prediction chains span whole shards."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_settle_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert res[r] == [float(r)] * 3, res


def _plane(rank, h, n=4096):
    """Deterministic stand-in for rank `rank`'s z-halo plane h (Himeno-like rows of equal values)."""
    i = np.arange(n) // 64
    return ((i * i).astype(np.float32) / np.float32(63 * 63) + np.float32(0.25 * rank + 0.1 * h)).astype(np.float32)


def _halo_worker(rank, world, port, ct, q, empty=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcamd
        from pyoracle import Oracle
        O = Oracle()

        def enc(r, h):
            mn, xs = O.to_small(_plane(r, h))
            s, nb, pos = O.compress(ct, xs, 1e-3, 0, 0)
            return s, _bits_of(nb, pos), mn

        def enc_side(r, h):                              # empty: every plane k = kmax - 2 is a 0-bit stream
            return (np.zeros(0, np.uint8), 0, 0.0) if (empty and h == 1) else enc(r, h)

        mine = [enc_side(rank, 0), enc_side(rank, 1)]
        down = rank - 1 if rank > 0 else None            # MPI_Cart, non-periodic: PROC_NULL at the ends
        up = rank + 1 if rank + 1 < world else None
        got = dcamd.halo_exchange([torch.from_numpy(m[0]) for m in mine], [m[1] for m in mine],
                                  [m[2] for m in mine], down, up)
        ok = True
        # from up: its plane k = 1 (h = 0), for our k = kmax - 1; from down: its plane k = kmax - 2 (h = 1)
        for peer, h, rec in ((up, 0, got[0]), (down, 1, got[1])):
            if peer is None:
                ok &= rec is None
                continue
            s, bits, mn = enc_side(peer, h)
            rs, rbits, rmn = rec
            ok &= rbits == bits and rmn == mn and np.array_equal(rs.numpy(), s)
            if bits == 0:
                continue
            d, n = O.decompress(ct, rs.numpy(), 4096, 1e-3, 0, 0)
            ok &= n == 4096 and bool(np.all(np.abs(d + rmn - _plane(peer, h)) <= 1e-3 * 1.01))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,empty", [(2, False), (3, False), (4, False), (3, True)])
def test_halo_exchange(world, empty):
    """dcamd.halo_exchange (impl/himenoBMTxps.c:644-690: sizes first, then min + stream bytes, to the
    z-neighbours of a non-periodic line of ranks) delivers every neighbour's compressed plane intact."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, 5, q, empty)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] for r in res), res


class _NpCT9:
    """Host stand-in for dcamd.LibCT9 (zlib's CRC-32 = the reference's do_crc32; the flips at
    dcamd.flip_positions, as dc_flip_bits_device places them)."""

    def crc(self, buf, nbytes, dst):
        import zlib
        dst[0] = zlib.crc32(buf[:nbytes].numpy().tobytes())

    def flip(self, buf, nbits, count, seed):
        import dcamd
        for p in dcamd.flip_positions(nbits, count, seed):
            buf[p // 8] ^= 0x80 >> (p % 8)


def _ct9_worker(rank, world, port, nflip, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcamd
        from pyoracle import Oracle
        O = Oracle()
        n = 5000 + 777 * rank                          # shards of different lengths: different stream sizes
        x = O.gen_u10(n) + np.float32(rank)
        _, xs = O.to_small(x)
        t, m17 = O.type_mask(xs)
        s, nb, pos = O.compress(7, xs, 1e-3, t, m17)
        nbits = _bits_of(nb, pos)
        partner = dcamd.ct9_partner(rank, world)
        stream = torch.zeros(nb + 64, dtype=torch.uint8)
        stream[:nb] = torch.from_numpy(s)
        nbits_rx = dcamd.ct9_sizes(nbits, partner, stream.device)
        nb_rx = (nbits_rx + 7) // 8
        rcv = torch.zeros(nb_rx + 64, dtype=torch.uint8)
        meta_tx = torch.zeros(2, dtype=torch.int64)
        meta_tx[1] = nbits
        meta_rx, crc_rx, ack = (torch.zeros(2, dtype=torch.int64), torch.zeros(1, dtype=torch.int64),
                                torch.zeros(2, dtype=torch.int64))
        res = dcamd.ct9_exchange(_NpCT9(), stream, nb, meta_tx, rcv, nb_rx, nbits_rx, meta_rx, crc_rx, ack, partner,
                                 nflip, 7 + rank)
        # what arrived is the partner's stream exactly (after the resend), and decodes as the partner's data
        xp = O.gen_u10(5000 + 777 * partner) + np.float32(partner)
        _, xps = O.to_small(xp)
        tp, mp_ = O.type_mask(xps)
        sp, nbp, _ = O.compress(7, xps, 1e-3, tp, mp_)
        same = bool(nb_rx == nbp and np.array_equal(rcv[:nb_rx].numpy(), sp))
        q.put((rank, partner, res, same))
    except Exception as e:
        q.put((rank, None, repr(e), False))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nflip", [(2, 3), (2, 0), (3, 2), (4, 1)])
def test_ct9_exchange(world, nflip):
    """BASELINE config 5 across ranks, the protocol on host tensors (gloo): rank pairs swap CT7 streams with
    their CRC-32, the receiver's copy is damaged by nflip bit flips, the CRC check rejects it, the sender
    resends and the second check passes; the partner's stream arrives bit-exact.  An odd world's last rank is
    its own partner (local channel)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ct9_worker, args=(r, world, port, nflip, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, partner, r, same in res:
        assert partner == (rank ^ 1 if (rank ^ 1) < world else rank), res
        rounds, resent_tx, resent_rx, ok = r
        assert ok and same, res
        assert rounds == (2 if nflip else 1) and resent_rx == (1 if nflip else 0), res
        assert resent_tx == (1 if nflip else 0), res
