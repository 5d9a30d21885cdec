"""Host logic of the multi-GPU med_dataset_float (dcamd.global_med, the exscan of whole-shard binade
transducers) on CPU: gloo ranks run global_med against a numpy stand-in of the three device entry points
(dc_med_shard_stats, dc_med_shard_trans, dc_med_sum_device) whose transducers come from brute-force
sequential float32 sums, and the mean and type must equal the oracle's single-array med_dataset_float
(oracle/dc_oracle.c, impl/dataCompression.c:3593-3620) bit for bit.  The device kernels themselves are
checked the same way in tests/test_gpu_dist.py."""
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

MW = 6


def _seq_sum(x, s0):
    """left-to-right float32 sum of x from s0 (np.add.accumulate is sequential)"""
    a = np.concatenate([np.array([s0], np.float32), np.asarray(x, np.float32)])
    return np.add.accumulate(a, dtype=np.float32)[-1]


def _expo(s):
    return (int(np.array([np.float32(s)], np.float32).view(np.uint32)[0]) >> 23) & 0xFF


class _FakeL:
    """numpy stand-in of the library's three shard entry points (the xs_ptr argument is the array)"""

    class _C:
        @staticmethod
        def dc_med_shard_binades():
            return MW

    L = _C()

    def __init__(self):
        self.exact_calls = 0

    def med_shard_stats(self, x, n):
        v = x[~np.isnan(x)]
        mx = np.float32(v.max()) if v.size else np.float32(-np.inf)
        return float(np.sum(x[np.isfinite(x)], dtype=np.float64)), mx, np.float32(x[0])

    def med_sum_device(self, x, n, s):
        self.exact_calls += 1
        return _seq_sum(x, np.float32(s)), None

    def med_shard_trans(self, x, n, s_est):
        e_lo = _expo(np.float32(min(max(s_est, 0.0), 3.0e38))) - 4
        units = np.zeros((MW, 2), np.int64)
        flags = np.zeros(MW, np.uint8)
        neg = bool(np.any(~(x >= 0)))
        for w in range(MW):
            E = e_lo + w
            f = 0
            for p in range(2):
                if neg or E < 24 or E > 253:
                    f = 4
                    break
                k0 = (1 << 23) + p
                s1 = _seq_sum(x, np.float32(k0 * 2.0 ** (E - 150)))
                if _expo(s1) != E:
                    f = 4
                    break
                k1 = (int(np.array([s1], np.float32).view(np.uint32)[0]) & 0x7FFFFF) | 0x800000
                units[w, p] = k1 - k0
                f |= (k1 & 1) << p
            flags[w] = f
        return e_lo, units, flags

    @staticmethod
    def type_from_max(mx):
        add = 0
        for i in range(7, 0, -1):
            add += 1 << i
            if float(mx) < 2.0 ** (add - 127):
                return 8 - i
        return 0


def _case(kind, world, n):
    from pyoracle import Oracle
    O = Oracle()
    N = world * n
    if kind == "u10":
        _, xs = O.to_small(O.gen_u10(N))
    elif kind == "neg":
        xs = np.random.default_rng(5).standard_normal(N).astype(np.float32)
    elif kind == "nan_cut":
        _, xs = O.to_small(O.gen_u10(N))
        xs[n] = np.nan                     # the second shard's first value: NaN (max, and the sum goes NaN)
    elif kind == "zeros_head":
        _, xs = O.to_small(O.gen_u10(N))
        xs[:n + 100] = 0.0                 # the first shard sums to +0: rank 1 starts from 0
    else:
        raise ValueError(kind)
    return np.ascontiguousarray(xs, np.float32)


def _worker(rank, world, port, kind, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcamd
        from pyoracle import Oracle
        xs = _case(kind, world, n)
        L = _FakeL()
        mean, typ = dcamd.global_med(L, xs[rank * n:(rank + 1) * n].copy(), n, torch.device("cpu"))
        m_ref, t_ref = Oracle().med(xs)
        ok = bool(np.array([mean], np.float32).view(np.uint32)[0] == np.array([m_ref], np.float32).view(np.uint32)[0]
                  and typ == t_ref)
        q.put((rank, ok, L.exact_calls, float(mean), float(m_ref)))
    except Exception as e:
        q.put((rank, False, repr(e), None, None))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("kind,world,n", [("u10", 4, 30000), ("u10", 2, 20001), ("neg", 3, 10000),
                                          ("nan_cut", 2, 10000), ("zeros_head", 3, 8000)])
def test_global_med_exscan(kind, world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True for r in res), res
    if kind == "u10" and world == 4:       # ranks whose sum stays in one binade take no exact pass
        assert sum(r[2] for r in res) < world, res


def test_med_apply_shard_matches_sequential_sum():
    """The transducer claim behind the exscan: within one binade a shard adds units that depend only on
    the incoming k's parity, for every k that keeps the sum in the binade."""
    import dcamd
    rng = np.random.default_rng(11)
    L = _FakeL()
    for trial in range(20):
        E = int(rng.integers(120, 140))
        u = 2.0 ** (E - 150)
        x = (rng.random(400) * rng.choice([0.3, 2.0, 50.0]) * u).astype(np.float32)
        if trial % 5 == 0:
            x[::7] = np.float32(u * 0.5)        # ties
        e_lo, units, flags = L.med_shard_trans(x, x.size, float(np.float32(1.5 * 2.0 ** (E - 127))))
        for k in rng.integers(1 << 23, 1 << 24, 40):
            s = np.float32(int(k) * u)
            got = dcamd.med_apply_shard(e_lo, units, flags, s)
            ref = _seq_sum(x, s)
            if got is None:
                assert _expo(ref) != E or int(flags[E - e_lo]) & 4
            else:
                assert got == ref, (trial, int(k))
