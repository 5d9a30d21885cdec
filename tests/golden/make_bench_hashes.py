"""Hashes of the oracle's streams and decodes for bench.py's self-check (tests/golden/bench_hashes.json).

bench.py runs one more step after its timed steps into poisoned buffers and compares dc_hash_device of the
stream and of the decoded floats with these.  Each entry replays bench.prepare on the CPU oracle:

  N = 1       x = gen_u10(n) (or the EQ constant), toSmallDataset, exact sequential mean -> type / mask17,
              stream = oracle.compress, out = oracle.decompress (the grammar decoder, pinned to the compiled
              reference by tests/test_oracle.py)
  N = W > 1   the global array X = gen_u10(W n); toSmallDataset over X, the exact mean over X; rank r owns
              X[r n, (r+1) n) with a 3-float history.  Its shard stream holds the tokens of its elements
              (bits [B_r, B_r+1) of the global stream, re-aligned to bit 0: the stream of X[r n - 3, (r+1) n)
              without its first three tokens), its plain decode out_r = oracle.decompress(shard stream);
              the end-to-end step's merged global stream = oracle.compress(X) and each rank's shard-mode
              decode = oracle.decompress(global stream)[r n, (r+1) n).

The hash (dcamd.hash_words = dc_hash_device): sum over 32-bit little-endian words w_i of
splitmix64(i << 32 | w_i) mod 2^64, bytes past the stream's last byte zero.

    python tests/golden/make_bench_hashes.py [--worlds 1,2,4,8]      (CPU, a few minutes)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
from pyoracle import Oracle  # noqa: E402
import dcamd  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_hashes.json")


def key(ct, kind, log2n, bound, world):
    return f"ct{ct}_{kind}_2^{log2n}_{bound:g}_w{world}"


def gen(kind, n, offset=0):
    if kind == "u10":
        return dcamd.gen_u10(n, 42, offset)
    return np.full(n, np.float32(0.123456789), np.float32)


def nbits_of(nbytes, pos):
    # pos = the free bits left in the last byte (8: it is full), impl/dataCompression.c's convention
    return nbytes * 8 - (pos % 8)


def drop_bits(s, nbits, b):
    """Bits [b, nbits) of stream s as a stream starting at bit 0 (zero-padded last byte)."""
    m = nbits - b
    if m <= 0:
        return np.zeros(0, np.uint8), 0
    bits = np.unpackbits(s[b // 8:(nbits + 7) // 8])[b % 8:b % 8 + m]
    return np.packbits(bits), m


def entry(O, ct, kind, log2n, bound, world):
    n = 1 << log2n
    X = gen(kind, world * n)
    _, xs = O.to_small(X)
    del X
    mean, typ = O.med(xs)
    m17 = O.mask17(mean)
    t0 = time.time()
    s, nb, pos = O.compress(ct, xs, bound, typ, m17)
    nbits = nbits_of(nb, pos)
    e = {"type": int(typ), "mask17": f"{m17:05x}", "nbits": int(nbits), "stream": dcamd.hash_words(s, nb)}
    if world == 1:
        out, _ = O.decompress(ct, s, n, bound, typ, m17)
        e["out"] = dcamd.hash_words(out.view(np.uint8))
    else:
        glob, _ = O.decompress(ct, s, world * n, bound, typ, m17)
        e["e2e_outs"] = [dcamd.hash_words(glob[r * n:(r + 1) * n].view(np.uint8)) for r in range(world)]
        del glob
        ranks = []
        for r in range(world):
            if r == 0:
                ss, sb, sp = O.compress(ct, xs[:n], bound, typ, m17)
                sh, m = ss, nbits_of(sb, sp)
            else:
                full, fb, fp = O.compress(ct, xs[r * n - 3:(r + 1) * n], bound, typ, m17)
                _, hb, hp = O.compress(ct, xs[r * n - 3:r * n], bound, typ, m17)
                sh, m = drop_bits(full, nbits_of(fb, fp), nbits_of(hb, hp))
                del full
            o, _ = O.decompress(ct, sh, n, bound, typ, m17)
            ranks.append({"nbits": int(m), "stream": dcamd.hash_words(sh, (m + 7) // 8),
                          "out": dcamd.hash_words(o.view(np.uint8))})
            del sh, o
        e["ranks"] = ranks
    print(f"{key(ct, kind, log2n, bound, world)}: {nbits} bits, {time.time() - t0:.1f} s", flush=True)
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--only", default="", help="comma-separated keys to (re)generate")
    a = ap.parse_args()
    O = Oracle()
    res = json.load(open(OUT)) if os.path.exists(OUT) else {}
    jobs = []
    worlds = [int(w) for w in a.worlds.split(",")]
    if 1 in worlds:
        # bench.py at N = 1: the headline, the size sweep and BASELINE configs 2 / 3 (config 5 decodes the
        # resent copy of the headline's stream)
        jobs += [(7, "u10", 26, 1e-3, 1), (7, "u10", 14, 1e-3, 1), (7, "u10", 18, 1e-3, 1), (7, "u10", 22, 1e-3, 1),
                 (7, "u10", 28, 1e-3, 1), (6, "u10", 26, 1e-3, 1), (7, "eq", 28, 1e-3, 1)]
    jobs += [(7, "u10", 26, 1e-3, w) for w in worlds if w > 1]
    only = set(k for k in a.only.split(",") if k)
    for j in jobs:
        k = key(*j)
        if only and k not in only:
            continue
        res[k] = entry(O, *j)
        json.dump(res, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
