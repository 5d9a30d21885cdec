"""Self-synchronisation statistics of the bit-wise token grammar (diagnostic, not a test).

For a stream produced by the oracle encoder, start a parse at random bit offsets and count the tokens
until the parse lands on a true token boundary, (a) plain, (b) "pruned": a token that the encoder can
never emit at this bound / mask (a raw token whose whole binade is zero-coded, a CT7 raw token with
the mask's exponent, a raw exponent above the CT7 type's range) makes the walk slide one bit instead
of taking the token.  The parse kernels use (b) for their speculative pre-walks.

usage: python tools/sync_stats.py [ct] [u10|eq|himeno|ramp] [log2n]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from pyoracle import Oracle  # noqa: E402


def main():
    ct = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    kind = sys.argv[2] if len(sys.argv) > 2 else "u10"
    lg = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    bound = 1e-3
    O = Oracle()
    n = 1 << lg
    if kind == "u10":
        x = O.gen_u10(n)
    elif kind == "eq":
        x = np.full(n, np.float32(0.123456789), np.float32)
    elif kind == "himeno":
        x = O.gen_himeno_plane()
    else:
        x = (np.arange(n, dtype=np.float32) * np.float32(0.0005)).astype(np.float32)
    mn, xs = O.to_small(x)
    mean, typ = O.med(xs)
    m17 = O.mask17(mean)
    s, nb, pos = O.compress(ct, xs, bound, typ, m17)
    bits = np.unpackbits(np.frombuffer(bytes(s) + b"\0" * 64, np.uint8))
    B = O.bound_binary(bound)
    thr_lt, thr_le = O.thr(bound)
    mm = min(max(B + ((m17 >> 8) & 0xFF) - 127, 0), 23)
    mm0 = max(mm - 8, 0)
    # type range: max < 2^(sum_{k=i}^{7} 2^k - 127), i = 8 - type
    emax = 255
    if ct == 7:
        i = 8 - typ
        emax = min(255, sum(1 << k for k in range(i, 8)) - 1)   # exponent of max < 2^(S-127): E <= S-1

    def tok(p):
        w = 0
        for k in range(10):
            w = (w << 1) | int(bits[p + k])
        first = w >> 9
        E = (w >> 1) & 0xFF
        if ct != 6 and first:
            return 3, True
        if ct == 7:
            head = (w >> (9 - typ)) & ((1 << typ) - 1)
            if (w >> 9) == 0 and head == (1 << typ) - 1:
                flag = (w >> (8 - typ)) & 1
                return typ + 2 + (mm if flag else mm0), True
        ln = 32 if ct == 11 else 9 + min(max(B + E - 127, 0), 23)
        if ct == 6:
            return ln, first == 0
        maxv = np.array([(E << 23) | 0x7FFFFF], np.uint32).view(np.float32)[0]
        valid = not (maxv <= thr_lt)
        if ct == 7 and E == ((m17 >> 8) & 0xFF) and (m17 >> 16) == 0:
            valid = False
        if ct == 7 and E > emax:
            valid = False
        return ln, valid

    nbits = nb * 8
    truth = np.zeros(nbits + 64, bool)
    p = 0
    while p < nbits:
        truth[p] = True
        p += tok(p)[0]
    rng = np.random.default_rng(1)
    def slide(p):                      # to the next '1' bit within the token's first 9 bits
        for k in range(1, 9):
            if bits[p + k]:
                return k
        return 9

    for prune in (0, 1, 2):
        res = []
        for _ in range(2000):
            p = int(rng.integers(0, max(nbits - 4096, 1)))
            k = 0
            while not truth[p] and k < 5000:
                ln, ok = tok(p)
                p += ln if (ok or not prune) else (1 if prune == 1 else slide(p))
                k += 1
            res.append(k)
        r = np.array(res)
        print(f"CT{ct} {kind} 2^{lg} {['plain ', 'prune+1', 'prune>1'][prune]}: steps to sync mean {r.mean():.1f} "
              f"p99 {np.percentile(r, 99):.0f} p99.9 {np.percentile(r, 99.9):.0f} max {r.max()}  "
              f"(stream {nb} B, {nbits / n:.2f} bits/elem)")


if __name__ == "__main__":
    main()
