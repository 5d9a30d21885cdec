"""CPU model of parse3's self-synchronisation (test/analysis tool, uses the oracle as the stream source).

Every parse segment (SEG x 256 bits) is entered by a walk that starts PRE bits before it; the walk's
first token boundary inside the segment is the segment's recorded entry.  A link is broken when that
entry differs from the previous segment's exit; parse3 then re-walks the segment from the true entry
until the walk meets the recorded chunk entries again.  This prints how often links break and how many
tokens / chunks the repairs take, for a few pre-walk lengths.

    [CT=6|7] python3 tools/sync_sim.py [log2n] [seg]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import pyoracle as po  # noqa: E402


def params(O, bound, type_, mask17):
    B = O.bound_binary(bound)
    m = B + ((mask17 >> 8) & 0xFF) - 127
    mm = min(max(m, 0), 23)
    mm0 = mm - 8 if mm > 8 else 0
    return dict(ct=7, rawadd=B - 118, hm=(((1 << type_) - 1) << (31 - type_)) if type_ > 0 else 0, fsh=30 - type_,
                lm0=type_ + 2 + mm0, dlm=mm - mm0, type=type_)


def tok_len(t, P):
    t = t.astype(np.uint64)
    E = ((t >> 23) & 0xFF).astype(np.int64)
    ln = np.clip(E + P["rawadd"], 9, 32)
    if P["ct"] == 6:
        return ln
    if P["type"] > 0:
        msk = (t & P["hm"]) == P["hm"]
        lm = ((t >> P["fsh"]) & 1).astype(np.int64) * P["dlm"] + P["lm0"]
        ln = np.where(msk, lm, ln)
    return np.where((t >> 31) & 1 == 1, 3, ln)


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    seg = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    ct = int(os.environ.get("CT", "7"))
    O = po.Oracle()
    n = 1 << lg
    xs = O.gen_u10(n)
    if len(sys.argv) <= 3 or sys.argv[3] != 'raw':
        xs = O.to_small(xs)[1]                 # x - min, as bench.py's workload
    t, m17 = O.type_mask(xs)
    s, nbytes, _ = O.compress(ct, xs, 1e-3, t, m17)
    P = params(O, 1e-3, t, m17)
    P["ct"] = ct
    if ct == 6:
        P["type"] = 0
    nbits = int(nbytes) * 8
    buf = np.zeros(int(nbytes) + 16, np.uint8)
    buf[:nbytes] = np.asarray(s[:nbytes], np.uint8)
    W = np.frombuffer(buf[: (len(buf) // 4) * 4].tobytes(), ">u4").astype(np.uint64)

    def window(pos):                          # the 32 stream bits from bit pos, MSB-first
        q = np.clip(pos, 0, nbits)
        wi = q >> 5
        sh = (q & 31).astype(np.uint64)
        v = (W[wi] << np.uint64(32)) | W[wi + 1]
        return (v >> (np.uint64(32) - sh)) & np.uint64(0xFFFFFFFF)

    L = seg * 256
    nseg = (nbits + L - 1) // L
    starts = np.arange(nseg, dtype=np.int64) * L
    print(f"n 2^{lg} stream {nbytes} B ({nbits / n:.2f} bits/value) type {t} segments {nseg} of {seg} chunks")
    for pre in (512, 768, 1024, 1536, 2048):
        pos = np.maximum(starts - pre, 0)
        pos[0] = 0
        # walk to the segment start, then record chunk entries for the whole segment
        ent = np.zeros((nseg, seg), np.int64)
        for c in range(seg + 1):
            lim = starts + c * 256
            while True:
                m = pos < lim
                if not m.any():
                    break
                pos[m] += tok_len(window(pos[m]), P)
            if c < seg:
                ent[:, c] = pos - lim
        exitp = pos - (starts + L)           # entry of the next segment relative to its start
        bad = np.nonzero(ent[1:, 0] != exitp[:-1])[0] + 1
        # repairs: walk from the true entry until a chunk entry matches the record
        steps = np.zeros(len(bad), np.int64)
        chunks = np.zeros(len(bad), np.int64)
        rp = starts[bad] + exitp[bad - 1]
        live = np.ones(len(bad), bool)
        for c in range(1, seg + 1):
            lim = starts[bad] + c * 256
            while True:
                m = live & (rp < lim)
                if not m.any():
                    break
                rp[m] += tok_len(window(rp[m]), P)
                steps[m] += 1
            if c < seg:
                met = live & (rp - lim == ent[bad, c])
                chunks[live] = c
                live &= ~met
        chunks[live] = seg
        never = int(live.sum())
        jobs = (nseg + 63) // 64
        badjobs = len(np.unique(bad // 64))
        print(f"pre {pre:5d}: broken links {len(bad)} ({100 * len(bad) / nseg:.3f}%), jobs with a repair "
              f"{badjobs}/{jobs} ({100 * badjobs / jobs:.1f}%), repair tokens mean {steps.mean() if len(bad) else 0:.1f} "
              f"max {steps.max() if len(bad) else 0}, chunks walked mean {chunks.mean() if len(bad) else 0:.2f}, "
              f"never met {never}; walks per token {(pre + L) / L:.3f}")
        if len(bad):
            h = np.bincount(np.minimum(chunks, seg), minlength=seg + 1)
            print("   chunks-walked histogram:", h.tolist())


if __name__ == "__main__":
    main()
