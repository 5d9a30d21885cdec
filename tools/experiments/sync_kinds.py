import os, sys
import numpy as np
sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0, '/root/repo/tools')
import pyoracle as po
from sync_sim import params
O = po.Oracle()
def tok_len(t, P):
    t = t.astype(np.uint64)
    E = ((t >> 23) & 0xFF).astype(np.int64)
    if P["ct"] == 11:
        ln = np.full(t.shape, 32, np.int64)
    else:
        ln = np.clip(E + P["rawadd"], 9, 32)
    if P["ct"] == 6:
        return ln
    if P["ct"] == 7 and P["type"] > 0:
        msk = (t & P["hm"]) == P["hm"]
        lm = ((t >> P["fsh"]) & 1).astype(np.int64) * P["dlm"] + P["lm0"]
        ln = np.where(msk, lm, ln)
    return np.where((t >> 31) & 1 == 1, 3, ln)
def gen(kind, n):
    i = np.arange(n, dtype=np.float64)
    if kind == "sine": x = (np.sin(i * 1e-3) * 50.0 + np.sin(i * 0.37) * 0.5)
    elif kind == "normal": x = np.random.default_rng(1).standard_normal(n)
    elif kind == "ramp": x = i * 1e-4 + np.random.default_rng(2).random(n) * 1e-2
    else: x = O.gen_u10(n)
    x = x.astype(np.float32); return x - x.min()
ct, kind, bound, lg = int(sys.argv[1]), sys.argv[2], float(sys.argv[3]), int(sys.argv[4])
n = 1 << lg
xs = gen(kind, n)
t, m17 = O.type_mask(xs)
s, nbytes, _ = O.compress(ct, xs, bound, t, m17)
P = params(O, bound, t, m17); P["ct"] = ct
if ct != 7: P["type"] = 0
nbits = int(nbytes) * 8
buf = np.zeros(int(nbytes) + 16, np.uint8); buf[:nbytes] = s[:nbytes]
W = np.frombuffer(buf[: (len(buf) // 4) * 4].tobytes(), ">u4").astype(np.uint64)
def window(pos):
    q = np.clip(pos, 0, nbits); wi = q >> 5; sh = (q & 31).astype(np.uint64)
    v = (W[wi] << np.uint64(32)) | W[wi + 1]
    return (v >> (np.uint64(32) - sh)) & np.uint64(0xFFFFFFFF)
# true token boundaries
tb = [0]; pos = np.array([0]); 
# walk from true start collecting boundaries set (bitmap)
true = np.zeros(nbits + 64, bool)
p = 0
lens = []
cur = np.array([0], np.int64)
while cur[0] < nbits:
    true[cur[0]] = True
    cur += tok_len(window(cur), P)
print(f"{kind} ct{ct} @{bound:g} 2^{lg}: {nbits/n:.2f} bits/value")
# sample starting points, measure distance (bits) until hitting a true boundary
rng = np.random.default_rng(0)
starts = rng.integers(0, nbits - 200000, 4000)
pos = starts.copy(); dist = np.full(len(starts), -1, np.int64)
live = np.ones(len(starts), bool)
for step in range(20000):
    m = live
    if not m.any(): break
    hit = true[pos] & m
    dist[hit] = pos[hit] - starts[hit]
    live &= ~hit
    pos[live] += tok_len(window(pos[live]), P)
never = (dist < 0).sum()
d = dist[dist >= 0]
print(f"  sync distance bits: median {np.median(d) if len(d) else -1:.0f} p90 {np.percentile(d,90) if len(d) else -1:.0f} p99 {np.percentile(d,99) if len(d) else -1:.0f} max {d.max() if len(d) else -1}; never (20000 tokens) {never}/{len(starts)}")
