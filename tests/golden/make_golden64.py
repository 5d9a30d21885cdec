"""Generate the DOUBLE-codec golden fixtures in tests/golden/ from the compiled reference (oracle/_ref).

Run in the dev container (needs /root/reference and oracle/_ref/libref_<bound>.so):

    python tests/golden/make_golden64.py

Outputs (data only -- inputs and the reference's outputs, no reference source):
  golden64_<bound>.npz  per bound: for every case and CT 5/6/7/11 the stream of
                        myCompress_bitwise_double{,_np,_mask,_op} (impl/dataCompression.c:3189,
                        :2633, :1590, :355), bytes, pos, type, mask20, the reference decoder's output
                        (run in a child process: on quirk streams it corrupts its heap) and whether
                        it is self-consistent (equal to the grammar decoder); CT1 arrays of
                        myCompress_double (:3815); append-mode streams.
  kat64_*               the reference tree's double KATs, copied verbatim: the binary inputs (.bi),
                        the streams (.bc: CT6 / CT11 at absErrorBound 1e-6) and the decoded text.
"""
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from pyoracle import Oracle, RefLib  # noqa: E402

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def inputs(O):
    ds = os.path.join(REF, "impl", "dataset")
    rs = np.random.RandomState(11)
    ins = {
        "testdouble": np.fromfile(os.path.join(ds, "testdouble_8_8_128.txt.bi"), np.float64),
        "u10_16k": O.gen_u10_64(1 << 14),
        "eq16k": np.full(1 << 14, 0.123456789),
        "unit32k": rs.rand(1 << 15),                                  # mean ~0.5: the Q1 analogue for CT7
        "q2": np.full(8, 0.0015),
        "ramp20k": 0.0005 * np.arange(20000, dtype=np.float64),
        "mixed": np.concatenate([np.full(700, 2.5), O.gen_u10_64(900), np.arange(600) * 1e-4,
                                 rs.rand(500) * 1e5, rs.rand(300) * 1e200]),
    }
    ins["edge"] = np.concatenate([
        np.zeros(5),
        np.array([5e-324, 1e-310, 2.2e-308, 1e-300]),                 # subnormals / tiny
        rs.rand(200) * 1e-3, rs.rand(200) * 3.0,
        rs.rand(200) * 1e15,                                          # m = 52 tokens
        np.array([8192.0, 16384.5, 2.0, 1.0, 0.5, 0.25, 1e6, 3e7, 1e300]),
        np.repeat(2.5, 50), np.linspace(0, 5, 300),
    ])
    return ins


def ref_decode_safe(bound, ct, stream, n, t, m20):
    code = (
        "import sys,numpy as np;sys.path.insert(0,%r);from pyoracle import RefLib;"
        "s=np.frombuffer(sys.stdin.buffer.read(),np.uint8);"
        "out=RefLib(%r).decompress64(%d,s,%d,%d,%d);sys.stdout.buffer.write(out.tobytes())"
        % (os.path.join(ROOT, "oracle"), bound, ct, n, t, m20))
    p = subprocess.run([sys.executable, "-c", code], input=stream.tobytes(), capture_output=True)
    if p.returncode != 0 or len(p.stdout) != 8 * n:
        return None
    return np.frombuffer(p.stdout, np.float64).copy()


def main():
    O = Oracle()
    ins = inputs(O)
    for bound in (1e-3, 1e-6):
        R = RefLib(bound)
        rec = {}
        for name, x in ins.items():
            rec[f"{name}/input"] = x
            mn, xs = R.to_small64(x)
            mean, t = R.med64(xs)
            m20 = O.mask20(mean)
            rec[f"{name}/min"] = np.float64(mn)
            rec[f"{name}/mean"] = np.float64(mean)
            rec[f"{name}/type"] = np.int32(t)
            rec[f"{name}/mask20"] = np.uint32(m20)
            for ct in (5, 6, 7, 11):
                s, nb, pos = R.compress64(ct, xs, t, m20)
                key = f"{name}/ct{ct}"
                rec[key + "/stream"] = s
                rec[key + "/pos"] = np.int32(pos)
                dec = ref_decode_safe(bound, ct, s, xs.size, t, m20)
                spec, got = O.decompress64(ct, s, xs.size, bound, t, m20)
                ok = dec is not None and got == xs.size and np.array_equal(spec.view(np.uint64), dec.view(np.uint64))
                rec[key + "/ref_consistent"] = np.bool_(ok)
                if dec is not None:
                    rec[key + "/ref_decoded"] = dec
                print(f"{bound:g} {name:10s} ct{ct:2d} bytes={nb:7d} pos={pos} type={t} consistent={ok}")
            raw, codes, p1 = R.bytewise64(x)                   # CT1: myCompress_double (:3815)
            rec[f"{name}/ct1/raw"] = raw
            rec[f"{name}/ct1/codes"] = np.frombuffer(codes, np.uint8).copy()
            rec[f"{name}/ct1/pos"] = p1
        x = ins["edge"]
        mn, xs = R.to_small64(x)
        import ctypes as C
        for ct in (5, 6, 11):
            p = C.c_void_p(None); nb = C.c_int(0); pos = C.c_int(8)
            a, b = np.ascontiguousarray(xs[:333]), np.ascontiguousarray(xs[333:])
            fn = getattr(R.L, "myCompress_bitwise_double" + R._D[ct])
            fn(a, a.size, C.byref(p), C.byref(nb), C.byref(pos))
            rec[f"append/ct{ct}/first_bytes"] = np.int32(nb.value)
            rec[f"append/ct{ct}/first_pos"] = np.int32(pos.value)
            fn(b, b.size, C.byref(p), C.byref(nb), C.byref(pos))
            rec[f"append/ct{ct}/stream"] = np.frombuffer(C.string_at(p.value, nb.value), np.uint8).copy()
            rec[f"append/ct{ct}/pos"] = np.int32(pos.value)
        rec["append/input"] = xs
        path = os.path.join(OUT, "golden64_%g.npz" % bound)
        np.savez_compressed(path, **rec)
        print("wrote", path, os.path.getsize(path))
    for src, dst in [
        ("impl/dataset/testdouble_8_8_128.txt.bi", "kat64_testdouble_8_8_128.bi"),
        ("impl/dataset/testdouble_8_8_128.txt.bc", "kat64_testdouble_8_8_128.bc"),
        ("impl/dataset/testdouble_8_8_128.txt.bnp.txt", "kat64_testdouble_8_8_128.bnp.txt"),
        ("impl/dataset/testdouble_8_8_8_128.txt.bi", "kat64_testdouble_8_8_8_128.bi"),
        ("impl/dataset/testdouble_8_8_8_128.txt.bc", "kat64_testdouble_8_8_8_128.bc"),
        ("impl/dataset/testdouble_8_8_8_128.txt.bop.txt", "kat64_testdouble_8_8_8_128.bop.txt"),
    ]:
        shutil.copyfile(os.path.join(REF, src), os.path.join(OUT, dst))


if __name__ == "__main__":
    main()
