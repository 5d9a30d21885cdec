"""Generate the golden fixtures in tests/golden/ from the compiled reference (oracle/_ref).

Run in the dev container (needs /root/reference for the inputs that come from the reference
tree and oracle/_ref/libref_<bound>.so built by oracle/build_ref.sh):

    python tests/golden/make_golden.py

Outputs (data only -- inputs and the reference's outputs, no reference source):
  golden_<bound>.npz   per bound: for every case and CT 5/6/7/11 the reference stream, bytes, pos,
                       type, mask17, the reference decoder's output and whether it is
                       self-consistent; CT1 arrays; CRC32 of every stream; Hamming blocks.
  kat_*                KAT files copied verbatim from the reference tree (impl/dataset, tools).
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
    ins = {
        "testfloat": np.loadtxt(os.path.join(ds, "testfloat_8_8_128.txt"), dtype=np.float32),
        "rand16k": np.loadtxt(os.path.join(ds, "float_rand_16384.txt"), dtype=np.float32),
        "u10_16k": O.gen_u10(1 << 14),
        "eq16k": np.full(1 << 14, np.float32(0.123456789)),
        "himeno": O.gen_himeno_plane(256, 256),
        "unit64k": np.random.RandomState(42).rand(65536).astype(np.float32),   # Q1 case
        "q2": np.full(8, np.float32(0.0015)),
        "ramp20k": (np.float32(0.0005) * np.arange(20000, dtype=np.float32)).astype(np.float32),
    }
    rs = np.random.RandomState(7)
    edge = np.concatenate([
        np.zeros(5, np.float32),
        np.array([1e-45, 1e-40, 1e-38, 1.2e-38, 3e-39], np.float32),      # subnormals
        rs.rand(200).astype(np.float32) * np.float32(1e-3),
        rs.rand(200).astype(np.float32) * np.float32(3.0),
        rs.rand(200).astype(np.float32) * np.float32(1e5),                 # m = 23 tokens at 1e-3
        np.array([8192.0, 16384.5, 2.0, 1.0, 0.5, 0.25, 1e6, 3e7], np.float32),
        np.repeat(np.float32(2.5), 50),                                     # predictable runs
        np.linspace(0, 5, 300).astype(np.float32),
    ])
    ins["edge"] = edge
    return ins


def ref_consistent(O, ct, stream, n, bound, t, m17, dec_ref):
    spec, got = O.decompress(ct, stream, n, bound, t, m17)
    cref, ncref, stuck = O.decompress_cref(ct, stream, n, bound, t, m17)
    return bool(stuck == 0 and ncref == n and got == n and
                np.array_equal(spec.view(np.uint32), dec_ref.view(np.uint32)))


def ref_decode_safe(bound, ct, stream, n, t, m17):
    """Run the reference decoder in a child process: on quirk streams it may corrupt its heap."""
    code = (
        "import sys,numpy as np;sys.path.insert(0,%r);from pyoracle import RefLib;"
        "s=np.frombuffer(sys.stdin.buffer.read(),np.uint8);"
        "out=RefLib(%r).decompress(%d,s,%d,%d,%d);sys.stdout.buffer.write(out.tobytes())"
        % (os.path.join(ROOT, "oracle"), bound, ct, n, t, m17))
    p = subprocess.run([sys.executable, "-c", code], input=stream.tobytes(), capture_output=True)
    if p.returncode != 0 or len(p.stdout) != 4 * n:
        return None
    return np.frombuffer(p.stdout, np.float32).copy()


def main():
    O = Oracle()
    ins = inputs(O)
    for bound in (1e-3, 1e-6):
        R = RefLib(bound)
        rec = {}
        for name, x in ins.items():
            rec[f"{name}/input"] = x
            mn, xs = R.to_small(x)
            mean, t = R.med(xs)
            m17 = O.mask17(mean)
            rec[f"{name}/min"] = np.float32(mn)
            rec[f"{name}/mean"] = np.float32(mean)
            rec[f"{name}/type"] = np.int32(t)
            rec[f"{name}/mask17"] = np.uint32(m17)
            for ct in (5, 6, 7, 11):
                s, nb, pos = R.compress(ct, xs, t, m17)
                key = f"{name}/ct{ct}"
                rec[key + "/stream"] = s
                rec[key + "/pos"] = np.int32(pos)
                rec[key + "/crc"] = np.uint32(R.crc32(s))
                dec = ref_decode_safe(bound, ct, s, xs.size, t, m17)
                ok = dec is not None and ref_consistent(O, ct, s, xs.size, bound, t, m17, dec)
                rec[key + "/ref_consistent"] = np.bool_(ok)
                if dec is not None:
                    rec[key + "/ref_decoded"] = dec
                print(f"{bound:g} {name:10s} ct{ct:2d} bytes={nb:7d} pos={pos} type={t} consistent={ok}")
            raw, codes, p1 = R.bytewise(x)
            rec[f"{name}/ct1/raw"] = raw
            rec[f"{name}/ct1/codes"] = np.frombuffer(codes, np.uint8).copy()
            rec[f"{name}/ct1/pos"] = p1
        # append mode: two consecutive calls into one stream (add_bit_to_bytes append semantics)
        x = ins["edge"]
        mn, xs = R.to_small(x)
        import ctypes as C
        for ct in (5, 6, 11):
            p = C.c_void_p(None); nb = C.c_int(0); pos = C.c_int(8)
            a, b = np.ascontiguousarray(xs[:333]), np.ascontiguousarray(xs[333:])
            fn = {5: R.L.myCompress_bitwise, 6: R.L.myCompress_bitwise_np, 11: R.L.myCompress_bitwise_op}[ct]
            fn(a, a.size, C.byref(p), C.byref(nb), C.byref(pos))
            rec[f"append/ct{ct}/first_bytes"] = np.int32(nb.value)
            rec[f"append/ct{ct}/first_pos"] = np.int32(pos.value)
            fn(b, b.size, C.byref(p), C.byref(nb), C.byref(pos))
            rec[f"append/ct{ct}/stream"] = np.frombuffer(C.string_at(p.value, nb.value), np.uint8).copy()
            rec[f"append/ct{ct}/pos"] = np.int32(pos.value)
        rec["append/input"] = xs
        # Hamming over BER=1e-6 blocks of a >= 125,000-byte stream (CT10 = CT5 stream + CRC + Hamming)
        u = O.gen_u10(1 << 16)
        mn, xs = R.to_small(u)
        s, nb, pos = R.compress(5, xs)
        bs = int(R.L.block_size(nb))
        rec["hamming/stream"] = s
        rec["hamming/block_size"] = np.int32(bs)
        nblk = (nb + bs - 1) // bs
        for i in range(nblk):
            blk = s[i * bs: min(nb, (i + 1) * bs)]
            r, c = R.hamming_encode(blk)
            rec[f"hamming/r{i}"] = np.int32(r)
            rec[f"hamming/c{i}"] = np.frombuffer(c, np.uint8).copy()
            print(f"hamming block {i}: {blk.size} B r={r}")
        path = os.path.join(OUT, "golden_%g.npz" % bound)
        np.savez_compressed(path, **rec)
        print("wrote", path, os.path.getsize(path))
    # KAT files shipped in the reference tree (data files, copied verbatim)
    for src, dst in [
        ("impl/dataset/testfloat_8_8_128.txt", "kat_testfloat_8_8_128.txt"),
        ("impl/dataset/testfloat_8_8_128.txt.bc", "kat_testfloat_8_8_128.txt.bc"),
        ("impl/dataset/testfloat_8_8_128.txt.bc.txt", "kat_testfloat_8_8_128.txt.bc.txt"),
        ("tools/float_eq_8192.txt.bc", "kat_float_eq_8192.txt.bc"),
    ]:
        shutil.copyfile(os.path.join(REF, src), os.path.join(OUT, dst))


if __name__ == "__main__":
    main()
