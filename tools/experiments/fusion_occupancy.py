"""Experiment: how parse3 and decode3 slow down when they get fewer resident waves --
the residency a single parse + decode launch would leave each phase.  CT7 U10 2^26 at 1e-3, the library's
per-kernel HIP events, 10 decodes per setting.  Usage: python tools/experiments/fusion_occupancy.py"""
import ctypes, os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import sys, os, json, ctypes
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "data-compression_amd"))
import torch, dcamd
L = dcamd.Lib(); L.init(0); L.set_bound(1e-3)
n = 1 << 26
x = torch.from_numpy(dcamd.gen_u10(n)).cuda()
xs = torch.empty_like(x)
mn = ctypes.c_float(0)
L.check(L.L.dc_to_small_device(ctypes.c_void_p(x.data_ptr()), n, ctypes.c_void_p(xs.data_ptr()), ctypes.byref(mn)), "ts")
mean, t = L.med_device(xs.data_ptr(), n)
m17 = int(np.array([mean], np.float32).view(np.uint32)[0] >> 15)
cap = L.stream_capacity(n)
st = torch.empty(cap, dtype=torch.uint8, device="cuda"); out = torch.empty(n, dtype=torch.float32, device="cuda")
d_nb = torch.zeros(1, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
L.encode_device(7, xs.data_ptr(), n, st.data_ptr(), type_=t, mask17=m17, total_ptr=d_nb.data_ptr())
L.encode_result()
for _ in range(3):
    L.decode_device(7, st.data_ptr(), -1, n, out.data_ptr(), type_=t, mask17=m17, d_nbits=d_nb.data_ptr(), max_bytes=cap)
    L.decode_finish()
K = 10
L.L.dc_timing_enable(K)
for _ in range(K):
    L.decode_device(7, st.data_ptr(), -1, n, out.data_ptr(), type_=t, mask17=m17, d_nbits=d_nb.data_ptr(), max_bytes=cap)
L.synchronize()
status = L.decode_status()
L.decode_finish()
ms = np.zeros((K, 6))
for k in range(K):
    buf = (ctypes.c_float * 6)()
    L.L.dc_timing_read(k, buf)
    ms[k] = np.frombuffer(buf, np.float32)
L.L.dc_timing_enable(0)
m = ms.mean(axis=0)
print(json.dumps({"parse3_us": round(float(m[3]) * 1e3, 1), "decode3_us": round(float(m[5]) * 1e3, 1), "status": status}))
'''

def run(env):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=e, capture_output=True, text=True, timeout=240)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return json.loads(line[-1]) if line else {"error": r.stderr[-400:]}

print("# parse3 / decode3 at CT7 U10 2^26 @1e-3 with capped residency (per CU): DC_P3_PER_CU parse waves,")
print("# DC_D3_PER_CU decode workgroups of 4 waves; default: parse 24 (LDS), decode 4 (VGPRs)", flush=True)
print("default", run({}), flush=True)
for p in (4, 8, 12, 16, 20):
    print(f"parse waves/CU {p}", run({"DC_P3_PER_CU": str(p)}), flush=True)
for d in (1, 2, 3):
    print(f"decode WGs/CU {d} ({4 * d} waves)", run({"DC_D3_PER_CU": str(d)}), flush=True)
