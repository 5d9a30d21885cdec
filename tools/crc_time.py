"""Diagnostic (not a test): average time of dc_crc32_device_async over a 163 MB device buffer."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "data-compression_amd"))
import torch, dcamd
L = dcamd.Lib(); L.init(0)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 162634383
s = torch.randint(0, 255, (nb + 64,), dtype=torch.uint8, device="cuda")
crc = torch.zeros(4, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
ls = torch.cuda.ExternalStream(L.L.dc_get_stream())
for _ in range(3):
    L.crc32_device_async(s.data_ptr(), nb, crc.data_ptr())
L.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(ls)
for _ in range(20):
    L.crc32_device_async(s.data_ptr(), nb, crc.data_ptr())
e1.record(ls)
L.synchronize(); torch.cuda.synchronize()
print(os.environ.get("DCAMD_LIB", "lib"), "crc us per pass", round(e0.elapsed_time(e1) * 1000 / 20, 2))
