"""Issue cost of short instruction sequences on gfx950 (diagnostic; tools/isa_bench2.hip).
Cycles per sequence per SIMD = wall time x in-kernel clock x SIMDs / sequences issued."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libisabench2.so"))
L.seq_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
NAMES = ["v_add_u32", "v_cndmask vcc", "cmp vcc + cndmask vcc", "cmp s + cndmask_e64 s", "sub_co vcc + 2 cndmask vcc",
         "sub_co s + 2 cndmask_e64 s", "lshlrev #3", "lshrrev #3", "v_max_u32", "v_min_u32", "v_sub_u32", "v_or_b32",
         "v_alignbit", "v_bfe #23,#8", "lshlrev v", "lshrrev v", "v_mul_f32", "v_max_f32", "sub+add dep pair",
         "v_cmp vcc", "v_addc_co vcc", "and#31+add+xor"]
ncu = torch.cuda.get_device_properties(0).multi_processor_count
out = torch.zeros(8, dtype=torch.int64, device="cuda")
ms = ctypes.c_float(0)
iters = 4000
for W in (2, 4, 8):
    for op, name in enumerate(NAMES):
        L.seq_run(op, ncu * W, iters, out.data_ptr(), ctypes.byref(ms))
        cyc, real = int(out[0]), int(out[1])
        ghz = cyc / (real * 10.0)                      # memrealtime: 100 MHz
        seqs_per_simd = W * iters * 4 * 8              # W waves per SIMD, 32 sequences per iteration
        c = ms.value * 1e-3 * ghz * 1e9 / seqs_per_simd
        print(f"W={W} {name:28s} {c:6.2f} cyc per sequence per SIMD  ({ms.value:.3f} ms, {ghz:.2f} GHz)")
