"""Per-instruction VALU issue cost and LDS latency on gfx950 (diagnostic; tools/isa_bench.hip).

Prints, for W waves per SIMD, the cycles per wave-instruction per SIMD: median over waves of
(s_memtime elapsed) / (instructions the wave issued), divided by W (the W waves share the SIMD)."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libisabench.so"))
L.isa_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                      ctypes.POINTER(ctypes.c_float)]
NAMES = ["v_add_u32", "v_xor_b32", "v_lshlrev_b32", "v_alignbit_b32", "v_bfe_u32", "v_cndmask_b32",
         "v_med3_i32", "v_lshl_or_b32", "v_and_or_b32", "v_add3_u32", "v_perm_b32", "v_add_f32", "v_fma_f32",
         "v_min3_f32", "v_pk_add_f32", "v_lshlrev_b64", "v_sub_co_u32", "v_cmp_gt_u32", "v_mul_lo_u32",
         "v_mad_u32_u24", "v_bcnt_u32_b32", "v_ffbh_u32", "v_mov_dpp", "v_add_u32_dpp", "v_pk_add_u16",
         "v_lshrrev_b32", "v_sub_f32", "v_cmp_lt_f32", "v_add_lshl_u32", "v_pk_mul_f32", "v_max_u32",
         "v_and_b32", "v_cndmask_e64", "v_mov_b32"]
ncu = torch.cuda.get_device_properties(0).multi_processor_count
out = torch.zeros(ncu * 8 * 4 * 2 + 16, dtype=torch.int64, device="cuda")
ms = ctypes.c_float(0)
iters = 2000


def run(op, lds, W, per_iter):
    grid = ncu * W
    L.isa_run(op, lds, grid, iters, out.data_ptr(), ctypes.byref(ms))   # warm
    L.isa_run(op, lds, grid, iters, out.data_ptr(), ctypes.byref(ms))
    cyc = out[: grid * 4 * 2: 2].float().cpu()
    med = float(cyc.median())
    return med / (iters * per_iter), ms.value


for W in (1, 2, 4):
    for op, name in enumerate(NAMES):
        c, t = run(op, 0, W, 64)
        print(f"W={W} {name:16s} {c:6.2f} cyc/instr/wave  -> {c / W:5.2f} cyc per wave-instr per SIMD  ({t:.3f} ms)")
    sys.stdout.flush()
for W in (1, 4):
    c, _ = run(0, 1, W, 8)
    print(f"W={W} ds_read_b32 dependent chain: {c:6.1f} cyc per read")
    c, _ = run(1, 1, W, 64)
    print(f"W={W} ds_read_b32 8 chains: {c:6.2f} cyc per read per wave -> {c / W:5.2f} per SIMD")
    c, _ = run(2, 1, W, 64)
    print(f"W={W} ds_or_b32 8 per step: {c:6.2f} cyc per op per wave -> {c / W:5.2f} per SIMD")
