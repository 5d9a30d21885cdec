"""CPU-side checks of the product library: it builds, loads and exports every C-ABI symbol
declared in include/*.h (no compute call: there is no GPU in the dev container)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    import dcamd
    L = dcamd.Lib()
    for sym in dcamd.ABI_SYMBOLS + dcamd.EXT_SYMBOLS:
        assert hasattr(L.L, sym), sym
    # every function prototype in include/*.h is exported
    for h in ("dc_gpu.h", "dataCompression.h"):
        path = os.path.join(ROOT, "include", h)
        if not os.path.exists(path):
            continue
        src = open(path).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for name in re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", src):
            if name in ("if", "while", "for", "sizeof", "return"):
                continue
            assert hasattr(L.L, name), f"{h}: {name} not exported"
