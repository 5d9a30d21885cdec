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


def test_host_asan():
    """The host C of the library under AddressSanitizer + UBSan: `make asan` builds
    tests/native/host_asan_check.c against ASan-instrumented dc_host*.c and runs it (no GPU call)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None or not os.path.exists("/opt/rocm/lib/libamdhip64.so"):
        pytest.skip("gcc / the HIP runtime library not available")
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data-compression_amd")
    r = subprocess.run(["make", "-s", "-C", d, "asan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "host_asan_check: ok" in r.stdout
