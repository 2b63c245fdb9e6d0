"""The C-ABI libraries load (no GPU needed) and export every entry point that
include/consensuscruncher_amd.h declares."""
import ctypes
import os
import re

from consensuscruncher_amd import native

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "consensuscruncher_amd.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b((?:cc|ccio)_[a-z_0-9]+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    io = ctypes.CDLL(os.path.join(native.LIBDIR, "libccio.so"))
    amd = ctypes.CDLL(os.path.join(native.LIBDIR, "libccamd.so"))
    names = declared()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(io if n.startswith("ccio_") else amd, n)]
    assert not missing, missing


def test_bindings_cover_header():
    names = set(declared())
    bound = set(native.IO_SIGS) | set(native.AMD_SIGS)
    assert names == bound, (names - bound, bound - names)


def test_engine_fails_loudly_without_gpu():
    """No CPU fallback: creating a context without a usable GPU raises."""
    import pytest
    from consensuscruncher_amd.engine import Engine
    if os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "") != "-1":
        pytest.skip("a GPU may be present")
    with pytest.raises(native.CCError):
        Engine(0)
