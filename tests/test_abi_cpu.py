"""CPU-side checks of the boundary: the C-ABI library loads and exports every
symbol include/tmatch.h declares; the product refuses to run without a GPU."""
import re
from pathlib import Path

import pytest

from emqx_amd import _native, build

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    src = (ROOT / "include" / "tmatch.h").read_text()
    return set(re.findall(r"^\s*(?:int|uint32_t|const char \*)\s*\*?\s*(tm_\w+)\s*\(", src, re.M))


def test_header_and_binding_agree():
    assert declared_symbols() == set(_native.EXPORTS)


def test_library_exports_every_symbol():
    build.build_tmatch()
    lib = _native.load_library()
    for name in _native.EXPORTS:
        assert hasattr(lib, name), name
    assert lib.tm_abi_version() >> 16 == 1


def test_kernels_are_gfx950_code_objects():
    import subprocess
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(build.LIB_TMATCH)],
                         capture_output=True, text=True).stdout + \
        subprocess.run(["strings", str(build.LIB_TMATCH)], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_no_gpu_means_loud_failure(monkeypatch):
    monkeypatch.setattr(_native, "_gpu_present", lambda: False)
    with pytest.raises(_native.NativeUnavailable):
        _native.Index()


def test_null_handle_is_einval():
    lib = _native.load_library()
    assert lib.tm_destroy(None) == _native.TM_EINVAL
    assert lib.tm_apply_deltas(None, 0, None, None, None, None, None) == _native.TM_EINVAL
    assert lib.tm_match_batch(None, 0, None, None, None, None, 0, None) == _native.TM_EINVAL
    assert lib.tm_host_alloc(None, 16, None) == _native.TM_EINVAL
    assert lib.tm_host_free(None, None) == _native.TM_EINVAL
