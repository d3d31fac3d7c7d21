"""CPU checks of the drop-in boundary: the library loads and exports every declared symbol,
the ctypes signature table matches the header, and argument validation works without a GPU."""

import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "vmatting.h")
LIB = os.path.join(REPO, "video-matting_amd", "vmatting", "libvmatting.so")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vm_[a-z0-9_]+)\s*\(", src)))


def test_library_built_for_gfx950():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    data = open(LIB, "rb").read()
    assert b"gfx950" in data


def test_every_declared_symbol_is_exported():
    lib = ctypes.CDLL(LIB)
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s


def test_ctypes_table_matches_header():
    from vmatting import _lib
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == declared_symbols()


def test_abi_version_and_error_path():
    from vmatting import _lib
    lib = _lib.lib()
    assert lib.vm_abi_version() == _lib.ABI_VERSION
    # argument validation happens before any HIP call: NULL tensors -> VM_EINVAL + message
    rc = lib.vm_conv3x3_nhwc(None, None, 3, 64, None, None, None, 0, None, None)
    assert rc == _lib.VM_EINVAL
    assert b"conv3x3" in lib.vm_last_error()
    with pytest.raises(ValueError):
        _lib.check(rc, "conv3x3")
    assert lib.vm_conv3x3_packed_bytes(7, 64, _lib.VM_BF16) == 64 * 128 * 2  # cin 7->8, K 72->128, cout 64
    assert lib.vm_conv3x3_packed_bytes(512, 512, _lib.VM_F32) == 512 * 4608 * 4
    assert lib.vm_conv3x3_packed_bytes(0, 1, 0) == 0


def test_status_codes_map_to_reference_exceptions():
    from vmatting import _lib
    with pytest.raises(IndexError):
        _lib.check(_lib.VM_EINDEX, "fb")
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.VM_EUNSUPPORTED, "x")
    with pytest.raises(RuntimeError):
        _lib.check(_lib.VM_EHIP, "x")


def test_ops_refuse_cpu_tensors():
    """The product never computes on the CPU: host tensors are rejected, not silently handled."""
    import torch
    from vmatting import ops
    with pytest.raises(TypeError):
        ops.maxpool2x2(torch.zeros(1, 4, 4, 8))


def test_raw_stream_falls_back_to_public_getter(monkeypatch):
    """if a torch release drops the private stream getters, every launch still gets the current stream's
    handle, from torch.cuda.current_stream(d).cuda_stream (no GPU needed: the public call is stubbed)."""
    import torch
    from vmatting import _lib

    class FakeStream:
        cuda_stream = 0x1234

    seen = []
    monkeypatch.setattr(_lib, "_GET_RAW_STREAM", None)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda d=None: seen.append(d) or FakeStream())
    assert _lib.current_raw_stream() == 0x1234
    assert _lib.current_raw_stream(3) == 0x1234
    assert seen == [None, 3]


@pytest.mark.gpu
@pytest.mark.skipif(not __import__("conftest").gpu_available(), reason="needs a ROCm GPU")
def test_raw_stream_matches_public_getter():
    """The private getters return torch.cuda.current_stream().cuda_stream, outside and inside a stream context."""
    import torch
    from vmatting import _lib
    assert _lib.current_raw_stream() == torch.cuda.current_stream().cuda_stream
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        assert _lib.current_raw_stream() == s.cuda_stream == torch.cuda.current_stream().cuda_stream
        assert _lib.current_raw_stream(torch.cuda.current_device()) == s.cuda_stream
    assert _lib.current_raw_stream() == torch.cuda.current_stream().cuda_stream != s.cuda_stream
