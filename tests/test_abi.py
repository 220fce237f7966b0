"""CPU checks of the drop-in boundary: the gfx950 library builds/loads, exports
every symbol include/ymerge.h declares, and fails loudly (no CPU fallback)
without a GPU."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, gpu_available

HDR = os.path.join(ROOT, "include", "ymerge.h")
LIB = os.path.join(ROOT, "y-crdt_amd", "lib", "libymerge.so")


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b(y\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_boundary():
    names = declared_functions()
    for must in ["ymerge_updates_v1", "ydiff_updates_v1", "yencode_state_vector_from_update_v1",
                 "ybinary_destroy", "ymerge_updates_v1_batch_device", "ymerge_ctx_create"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_library_targets_gfx950():
    data = open(LIB, "rb").read()
    assert b"gfx950" in data


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU behaviour")
def test_fails_loudly_without_gpu():
    import ymerge
    with pytest.raises(ymerge.DeviceError):
        ymerge.Engine(0)
    with pytest.raises(ymerge.DeviceError):
        ymerge.merge_updates_v1([b"\x00\x00"])
