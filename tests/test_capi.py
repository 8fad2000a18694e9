"""CPU tests: the C-ABI library builds for gfx950, loads without a GPU, and exports every entry point
include/irx.h declares with the ctypes signatures `_lib.py` binds (no compute calls here)."""
import ctypes as C
import re
from pathlib import Path

import pytest

from image_restoration_and_enhancement_amd import _lib as L
from image_restoration_and_enhancement_amd import build as B

HEADER = Path(__file__).resolve().parents[1] / "include" / "irx.h"


def declared():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    return sorted(set(re.findall(r"\b(irx_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    path = B.build()
    return C.CDLL(str(path))


def test_header_declares_entry_points():
    names = declared()
    assert len(names) > 30
    for must in ("irx_unet_forward", "irx_vae_encode", "irx_vae_decode", "irx_clip_encode", "irx_sched_step",
                 "irx_model_bind", "irx_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_bindings_cover_header():
    assert sorted(L.EXPORTED) == declared()


def test_load_binds_signatures_and_version(lib):
    h = L.load()
    assert L.call("irx_version") > 0
    assert h is L.load()      # loaded once


def test_error_path_without_gpu(lib):
    """A compute call without a usable device must return a status and set irx_last_error, not crash."""
    h = L.load()
    rc = h.irx_set_option(b"no_such_option", 1)
    assert rc != 0
    assert b"option" in h.irx_last_error()


def test_missing_library_raises(tmp_path):
    with pytest.raises(L.IrxError):
        L.load(tmp_path / "libirx_missing.so", force=True)


def test_rccl_entry_points_without_gpu(lib):
    """The RCCL boundary resolves librccl lazily (dlopen) and reports errors through the status path."""
    h = L.load()
    assert L.call("irx_rccl_available") in (0, 1)
    assert h.irx_weights_bcast(None, None, 0, None) != 0
    assert b"null model" in h.irx_last_error()
    assert h.irx_rccl_broadcast(None, None, 16, 0, None) != 0
