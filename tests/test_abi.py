"""CPU checks of the C ABI: the library loads, exports every symbol include/irc.h
declares, and the ctypes table binds each of them (no compute without a GPU)."""
import ctypes
import os
import re

from conftest import PKG, ROOT

from irc_amd import _lib


def _declared():
    txt = open(os.path.join(ROOT, "include", "irc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(irc_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 5
    for n in names:
        assert hasattr(lib, n), f"{n} declared in irc.h but not exported"


def test_binding_table_matches_header():
    assert set(_declared()) == set(_lib.SIGNATURES), "irc_amd/_lib.py SIGNATURES out of sync"


def test_host_side_validation_without_gpu():
    lib = _lib.load()
    assert lib.irc_abi_version() == 1
    # bad D is rejected on the host before any launch
    rc = lib.irc_scan_topk(None, None, 4, 10, 100, 5, 0, None, 0, None, None, None)
    assert rc == 1001
    assert b"unsupported D" in lib.irc_last_error()
    ws = lib.irc_scan_topk_workspace(256, 100000, 768, 100)
    assert ws >= 256 * 100000 * 8 // 4  # survivors region sized for the worst case


def test_product_path_refuses_cpu_tensors():
    import pytest
    import torch

    from irc_amd import retrieval

    with pytest.raises(RuntimeError, match="no CPU fallback"):
        retrieval.scan_topk(torch.zeros(2, 128), torch.zeros(4, 128), 2)
