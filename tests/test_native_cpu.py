"""CPU-side checks of the C-ABI boundary: the library loads, exports every entry point declared in
include/automerge_amd.h, and refuses to run (no CPU fallback) when no GPU is visible."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "automerge_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(am_[a-z0-9_]+)\s*\(", src)))


def test_header_compiles_as_c():
    import subprocess
    subprocess.check_call(["gcc", "-fsyntax-only", "-std=c99", "-x", "c", os.path.join(ROOT, "include", "automerge_amd.h")])


def test_exports_match_header():
    from automerge_amd import _native as N
    names = declared_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(N.lib, n), n
    assert set(N.EXPORTS) <= set(names)


def test_struct_layouts():
    from automerge_amd import _native as N
    assert ctypes.sizeof(N.ChunkDesc) == 16
    assert ctypes.sizeof(N.DocDesc) == 32
    assert ctypes.sizeof(N.KnownHash) == 40
    assert ctypes.sizeof(N.DocResult) == 96


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    from automerge_amd import _native as N
    from automerge_amd import backend
    with pytest.raises(N.AutomergeError, match="no HIP device"):
        backend.init()
