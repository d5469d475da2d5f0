"""DPP / permlane wave primitives (automerge_amd/csrc/am_wave.h) on the device against numpy.

Every k_doc_fast scan, sort and neighbour compare goes through these; a wrong DPP control word
shows up here as a wrong lane rather than as a mismatched document."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def run(vals):
    from automerge_amd import _native
    f = _native.lib.amx_wave_selftest
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_int
    vin = np.ascontiguousarray(vals, dtype=np.uint64)
    out = np.zeros((16, 64), dtype=np.uint64)
    assert f(vin.ctypes.data, out.ctypes.data) == 0
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_wave_primitives(seed):
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 2**63, size=64, dtype=np.uint64)
    if seed == 1:
        v = rng.integers(0, 8, size=64, dtype=np.uint64)  # many ties
    if seed == 2:
        v[::3] = np.uint64(2**64 - 1)  # padding keys
    out = run(v)
    v32 = (v & np.uint64(0xffffffff)).astype(np.uint32)
    inc = np.cumsum(v32.astype(np.uint64)) & np.uint64(0xffffffff)
    assert (out[0] == inc).all()
    assert (out[1] == (inc - v32.astype(np.uint64)) & np.uint64(0xffffffff)).all()
    assert (out[2] == inc[-1]).all()
    s32 = v32.view(np.int32).astype(np.int64)
    assert (out[3].view(np.int64) == np.maximum.accumulate(s32)).all()
    assert (out[4].view(np.int64) == v.view(np.int64).max()).all()
    lanes = np.arange(64)
    for row, j in zip(range(5, 11), [1, 2, 4, 8, 16, 32]):
        assert (out[row] == v[lanes ^ j]).all(), j
    assert (out[11] == np.sort(v)).all()
    assert out[12][0] == 7 and (out[12][1:] == v[:-1]).all()
    assert out[13][63] == 9 and (out[13][:-1] == v[1:]).all()
    assert (out[14] == v[37]).all()
    assert (out[15] == inc[-1]).all()
