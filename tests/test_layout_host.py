"""am_layout.h on the host: workspace regions and totals are 16-byte aligned (tests/host/layout_check.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_workspace_layout_aligned(tmp_path):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ missing")
    exe = str(tmp_path / "layout_check")
    subprocess.run([gxx, "-std=c++17", "-O1", "-I", os.path.join(ROOT, "automerge_amd", "csrc"), "-I",
                    os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "host", "layout_check.cpp"), "-o", exe],
                   check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
