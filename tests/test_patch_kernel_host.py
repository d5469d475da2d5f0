"""getPatch scan of the engine (automerge_amd/csrc/am_patch.h -- the code k_doc's lane 0 runs in
phase P7) compiled for the host and fed documents decoded by the CPU oracle; its patch logs,
materialized by the product's host stage (automerge_amd/patch.py), must equal the reference's
getPatch output for every step of every golden scenario."""
import os
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "_build")


@pytest.fixture(scope="module")
def patch_host():
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("g++ not available")
    import oracle_ffi as O
    O.lib()  # builds oracle/liboracle.so if needed
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "patch_host")
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-Wall", os.path.join(ROOT, "tests", "native", "patch_host.cpp"),
                           "-o", exe, "-L" + os.path.join(ROOT, "oracle"), "-loracle",
                           "-Wl,-rpath," + os.path.join(ROOT, "oracle")])
    return exe


def run_logs(exe, docs, tmp):
    src, dst = os.path.join(tmp, "docs.bin"), os.path.join(tmp, "logs.bin")
    with open(src, "wb") as f:
        for d in docs:
            f.write(struct.pack("<I", len(d)) + d)
    subprocess.check_call([exe, src, dst])
    data = open(dst, "rb").read()
    logs, off = [], 0
    while off < len(data):
        (n,) = struct.unpack_from("<I", data, off)
        logs.append(data[off + 4:off + 4 + n])
        off += 4 + n
    return logs


def jsonable(x):
    if isinstance(x, (bytes, bytearray)):
        return {"__bytes": bytes(x).hex()}
    if isinstance(x, dict):
        return {k: jsonable(v) for k, v in x.items()}
    if isinstance(x, list):
        return [jsonable(v) for v in x]
    return x


def test_patch_scan_matches_reference_getpatch(patch_host, docs, tmp_path):
    from automerge_amd import patch as P
    cases = [(sc["name"], i, res) for sc in docs for i, res in enumerate(sc["results"])
             if "getPatch" in res and "save" in res]
    logs = run_logs(patch_host, [bytes.fromhex(res["save"]) for _, _, res in cases], str(tmp_path))
    assert len(logs) == len(cases) > 400
    bad = []
    for (name, i, res), log in zip(cases, logs):
        exp = res["getPatch"]
        got = jsonable(P.materialize(log, exp["deps"], exp["pendingChanges"]))
        if got != exp:
            bad.append((name, i))
    assert not bad, bad[:10]


def test_js_host_stage_materializes_same_logs(patch_host, docs, tmp_path):
    """The Node host stage (backend.js materializePatch) on the same engine logs."""
    import json
    node = shutil.which("node")
    if not node or not os.path.exists(os.path.join(ROOT, "automerge_amd", "js", "am_napi.node")):
        pytest.skip("node or am_napi.node missing")
    cases = [res for sc in docs for res in sc["results"] if "getPatch" in res and "save" in res]
    logs = run_logs(patch_host, [bytes.fromhex(res["save"]) for res in cases], str(tmp_path))
    payload = [{"log": log.hex(), "deps": res["getPatch"]["deps"], "pending": res["getPatch"]["pendingChanges"],
                "expect": res["getPatch"]} for res, log in zip(cases, logs)]
    f = os.path.join(str(tmp_path), "cases.json")
    with open(f, "w") as fh:
        json.dump(payload, fh)
    out = subprocess.run([node, os.path.join(ROOT, "tests", "js", "patch_materialize.js"), f], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["n"] > 400 and res["nbad"] == 0, res
