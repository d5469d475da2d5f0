"""Host-only parity of the drop-in boundary (no GPU): encodeChange (am_encode_change) and the sync
codecs (am_sync_encode_message, am_sync_decode_messages, am_sync_encode_state,
am_sync_decode_state) against the calls recorded from the reference's own test files
(tests/golden/backend_log_*.json), through the Python host and through the Node host."""
import json
import os
import shutil
import subprocess
import zlib

import pytest

import backend_log as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
node = shutil.which("node")


def _change_deps(b):
    o, ln, sh = 9, 0, 0
    while True:
        x = b[o]
        o += 1
        ln |= (x & 0x7F) << sh
        sh += 7
        if not x & 0x80:
            break
    body = b[o:o + ln]
    if b[8] == 2:
        body = zlib.decompress(body, -15)
    n, o, sh = 0, 0, 0
    while True:
        x = body[o]
        o += 1
        n |= (x & 0x7F) << sh
        sh += 7
        if not x & 0x80:
            break
    return [body[o + 32 * i:o + 32 * i + 32].hex() for i in range(n)]


def test_encode_change_matches_every_recorded_local_change():
    """Every binary change the reference's applyLocalChange produced in its test files is
    reproduced byte for byte by encodeChange from the recorded request (columnar.js:710-739)."""
    from automerge_amd import backend as B
    n = 0
    for f in L.FILES:
        for sc in L.load(f)["scenarios"]:
            for e in sc["log"]:
                if e["fn"] != "applyLocalChange" or "result" not in e:
                    continue
                want = L.decode(e["result"][2], {})
                req = L.decode(e["args"][1], {})
                req["deps"] = _change_deps(want)
                assert B.encodeChange(req) == want, (f, sc["name"])
                n += 1
    assert n > 600


def test_encode_change_errors():
    """encodeChange raises the reference's error class and message (columnar.js, encoding.js)."""
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    actor = "aa" * 16
    base = {"actor": actor, "seq": 1, "startOp": 1, "time": 0, "deps": [], "ops": []}

    def err(change):
        with pytest.raises(N.AutomergeError) as ei:
            B.encodeChange(change)
        return ei.value.kind, str(ei.value)

    op = {"action": "set", "obj": "_root", "key": "x", "value": 1, "pred": []}
    assert err(dict(base, deps="x")) == ("TypeError", "deps is not an array")
    assert err(dict(base, deps=["zz"])) == ("RangeError", "value is not hexadecimal")
    assert err(dict(base, actor="xyz")) == ("RangeError", "value is not hexadecimal")
    assert err(dict(base, seq=1.5)) == ("RangeError", "value is not an integer")
    assert err(dict(base, seq=-1)) == ("RangeError", "number out of range")
    assert err(dict(base, message=5)) == ("TypeError", "value is not a string")
    assert err(dict(base, ops=[dict(op, obj="nope")])) == ("RangeError", "Not a valid opId: nope")
    assert err(dict(base, ops=[dict(op, obj="0@" + actor)]))[1].startswith("Unexpected objectId reference: ")
    assert err(dict(base, ops=[dict(op, action="frob")])) == ("RangeError", "Unexpected operation action: frob")
    assert err(dict(base, ops=[dict(op, value={"a": 1})])) == ("RangeError", "Unsupported value in operation: [object Object]")
    assert err(dict(base, ops=[dict(op, value=[1], datatype="x")])) == ("RangeError", "Unknown datatype x for value 1")
    assert err(dict(base, ops=[dict(op, value=1.5, datatype="counter")])) == ("RangeError", "value is not an integer")
    assert err(dict(base, ops=[dict(op, value=-1, datatype="uint")])) == ("RangeError", "number out of range")
    assert err(dict(base, ops=[{"action": "set", "obj": "_root", "elemId": "_head", "insert": True, "values": [1, "a"],
                                "pred": []}])) == ("RangeError", "Decode failed: bad value/datatype association (1,undefined)")
    assert err(dict(base, ops=[{"action": "set", "obj": "_root", "elemId": "_head", "insert": True, "values": ["a"],
                                "pred": ["1@" + actor]}])) == ("RangeError", "multi-insert pred must be empty")
    assert err(dict(base, ops=[{"action": "del", "obj": "_root", "elemId": "1@" + actor, "multiOp": 2, "pred": []}])) == \
        ("RangeError", "multiOp deletion must have exactly one pred")
    assert err(dict(base, hash="00" * 32))[1].startswith("Change hash does not match encoding: " + "00" * 32 + " != ")
    k, m = err(dict(base, ops=[{"action": "set", "obj": "_root", "value": 1, "pred": []}]))
    assert (k, m) == ("RangeError", 'Unexpected operation key: {"action":"set","obj":"_root","value":1,"pred":[],'
                                    '"id":{"counter":1,"actorNum":0,"actorId":"%s"}}' % actor)


def test_sync_codecs_replay_recorded_calls():
    """encode/decodeSyncMessage, encode/decodeSyncState and initSyncState: every recorded call
    (sync_test.js and the others) gives the reference's result or error."""
    from automerge_amd import backend as B
    calls, _, bad = L.replay(B, only=L.PURE)
    assert calls > 150
    assert bad == []


def test_sync_decode_errors():
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    cases = [(b"", "Unexpected message type: undefined"), (b"\x41", "Unexpected message type: 65"),
             (b"\x42", "buffer ended with incomplete number"), (b"\x42\x01", "subarray exceeds buffer size"),
             (b"\x42\xff\xff\xff\xff\x7f", "number out of range"), (b"\x42\x00\x00\x01\x00\x05ab", "subarray exceeds buffer size")]
    for data, msg in cases:
        with pytest.raises(N.AutomergeError, match=msg):
            B.decodeSyncMessage(data)
    with pytest.raises(N.AutomergeError, match="Unexpected record type: 66"):
        B.decodeSyncState(b"\x42\x00")
    with pytest.raises(N.AutomergeError, match="hashes must be sorted"):
        B.encodeSyncState({"sharedHeads": ["11" * 32, "00" * 32]})
    with pytest.raises(N.AutomergeError, match="heads hashes must be 256 bits"):
        B.encodeSyncMessage({"heads": ["00"], "need": [], "have": [], "changes": []})
    # a batch decodes every message and reports the malformed ones in place
    good = B.encodeSyncMessage({"heads": ["00" * 32], "need": [], "have": [{"lastSync": [], "bloom": b"\x01\x0a\x07\x00\x00"}],
                                "changes": [b"abc"]})
    r = B.decodeSyncMessages([good, b"\x41", good])
    assert r[0] == r[2] == {"heads": ["00" * 32], "need": [], "have": [{"lastSync": [], "bloom": b"\x01\x0a\x07\x00\x00"}],
                            "changes": [b"abc"]}
    assert isinstance(r[1], N.AutomergeError)


@pytest.mark.skipif(node is None or not os.path.exists(os.path.join(ROOT, "automerge_amd", "js", "am_napi.node")),
                    reason="node or am_napi.node missing")
def test_node_host_codecs():
    out = subprocess.run([node, os.path.join(ROOT, "tests", "js", "host_codec_check.js")], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["encoded"] > 600 and res["pure"] > 150
    assert res["nbad"] == 0, res["bad"]
