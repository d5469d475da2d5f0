"""Pins the CPU oracle (oracle/am_oracle.c) against golden vectors produced by the reference
(tests/golden/gen/make_fixtures.js). CPU-only."""
import pytest

import oracle_ffi as O
from conftest import golden

LEB_ENC = {"appendUint32": 0, "appendInt32": 1, "appendUint53": 2, "appendInt53": 3, "appendUint64": 4, "appendInt64": 5}
LEB_DEC = {"readUint32": 0, "readInt32": 1, "readUint53": 2, "readInt53": 3, "readUint64": 4, "readInt64": 5}


def test_leb_encode(codecs):
    for v in codecs["leb"]:
        fn = LEB_ENC[v["fn"]]
        if fn >= 4:
            got = O.leb_encode(fn, hi=v["high32"], lo=v["low32"])
        else:
            got = O.leb_encode(fn, value=int(v["value"]))
        assert got.hex() == v["bytes"], v


def test_leb_decode(codecs):
    for v in codecs["leb_decode"]:
        val, err, off = O.leb_decode(LEB_DEC[v["fn"]], bytes.fromhex(v["bytes"]))
        if v["error"]:
            assert err == v["error"], v
        else:
            assert err is None, (v, err)
            if isinstance(v["value"], list):
                assert list(val) == v["value"], v
            else:
                assert val == v["value"], v
            assert off == v["offset"], v


@pytest.mark.parametrize("kind", ["rle", "delta", "bool"])
def test_column_codecs(codecs, kind):
    for v in codecs[kind]:
        t = v.get("type", kind)
        assert O.col_encode(t, v["values"]).hex() == v["bytes"], v
        vals, err = O.col_decode(t, bytes.fromhex(v["bytes"]))
        assert err is None
        exp = v["values"]
        if t in ("uint", "int", "utf8", "delta") and all(x is None for x in exp):
            exp = []  # an all-null column encodes to nothing (encoding.js:780)
        assert vals == exp, v


def test_decode_errors(codecs):
    for v in codecs["decode_errors"]:
        vals, err = O.col_decode(v["type"], bytes.fromhex(v["bytes"]), maxn=64)
        assert err == v["error"], v
        assert vals == v["values"], v


def test_sha256():
    import hashlib
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 120, 1000):
        data = bytes(range(256)) * 4
        assert O.sha256(data[:n]) == hashlib.sha256(data[:n]).digest()


def test_change_meta():
    for v in golden("changes.json"):
        data = bytes.fromhex(v["bytes"])
        if v.get("error"):
            continue
        m = O.change_meta(data)
        assert m["hash"] == v["hash"]
        assert m["seq"] == v["decoded"]["seq"]
        assert m["startOp"] == v["decoded"]["startOp"]


def run_scenario(sc):
    """Replays a fixture scenario through the oracle; returns per-step results comparable to
    the reference's."""
    doc = None
    out = []
    for step in sc["steps"]:
        res = {}
        try:
            if step["op"] == "load":
                doc = O.Doc.load(bytes.fromhex(step["bytes"]))
            else:
                if doc is None:
                    doc = O.Doc.init()
                doc.apply([bytes.fromhex(c) for c in step["changes"]])
            res["save"] = doc.save().hex()
            res["heads"] = doc.heads()
            res["pending"] = doc.pending()
        except O.OracleError as e:
            res["error"] = str(e)
            res["code"] = e.code
            out.append(res)
            break
        out.append(res)
    return out


def test_doc_scenarios(docs):
    unsupported = []
    for sc in docs:
        got = run_scenario(sc)
        for exp, res in zip(sc["results"], got):
            if res.get("code") == 2:
                unsupported.append((sc["name"], res["error"]))
                break
            if "error" in exp:
                assert res.get("error") == exp["error"]["message"], (sc["name"], res, exp["error"])
                break
            assert "error" not in res, (sc["name"], res)
            assert res["heads"] == exp["heads"], sc["name"]
            assert res["pending"] == exp["pending"], sc["name"]
            assert res["save"] == exp["save"], sc["name"]
    # everything the fixtures exercise must be restated (no silent gaps)
    assert not unsupported, unsupported


def test_workload_vectors():
    w = golden("workload.json")
    for rec in w["c4"][:4]:
        doc = O.Doc.load(bytes.fromhex(rec["baseBytes"]))
        doc.apply([bytes.fromhex(c) for c in rec["changeBytes"]])
        assert doc.save().hex() == rec["mergedBytes"]
        assert doc.heads() == rec["heads"]


def test_mid_documents_oracle():
    """The oracle against the reference's digests of the mid-size workload (tests/golden/mid.json):
    save() bytes and heads of applyChanges(init(), all changes), for the first documents of each case."""
    import hashlib
    import json
    import os
    import workload as W
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "mid.json")))
    n = 0
    for cs in cases:
        k = min(cs["n"], 3)
        arena, chunks, docs, _ = W.mid(cs["first"], k, cs["nactors"], cs["rounds"], cs["min_ops"], cs["max_ops"], nthreads=2)
        for i in range(k):
            _, ch = W.doc_chunks(arena, chunks, docs, i)
            d = O.Doc.init()
            d.apply(ch)
            assert hashlib.sha256(d.save()).hexdigest() == cs["docs"][i]["full"]["save"], (cs["name"], i)
            n += 1
    assert n >= 9
