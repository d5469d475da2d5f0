"""Replay of tests/golden/newbackend_log.json (the reference's test/new_backend_test.js, recorded by
tests/golden/gen/make_newbackend_log.js) through a backend module with the backend/index.js surface
(automerge_amd.backend). Each recorded BackendDoc becomes a backend handle: `new` -> init()/load(),
`applyChanges` -> applyChanges() (patch compared, then save() bytes and getHeads() compared with the
reference's document after that call), `getPatch` -> getPatch(); thrown errors compare class and
message. Returns the mismatches."""
import json
import os

from backend_log import _err_name, canon

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    with open(os.path.join(GOLDEN, "newbackend_log.json")) as f:
        return json.load(f)


def _b(x):
    return bytes.fromhex(x["__bytes"])


def _same(rec, got):
    return json.dumps(rec, sort_keys=True) == json.dumps(canon(got), sort_keys=True)


def replay(B, only=None):
    data = load()
    calls, bad = 0, []
    for sc in data["scenarios"]:
        if only is not None and sc["name"] not in only:
            continue
        docs = {}
        for i, e in enumerate(sc["log"]):
            calls += 1
            where = (sc["name"], i, e["fn"])
            if e["fn"] == "new":
                docs[e["doc"]] = B.load(_b(e["args"][0])) if e["args"] else B.init()
                continue
            h = docs.get(e["doc"])
            if h is None:
                continue  # an earlier error ended this document's log
            try:
                if e["fn"] == "applyChanges":
                    h2, res = B.applyChanges(h, [_b(c) for c in e["args"][0]])
                else:
                    h2, res = h, B.getPatch(h)
                err = None
            except Exception as x:  # noqa: BLE001 -- the error is the result being compared
                h2, res, err = None, None, {"name": _err_name(x), "message": str(x)}
            if "error" in e:
                if err != e["error"]:
                    bad.append(where + (e["error"], err))
                docs[e["doc"]] = None
                continue
            if err is not None:
                bad.append(where + ("unexpected", err))
                docs[e["doc"]] = None
                continue
            if not _same(e["result"], res):
                bad.append(where + (json.dumps(e["result"])[:300], json.dumps(canon(res))[:300]))
                docs[e["doc"]] = None
                continue
            docs[e["doc"]] = h2
            if "save" in e:
                if B.save(h2).hex() != e["save"]:
                    bad.append(where + ("save", e["save"][:200], B.save(h2).hex()[:200]))
                    docs[e["doc"]] = None
                elif list(B.getHeads(h2)) != e["heads"]:
                    bad.append(where + ("heads", e["heads"], list(B.getHeads(h2))))
    return calls, bad
