"""Replay of the backend-boundary logs recorded from the reference's own test files
(tests/golden/backend_log_*.json, tests/golden/gen/make_backend_log.js) against the Python host
(automerge_amd.backend). Each entry is one call of a backend/index.js export with its arguments and
the reference's result or error; handles are matched by identity as the reference returned them."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = ["sync", "sync_random", "objmeta", "backend", "test", "text", "table", "errors"]
# Scenarios where this engine knowingly differs from the reference, with the reason. Each must still
# fail loudly with an "automerge_amd: unsupported" error (never a silently different result).
KNOWN_DIVERGENT = set()  # none: the last one (a null action) is restated since round 4
PURE = {"encodeSyncMessage", "decodeSyncMessage", "encodeSyncState", "decodeSyncState", "initSyncState"}
UNDEF = object()


def load(name):
    with open(os.path.join(GOLDEN, "backend_log_%s.json" % name)) as f:
        return json.load(f)


def _special(r):
    return isinstance(r, dict) and len(r) == 1 and next(iter(r)) in ("__bytes", "__f64", "__undef", "__view", "$h")


def decode(r, handles):
    if isinstance(r, list):
        return [decode(v, handles) for v in r]
    if isinstance(r, dict):
        if _special(r):
            k, v = next(iter(r.items()))
            if k == "$h":
                return handles[v]
            if k in ("__bytes", "__view"):
                return bytes.fromhex(v)
            if k == "__undef":
                return UNDEF
            return -0.0 if v == "-0" else float(v)
        return {k: decode(v, handles) for k, v in r.items()}
    return r


def canon(x):
    if x is UNDEF:
        return {"__undef": 1}
    if isinstance(x, bool) or x is None or isinstance(x, str):
        return x
    if isinstance(x, float):
        if x != x or x in (float("inf"), float("-inf")):
            return {"__f64": "NaN" if x != x else ("Infinity" if x > 0 else "-Infinity")}
        if x == 0 and str(x).startswith("-"):
            return {"__f64": "-0"}
        return int(x) if x.is_integer() and abs(x) < 2 ** 63 else x
    if isinstance(x, int):
        return x
    if isinstance(x, (bytes, bytearray, memoryview)):
        return {"__bytes": bytes(x).hex()}
    if isinstance(x, (list, tuple)):
        return [canon(v) for v in x]
    if isinstance(x, dict):
        return {k: canon(x[k]) for k in sorted(x)}
    if _is_handle(x):
        return {"$h": "?"}  # a backend state (only in mismatch reports)
    raise TypeError("cannot canonicalize %r" % (x,))


def _is_handle(x):
    return hasattr(x, "state") and hasattr(x, "heads") and hasattr(x, "frozen")


def match(rec, x, handles):
    if _special(rec) and "$h" in rec:
        if not _is_handle(x):
            return False
        if rec["$h"] in handles:
            return handles[rec["$h"]] is x
        handles[rec["$h"]] = x
        return True
    if isinstance(rec, list):
        return isinstance(x, (list, tuple)) and len(x) == len(rec) and all(match(a, b, handles) for a, b in zip(rec, x))
    if isinstance(rec, dict) and not _special(rec):
        return isinstance(x, dict) and sorted(rec) == sorted(x) and all(match(rec[k], x[k], handles) for k in rec)
    if rec == {"__undef": 1} and x is None:
        return True
    return json.dumps(canon(x), sort_keys=True) == json.dumps(rec, sort_keys=True)


def _err_name(e):
    from automerge_amd import _native as N
    if isinstance(e, N.AutomergeError):
        return e.kind
    if isinstance(e, TypeError):
        return "TypeError"
    return "Error"


def _args(fn, args):
    # JS `undefined` arguments are absent in Python (defaults apply)
    while args and args[-1] is UNDEF:
        args = args[:-1]
    return args


def replay(B, files=FILES, only=None, stop_at=40):
    """Replays the logs through backend module B; returns (calls, scenarios, bad)."""
    bad, calls, scen = [], 0, 0
    for f in files:
        for sc in load(f)["scenarios"]:
            handles = {}
            if only is not None and not any(e["fn"] in only for e in sc["log"]):
                continue
            scen += 1
            if (f, sc["name"]) in KNOWN_DIVERGENT:
                bad.extend(_divergent(B, f, sc, handles))
                continue
            for i, e in enumerate(sc["log"]):
                if only is not None and e["fn"] not in only:
                    continue
                calls += 1
                try:
                    res, err = getattr(B, e["fn"])(*_args(e["fn"], decode(e["args"], handles))), None
                except Exception as x:  # noqa: BLE001 -- the error is the result being compared
                    res, err = None, {"name": _err_name(x), "message": str(x)}
                if "error" in e:
                    if err is None or err["message"] != e["error"]["message"] or err["name"] != e["error"]["name"]:
                        bad.append((f, sc["name"], i, e["fn"], e["error"], err))
                    continue
                if err is not None:
                    bad.append((f, sc["name"], i, e["fn"], "unexpected", err))
                    break
                if not match(e["result"], res, handles):
                    bad.append((f, sc["name"], i, e["fn"], json.dumps(e["result"])[:400], json.dumps(canon(res))[:400]))
                    break
                if len(bad) >= stop_at:
                    return calls, scen, bad
    return calls, scen, bad


def _divergent(B, f, sc, handles):
    """A known divergence: the first call that differs from the reference must raise the engine's
    "unsupported" error; returns [] when it does."""
    for i, e in enumerate(sc["log"]):
        try:
            res = getattr(B, e["fn"])(*_args(e["fn"], decode(e["args"], handles)))
            if "result" in e:
                match(e["result"], res, handles)  # registers the handles the call returned
        except Exception as x:  # noqa: BLE001
            if str(x).startswith("automerge_amd: unsupported"):
                return []
            return [(f, sc["name"], i, e["fn"], "known divergence raised", str(x))]
    return [(f, sc["name"], -1, "", "known divergence did not raise", "")]


# the batched surface: fn -> (batch function of backend module B, how it takes the args columns)
BATCHED = {
    "applyChanges": "applyChangesBatch", "loadChanges": "loadChangesBatch", "load": "loadBatch",
    "save": "saveBatch", "getPatch": "getPatchBatch", "generateSyncMessage": "generateSyncMessages",
    "receiveSyncMessage": "receiveSyncMessages",
}


def replay_lockstep(B, files=FILES, stop_at=40):
    """The logs replayed in lockstep: call k of every scenario of every file at once, the calls of
    one function in one batched call (BATCHED), the rest one by one. A scenario's calls stay in
    order, so each sees the same handles and states as in replay(); results are compared the same
    way. Returns (calls, batched calls, bad)."""
    scens = [(f, sc) for f in files for sc in load(f)["scenarios"] if (f, sc["name"]) not in KNOWN_DIVERGENT]
    handles = [{} for _ in scens]
    live = [True] * len(scens)
    bad, calls, batched = [], 0, 0
    k = 0
    while any(live):
        groups = {}
        for j, (f, sc) in enumerate(scens):
            if not live[j]:
                continue
            if k >= len(sc["log"]):
                live[j] = False
                continue
            e = sc["log"][k]
            args = _args(e["fn"], decode(e["args"], handles[j]))
            key = e["fn"] if (e["fn"] in BATCHED and len(args) == (1 if e["fn"] in ("save", "getPatch", "load") else
                                                                    3 if e["fn"] == "receiveSyncMessage" else 2)) else None
            groups.setdefault(key, []).append((j, e, args))
        results = {}
        for key, items in groups.items():
            if key is None:
                for j, e, args in items:
                    try:
                        results[j] = (getattr(B, e["fn"])(*args), None)
                    except Exception as x:  # noqa: BLE001 -- the error is the result being compared
                        results[j] = (None, x)
                continue
            cols = list(zip(*[args for _, _, args in items]))
            out = getattr(B, BATCHED[key])(*[list(c) for c in cols])
            batched += len(items)
            for (j, e, _), r in zip(items, out):
                results[j] = (None, r) if isinstance(r, Exception) else (r, None)
        for key, items in groups.items():
            for j, e, _ in items:
                f, sc = scens[j]
                calls += 1
                res, x = results[j]
                err = None if x is None else {"name": _err_name(x), "message": str(x)}
                if "error" in e:
                    if err is None or err["message"] != e["error"]["message"] or err["name"] != e["error"]["name"]:
                        bad.append((f, sc["name"], k, e["fn"], e["error"], err))
                    continue
                if err is not None:
                    bad.append((f, sc["name"], k, e["fn"], "unexpected", err))
                    live[j] = False
                    continue
                if not match(e["result"], res, handles[j]):
                    bad.append((f, sc["name"], k, e["fn"], json.dumps(e["result"])[:400], json.dumps(canon(res))[:400]))
                    live[j] = False
        if len(bad) >= stop_at:
            break
        k += 1
    return calls, batched, bad
