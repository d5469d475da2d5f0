"""Dumps the engine generator's text histories (am_workload_text) and runs
make_text.js (the reference backend under Node, this container only) to write tests/golden/text.json.
Usage: python tests/golden/gen/make_text.py"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", "..", ".."))
sys.path.insert(0, ROOT)
from automerge_amd import workload as W  # noqa: E402

CASES = [  # name, first doc, docs, changes after change 0, ops per change, cross_every
    ("c3s", 0, 3, 40, 100, 10),
    ("c3m", 7, 1, 200, 100, 10),
    ("c1", 0, 1, 100, 100, 0),
    ("c1_op1", 3, 1, 2000, 1, 0),
    ("mixed", 11, 4, 30, 7, 3),
    ("c3full", 0, 2, 1000, 100, 10),  # configs[2] document size: 100,001 ops
]


def main():
    payload = []
    for name, first, n, nch, per, cross in CASES:
        arena, chunks, docs, _ = W.text(first, n, nch, per, cross)
        payload.append({"name": name, "first": first, "n": n, "nchanges": nch, "per_change": per, "cross_every": cross,
                        "docs": [[c.hex() for c in W.doc_chunks(arena, chunks, docs, i)[1]] for i in range(n)]})
    tmp = "/tmp/text_in.json"
    json.dump(payload, open(tmp, "w"))
    env = dict(os.environ, NODE_PATH=os.path.join(HERE, "node_modules"))
    subprocess.check_call(["node", os.path.join(HERE, "make_text.js"), tmp, os.path.join(HERE, "..", "text.json")],
                          env=env)


if __name__ == "__main__":
    main()
