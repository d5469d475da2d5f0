"""Dumps the engine generator's mid-size documents (workload.mid, am_workload.cpp gen_mid) and runs
make_mid.js (the reference backend under Node, this container only) to write tests/golden/mid.json.
Usage: python tests/golden/gen/make_mid.py"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", "..", ".."))
sys.path.insert(0, ROOT)
import workload as W  # noqa: E402

CASES = [  # name, first doc, docs, actors, rounds, min ops, max ops per change
    ("mid", 0, 24, 4, 12, 8, 40),
    ("mid_small", 100, 16, 4, 4, 2, 12),   # 50-200 ops: around the small-document kernel's envelope
    ("mid_wide", 200, 6, 8, 10, 8, 40),
]


def main():
    payload = []
    for name, first, n, na, rounds, lo, hi in CASES:
        arena, chunks, docs, _ = W.mid(first, n, na, rounds, lo, hi)
        payload.append({"name": name, "first": first, "n": n, "nactors": na, "rounds": rounds, "min_ops": lo, "max_ops": hi,
                        "docs": [[c.hex() for c in W.doc_chunks(arena, chunks, docs, i)[1]] for i in range(n)]})
    tmp = "/tmp/mid_in.json"
    json.dump(payload, open(tmp, "w"))
    env = dict(os.environ, NODE_PATH=os.path.join(HERE, "node_modules"))
    subprocess.check_call(["node", os.path.join(HERE, "make_mid.js"), tmp, os.path.join(HERE, "..", "mid.json")], env=env)


if __name__ == "__main__":
    main()
