"""Timing of each host/GPU step of the c3full parity case (tests/test_gpu_text.py)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from automerge_amd import patch as P  # noqa: E402
import workload as W  # noqa: E402
from automerge_amd.batch import WANT_DIFF, WANT_PATCH, Batch, pack  # noqa: E402

T0 = time.time()


def say(msg):
    print("%7.2f s  %s" % (time.time() - T0, msg), flush=True)


arena, chunks, docs, _ = W.text(0, 2, 1000, 100, 10)
chg = [W.doc_chunks(arena, chunks, docs, i)[1] for i in range(2)]
say("generated")
packed = pack([(None, c) for c in chg], flags=WANT_PATCH)
say("packed")
for flags in (0, WANT_PATCH, WANT_DIFF):
    b = Batch()
    b.stage(*pack([(None, c) for c in chg], flags=flags))
    say("staged flags %d" % flags)
    b.run()
    b.sync()
    say("ran; stages %s" % b.stage_times())
    r = b.results()
    s = b.doc_save(0)
    say("doc_save %d bytes" % len(s))
    if flags:
        blob = b.doc_patch(0)
        say("patch log %d bytes" % len(blob))
        heads = b.doc_heads(0, int(r[0]["nheads"]))
        p = P.materialize(blob, heads, 0, int(r[0]["max_op"]))
        say("materialized")

# split: base = first half, then load(base) + rest
half = len(chg[0]) // 2
b = Batch()
b.stage(*pack([(None, c[:half]) for c in chg]))
b.run()
b.sync()
bases = [b.doc_save(i) for i in range(2)]
say("bases %s" % [len(x) for x in bases])
for flags in (0, WANT_PATCH, WANT_DIFF):
    b = Batch()
    b.stage(*pack([(base, c[half:]) for base, c in zip(bases, chg)], flags=flags))
    say("split staged flags %d" % flags)
    b.run()
    b.sync()
    say("split ran; stages %s" % b.stage_times())
