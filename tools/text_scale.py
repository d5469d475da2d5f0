"""Scaling probe for long text histories on the GPU: one batched launch per (size, flags), stage
times per kernel. Usage: python tools/text_scale.py [ndocs] [nchanges ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workload as W  # noqa: E402
from automerge_amd.batch import WANT_DIFF, WANT_PATCH, Batch, pack  # noqa: E402


def main():
    ndocs = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    sizes = [int(x) for x in sys.argv[2:]] or [100, 200, 400]
    flags_list = [int(x) for x in os.environ.get("FLAGS", "0,2,4").split(",")]
    for nch in sizes:
        arena, chunks, docs, ops = W.text(0, ndocs, nch, 100, 10)
        chg = [W.doc_chunks(arena, chunks, docs, i)[1] for i in range(ndocs)]
        packed = {}
        for flags in flags_list:
            if flags not in packed:
                packed[flags] = pack([(None, c) for c in chg], flags=flags)
            b = Batch()
            b.stage(*packed[flags])
            t = time.time()
            b.run()
            b.sync()
            dt = time.time() - t
            r = b.results()
            print("nchanges %d ops/doc %d docs %d flags %d: %.1f ms wall, stages %s, status %s, ws %.1f MB" % (
                nch, ops // ndocs, ndocs, flags, dt * 1e3, ["%.2f" % x for x in (b.stage_times() or [])],
                sorted(set(int(x) for x in r["status"])), b.workspace_bytes() / 1e6), flush=True)


if __name__ == "__main__":
    main()
