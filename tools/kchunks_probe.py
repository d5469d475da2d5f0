"""k_chunks time on the C3 inputs split by kind: the 501k inflated changes alone, and the 1000
50k-op base documents alone (Batch.stage_times()[0], HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import workload as W
    from automerge_amd.batch import Batch, pack
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    arena, chunks, docs, _ = W.text(0, n, 1000, 100, 10)
    hist = [W.doc_chunks(arena, chunks, docs, i)[1] for i in range(n)]
    half = 501
    prep = Batch()
    prep.stage(*pack([(None, h[:half]) for h in hist]))
    prep.run(); prep.sync()
    bases = [prep.doc_save(i) for i in range(n)]
    del prep
    for name, items in (("changes only", [(None, h[half:]) for h in hist]), ("bases only", [(b, []) for b in bases])):
        b = Batch()
        b.stage(*pack(items))
        b.run(); b.sync()
        ms = []
        for _ in range(3):
            b.run(); b.sync()
            ms.append(b.stage_times()[0])
        print(name, "k_chunks ms", [round(x, 2) for x in ms], flush=True)
        del b


if __name__ == "__main__":
    main()
