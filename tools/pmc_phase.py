"""One staged C4 batch (with the applyChanges patch) run once: the command the per-phase PMC
passes of tools/pmc_phase.sh profile."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import workload  # noqa: E402
from automerge_amd.batch import WANT_DIFF, Batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
arena, chunks, docs, ops = workload.c4(0, n)
docs["flags"] |= WANT_DIFF
b = Batch(device=0)
b.stage(arena, chunks, docs)
b.run()
b.sync()
print("fast docs", int(b.fast_flags().sum()), "of", n)
