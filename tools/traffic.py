#!/usr/bin/env python3
"""roofline.traffic from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/gpu_prof.sh.

  python tools/traffic.py gpurun_out/<tag> profiles/<name>.json

Per launch of the k_doc stage (k_doc_fast + the general lds/glb k_doc launches of the same step,
which bench.py times together): HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes). The 2x is the
gfx950 correction of MI355X_MICROARCH.md (HBM section: FETCH_SIZE counts half the bytes of 16-B/lane
streaming reads, which is how k_doc_fast stages each document's input span). The JSON records the
digest of the kernel sources it was measured on; bench.py reports it only while the digest matches.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STAGE = ("k_doc_fast", "lds_mode::k_doc", "glb_mode::k_doc")


def kernel_key(name):
    """'void k_doc_fast<true>(...)' -> 'k_doc_fast'; 'lds_mode::k_doc(...)' -> 'lds_mode::k_doc'."""
    name = name.split("(")[0]
    if name.startswith("void "):
        name = name[5:]
    return name.split("<")[0]


def per_launch(root, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[kernel_key(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    root, out = sys.argv[1], sys.argv[2]
    from bench import kernel_source_digest
    fetch = per_launch(root, "FETCH_SIZE")
    write = per_launch(root, "WRITE_SIZE")
    batch = None
    try:  # the bench line of the FETCH_SIZE pass names its batch size
        line = [x for x in open(os.path.join(root, "FETCH_SIZE.log")) if x.startswith("{")][-1]
        batch = json.loads(line).get("batch_docs")
    except (OSError, IndexError, ValueError):
        pass
    kf = sum(v for k, v in fetch.items() if k in STAGE)
    kw = sum(v for k, v in write.items() if k in STAGE)
    rec = {
        "kernel": "k_doc",
        "src_digest": kernel_source_digest(),
        "batch_docs": batch,
        "fetch_size_kib": kf, "write_size_kib": kw,
        "traffic_bytes": int(2 * kf * 1024 + kw * 1024),
        "correction": "2 x FETCH_SIZE (gfx950, 16 B/lane streaming reads) + WRITE_SIZE",
        "per_kernel_fetch_kib": fetch, "per_kernel_write_kib": write,
        "source": root,
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: rec[k] for k in ("kernel", "traffic_bytes", "fetch_size_kib", "write_size_kib")}))


if __name__ == "__main__":
    main()
