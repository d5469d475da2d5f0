"""N>1 path of bench.py on CPU: two ranks (gloo, 127.0.0.1) shard the C4 job with bench.py's own
partition (SHA-256 of the base document, first byte mod N: workload.c4_shard), merge their shard
(here with the CPU checker; on the GPU box with the engine) and exchange the per-rank digest with
one all-gather: documents, ops, errors, output bytes, the merged documents' digest and the
applyChanges patches' digest. The gathered totals must equal one process over all documents, and
the shards must be disjoint and cover the job."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOTAL_DOCS = 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _merge_shard(world, rank):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    from automerge_amd import shard
    import workload
    ids = workload.c4_shard(0, TOTAL_DOCS, world, rank)
    arena, chunks, docs, ops = workload.c4_list(ids)
    lens, terms, pterms = [], [], []
    for i, gi in enumerate(ids):
        base, changes = workload.doc_chunks(arena, chunks, docs, i)
        assert shard.shard_of(base, world) == rank
        d = O.Doc.load(base)
        pterms.append(shard.patch_term(int(gi), d.apply_patch(changes)))
        out = d.save()
        lens.append(len(out))
        terms.append(shard.doc_digest(int(gi), 0, out))
    return [len(ids), ops, 0, sum(lens), shard.combine(terms), shard.combine(pterms)], [int(x) for x in ids]


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from automerge_amd import shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    digest, ids = _merge_shard(world, rank)
    tot, rows = shard.exchange(dist, digest, "cpu")
    np.save(os.path.join(outdir, "rank%d.npy" % rank), np.array(tot + ids, dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range():
    from automerge_amd import shard
    spans = [shard.shard_range(r, 4, 7) for r in range(4)]
    assert spans == [(0, 7), (7, 7), (14, 7), (21, 7)]
    with pytest.raises(ValueError):
        shard.shard_range(4, 4, 7)


def test_two_rank_gloo_digest_matches_single_process(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = [np.load(os.path.join(tmp_path, "rank%d.npy" % r)).tolist() for r in range(world)]
    nf = 6
    assert got[0][:nf] == got[1][:nf]  # every rank sees the same gathered totals
    ids = sorted(got[0][nf:] + got[1][nf:])
    assert ids == list(range(TOTAL_DOCS))  # disjoint, covering
    assert got[0][nf:] and got[1][nf:]
    single, _ = _merge_shard(1, 0)
    assert got[0][:nf] == single[:nf]


def test_digest_detects_one_wrong_byte_and_equal_lengths():
    """Documents of equal length do not cancel, and one changed output byte changes the digest."""
    from automerge_amd import shard
    outs = [bytes([0x85, 0x6F, 0x4A, 0x83, i, 7, 7, 7]) + bytes(20) for i in range(6)]
    base = shard.combine(shard.doc_digest(i, 0, o) for i, o in enumerate(outs))
    assert base != 0
    bad = list(outs)
    bad[3] = outs[3][:5] + b"\x08" + outs[3][6:]
    assert shard.combine(shard.doc_digest(i, 0, o) for i, o in enumerate(bad)) != base
    swapped = [outs[1], outs[0]] + outs[2:]  # same multiset, wrong owners
    assert shard.combine(shard.doc_digest(i, 0, o) for i, o in enumerate(swapped)) != base


def test_patch_term_covers_clock_and_diffs():
    from automerge_amd import shard
    p = {"maxOp": 3, "deps": [], "pendingChanges": 0, "clock": {"aa": 1},
         "diffs": {"objectId": "_root", "type": "map", "props": {"k": {"1@aa": {"type": "value", "value": 1}}}}}
    t = shard.patch_term(5, p)
    assert t == shard.patch_term(5, dict(p, maxOp=9, deps=["x"]))  # the document's checksum term covers these
    assert t != shard.patch_term(6, p)
    q = dict(p, diffs=dict(p["diffs"], props={"k": {"1@aa": {"type": "value", "value": 2}}}))
    assert t != shard.patch_term(5, q)
    assert t != shard.patch_term(5, dict(p, clock={"aa": 2}))
