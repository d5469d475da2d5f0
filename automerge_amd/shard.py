"""Document sharding across ranks: one process per GPU, documents are
independent, so there is no collective on the data path. The C4 job is sharded by document hash
(rank = first byte of the SHA-256 of the base document chunk, i.e. its container checksum
columnar.js:659-686, mod N: workload.c4_shard); shard_range is the plain range split other
workloads use. The only exchange is one all-gather of a small per-rank digest after the timed
region (RCCL over xGMI on the GPU box; gloo in the CPU tests)."""

DIGEST_FIELDS = ("docs", "ops", "errors", "out_bytes", "out_digest", "patch_digest")


def shard_range(rank, world, docs_per_rank):
    """Documents [first, first + n) merged by `rank` (weak scaling: n fixed per rank)."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    return rank * docs_per_rank, docs_per_rank


M64 = (1 << 64) - 1


def _mix64(x):
    """splitmix64 finalizer (the device's mix64 in am_kernels.hip)."""
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & M64
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def doc_digest(index, status, out):
    """Digest term of one document: its global index, the container checksum (bytes 4..8 of the
    merged chunk, columnar.js:659-686), its length and status. Equal lengths no longer cancel,
    and a wrong or missing byte anywhere in a document changes its checksum."""
    chk = int.from_bytes(out[4:8], "little") if status == 0 and len(out) >= 8 else 0
    n = len(out) if status == 0 else 0
    return (_mix64(((index << 32) | chk) & M64) + n * 0x9E3779B97F4A7C15 + status) & M64


def shard_of(doc_bytes, world):
    """Rank of a document (the base document chunk): SHA-256(chunk)[0] mod world, read from the
    container checksum (bytes 4..8 of the chunk are the first four bytes of that hash)."""
    return doc_bytes[4] % world


def doc_digest_np(index, status, out_len, chk):
    """doc_digest over arrays (numpy uint64, wrapping arithmetic); returns the combined digest."""
    import numpy as np
    index = np.asarray(index, np.uint64)
    status = np.asarray(status, np.uint64)
    ok = status == 0
    chk = np.where(ok, np.asarray(chk, np.uint64), np.uint64(0))
    n = np.where(ok, np.asarray(out_len, np.uint64), np.uint64(0))
    with np.errstate(over="ignore"):
        x = (index << np.uint64(32)) | chk
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
        t = x + n * np.uint64(0x9E3779B97F4A7C15) + status
        return int(t.sum(dtype=np.uint64)) & 0x7FFFFFFFFFFFFFFF


def _hexb(v):
    return bytes(v).hex()


def patch_canon(p):
    """The part of an applyChanges patch the device writes (new.js:1862-1865: clock and diffs; deps and
    maxOp follow from the merged document, which its checksum term covers) as canonical JSON."""
    import json
    return json.dumps({"clock": p["clock"], "diffs": p["diffs"]}, sort_keys=True, separators=(",", ":"),
                      default=_hexb).encode()


def patch_term(index, p):
    """Digest term of one document's patch: its global index mixed with the first 8 bytes of the
    SHA-256 of patch_canon(p) (summed mod 2^63 like the document terms)."""
    import hashlib
    h = int.from_bytes(hashlib.sha256(patch_canon(p)).digest()[:8], "little")
    return _mix64(h ^ _mix64(index & M64))


def patch_terms_of_logs(ids, logs):
    """Sum of patch_term over the engine's wire-form patch logs (automerge_amd/patch.py materializes
    them; a failed document's term is 0)."""
    from . import patch as P
    t = 0
    for i, log in zip(ids, logs):
        if log:
            t += patch_term(int(i), P.materialize(log, [], 0, 0))
    return t & 0x7FFFFFFFFFFFFFFF


def combine(terms):
    """Sum of per-document terms mod 2^63 (order independent; am_batch_digest computes the same)."""
    return sum(terms) & 0x7FFFFFFFFFFFFFFF


def exchange(dist, digest, device):
    """All-gather of the per-rank digest (len(DIGEST_FIELDS) int64); returns the summed fields
    (out_digest summed mod 2^63) and the per-rank rows. `dist` None means a single process."""
    import torch
    t = torch.tensor([int(v) for v in digest], dtype=torch.int64, device=device)
    if dist is None:
        rows = [t.tolist()]
    else:
        parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
        rows = [p.tolist() for p in parts]
    k = len(digest) - 2  # the last two fields are digests (summed mod 2^63)
    tot = [sum(r[i] for r in rows) for i in range(k)]
    return tot + [combine(r[j] for r in rows) for j in range(k, len(digest))], rows
