"""Document sharding across ranks: one process per GPU, documents are
independent, so rank r merges documents [r*D, (r+1)*D) with no collective on the data path.
The only exchange is one all-gather of a small per-rank digest after the timed region (RCCL over
xGMI on the GPU box; gloo in the CPU tests)."""

DIGEST_FIELDS = ("docs", "ops", "errors", "out_bytes", "out_xor")


def shard_range(rank, world, docs_per_rank):
    """Documents [first, first + n) merged by `rank` (weak scaling: n fixed per rank)."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    return rank * docs_per_rank, docs_per_rank


def out_digest(res):
    """Order-independent digest of a batch's results (numpy structured array of am_doc_result)."""
    import numpy as np
    x = np.bitwise_xor.reduce(res["out_len"].astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) if len(res) else 0
    return int(x) & 0x7FFFFFFFFFFFFFFF


def exchange(dist, digest, device):
    """All-gather of the per-rank digest (len(DIGEST_FIELDS) int64); returns the summed fields
    (out_xor is XOR-combined) and the per-rank rows. `dist` None means a single process."""
    import torch
    t = torch.tensor([int(v) for v in digest], dtype=torch.int64, device=device)
    if dist is None:
        rows = [t.tolist()]
    else:
        parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
        rows = [p.tolist() for p in parts]
    tot = [sum(r[i] for r in rows) for i in range(len(DIGEST_FIELDS) - 1)]
    x = 0
    for r in rows:
        x ^= r[-1]
    return tot + [x], rows
