"""sync.js Bloom filter + change selection kernels on the GPU (am_sync.hip) against the reference's
vectors (tests/golden/bloom.json) and the CPU oracle on seeded batches."""
import random

import pytest

import oracle_ffi as O
from conftest import golden

pytestmark = pytest.mark.gpu


def test_gpu_bloom_matches_reference_vectors():
    from automerge_amd import sync
    vecs = golden("bloom.json")
    filters = sync.build_filters([v["hashes"] for v in vecs])
    assert [f.hex() for f in filters] == [v["bytes"] for v in vecs]
    probes = [(i, h) for i, v in enumerate(vecs) for h in v["probes"]]
    expect = [bool(c) for v in vecs for c in v["contains"]]
    assert sync.probe(filters, probes) == expect
    bf = sync.BloomFilter(vecs[1]["hashes"])
    assert bf.bytes.hex() == vecs[1]["bytes"]
    assert all(bf.containsHash(h) for h in vecs[1]["hashes"])


def test_gpu_bloom_seeded_batch_matches_oracle():
    from automerge_amd import sync
    rnd = random.Random(7)
    lists = [[rnd.randbytes(32) for _ in range(rnd.choice([0, 1, 10, 10, 10, 37, 51, 52, 300]))] for _ in range(3000)]
    filters = sync.build_filters(lists)
    for hs, f in zip(lists, filters):
        assert f == O.bloom_build(hs)
    probes = [(rnd.randrange(len(lists)), rnd.randbytes(32)) for _ in range(20000)]
    got = sync.probe(filters, probes)
    assert got == [O.bloom_contains(filters[i], h) == 1 for i, h in probes]


def test_gpu_bloom_malformed_filter_raises_reference_error():
    from automerge_amd import _native as N
    from automerge_amd import sync
    good = sync.build_filters([[bytes(range(32))]])[0]
    with pytest.raises(N.AutomergeError, match="subarray exceeds buffer size"):
        sync.BloomFilter(good[:-1])
    with pytest.raises(N.AutomergeError, match="buffer ended with incomplete number"):
        sync.BloomFilter(b"\x80")
    with pytest.raises(N.AutomergeError, match="Not a 256-bit hash"):
        sync.BloomFilter(good).containsHash("abcd")


def test_gpu_select_changes_matches_oracle():
    from automerge_amd import sync
    rnd = random.Random(9)
    pairs = []
    for _ in range(2000):
        n = rnd.randint(0, 12)
        hashes = [rnd.randbytes(32) for _ in range(n)]
        deps = [[rnd.randint(-1, i - 1) for _ in range(rnd.randint(0, 2))] if i else [] for i in range(n)]
        filters = [O.bloom_build([h for h in hashes if rnd.random() < 0.7]) for _ in range(rnd.randint(1, 2))]
        pairs.append((hashes, deps, filters))
    got = sync.select_changes(pairs)
    for (hashes, deps, filters), g in zip(pairs, got):
        assert g == O.sync_select(hashes, deps, filters)


def test_gpu_bloom_edge_vectors_match_reference():
    """numProbes 0/1/2 and sparse filters (tests/golden/bloom_edge.json) probed on the GPU."""
    from automerge_amd import _native as N
    from automerge_amd import sync
    good = [v for v in golden("bloom_edge.json") if not v["error"]]
    filters = [bytes.fromhex(v["bytes"]) for v in good]
    probes = [(i, h) for i, v in enumerate(good) for h in v["probes"]]
    assert sync.probe(filters, probes) == [bool(c) for v in good for c in v["contains"]]
    for v in golden("bloom_edge.json"):
        if v["error"]:
            with pytest.raises(N.AutomergeError, match=v["error"]["message"]):
                sync.BloomFilter(bytes.fromhex(v["bytes"]))


def test_gpu_select_rejects_malformed_second_filter():
    """The reference decodes every `have` filter before selecting (sync.js:252-256): a malformed
    second filter raises even when the first already contains every change, and a pair with no
    changes still raises."""
    from automerge_amd import _native as N
    from automerge_amd import sync
    rnd = random.Random(3)
    hashes = [rnd.randbytes(32) for _ in range(3)]
    first = O.bloom_build(hashes)
    bad = first[:-1]
    with pytest.raises(N.AutomergeError, match="subarray exceeds buffer size"):
        sync.select_changes([(hashes, [[], [0], [1]], [first, bad])])
    with pytest.raises(N.AutomergeError, match="buffer ended with incomplete number"):
        sync.select_changes([([], [], [first, b"\x80"])])
