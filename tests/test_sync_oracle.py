"""CPU oracle of the sync.js Bloom filter (sync.js:38-125) and getChangesToSend selection
(sync.js:246-306) against tests/golden/bloom.json, which the reference produced."""
import random

import oracle_ffi as O
from conftest import golden


def test_bloom_bytes_and_probes_match_reference():
    vecs = golden("bloom.json")
    assert len(vecs) >= 40
    for v in vecs:
        hashes = [bytes.fromhex(h) for h in v["hashes"]]
        f = O.bloom_build(hashes)
        assert f.hex() == v["bytes"]
        for h in hashes:  # no false negatives
            assert O.bloom_contains(f, h) == 1
        for h, c in zip(v["probes"], v["contains"]):
            assert O.bloom_contains(f, bytes.fromhex(h)) == int(c)


def test_bloom_malformed_filters():
    f = O.bloom_build([bytes(range(32))])
    assert O.bloom_contains(f[:-1], bytes(range(32))) == -1  # bits shorter than the header says
    assert O.bloom_contains(b"\\x80", bytes(32)) == -1        # incomplete number
    assert O.bloom_contains(b"", bytes(32)) == 0              # empty filter contains nothing


def test_select_transitive_dependents():
    rnd = random.Random(5)
    hashes = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(6)]
    # chain 0 <- 1 <- 2, and 3 <- 4; 5 independent
    deps = [[-1], [0], [1], [], [3], []]
    have = O.bloom_build([hashes[i] for i in (0, 1, 2, 3, 5)])  # 4 is bloom-negative
    send = O.sync_select(hashes, deps, [have])
    assert send[4] == 1 and send[0] == 0 and send[5] == 0
    have2 = O.bloom_build([hashes[i] for i in (1, 2, 3, 4, 5)])  # 0 negative -> 1, 2 follow
    assert O.sync_select(hashes, deps, [have2])[:3] == [1, 1, 1]
    # a change present in either filter is not sent
    assert O.sync_select(hashes, deps, [have, have2])[0] == 0 or O.bloom_contains(have, hashes[0]) == 0


def test_bloom_edge_vectors_match_reference():
    """numProbes 0/1/2/7, 0-3 bits per entry and malformed headers (tests/golden/bloom_edge.json,
    made by the reference's BloomFilter): containsHash results and decode errors."""
    for v in golden("bloom_edge.json"):
        f = bytes.fromhex(v["bytes"])
        for i, h in enumerate(v["probes"]):
            got = O.bloom_contains(f, bytes.fromhex(h))
            if v["error"]:
                assert got == -1, v
            else:
                assert got == int(v["contains"][i]), (v["bytes"], i)
