"""bench.py's N>1 path on one GPU: two ranks (torch.distributed.run, gloo exchange, both on
device 0) split the C4 job by document hash (workload.c4_shard), each runs its shard
through the pipeline, and the all-gathered totals and digests -- of the merged documents and of
their applyChanges patches -- equal the single-rank run's and the oracle's pinned digests of the
same documents (tests/golden/c4_digest.json)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = 65536


def _run(cmd, extra_env):
    env = dict(os.environ)
    env.update(extra_env)
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_two_ranks_equal_one_rank():
    args = ["bench.py", "--docs", str(DOCS), "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--check", "4"]
    one = _run([sys.executable] + args, {})
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", "29517"] + args,
               {"AM_DIST_BACKEND": "gloo", "AM_BENCH_DEVICE": "0", "OMP_NUM_THREADS": "4"})
    rec = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_digest.json")))[str(DOCS)]
    pinned, pinned_p = rec["digest"], rec["patch_digest"]
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    for r in (one, two):
        assert r["config"]["total_docs"] == DOCS and r["errors"] == 0
        assert r["digest"] == pinned and r["digest_pinned"]["match"]
        # every document's applyChanges patch against the oracle's (clock + diffs, shard.patch_term)
        assert r["patch_digest"] == pinned_p and r["digest_pinned"]["patches"]["match"]
    assert two["config"]["docs_rank0"] < DOCS  # rank 0 merged only its shard
    assert one["output_bytes_rank0"] > two["output_bytes_rank0"]


def test_nccl_branch_on_one_rank():
    """bench.py's RCCL path (init_process_group('nccl') bound to the device, the digest all-gather of
    device tensors, the NUMA report's all_gather_object) on one rank of one GPU: the driver's
    multi-GPU run takes this branch with N ranks."""
    args = ["bench.py", "--docs", str(DOCS), "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--check", "4"]
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
              "--master-addr", "127.0.0.1", "--master-port", "29519"] + args, {"AM_DIST_FORCE": "1"})
    rec = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_digest.json")))[str(DOCS)]
    assert r["dist"]["backend"] == "nccl" and r["dist"]["world_size"] == 1
    assert r["errors"] == 0 and r["digest"] == rec["digest"] and r["patch_digest"] == rec["patch_digest"]
