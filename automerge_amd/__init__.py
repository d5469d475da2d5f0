"""automerge_amd -- MI355X batched merge engine for Automerge documents.

The hot path of the reference backend (backend/columnar.js change/document decoding and
backend/new.js applyChanges/save) runs as HIP kernels in libautomerge_amd.so. This package is the
host side: `backend` mirrors the reference's Backend module (backend/backend.js), `batch` exposes
the batched API (thousands of documents per launch).
"""
from . import _native  # noqa: F401  (fails loudly if the HIP library is missing)

__all__ = ["backend", "batch"]
