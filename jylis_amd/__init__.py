"""jylis_amd -- MI355X-native CRDT delta-convergence engine for Jylis.

The engine (libjylis_gpu.so, include/jylis_gpu.h) replaces the per-key loop of
RepoManagerCore.converge_deltas (jylis/repo_manager.pony:92-93) with one
batched HIP call per delta batch.  See DESIGN.md.
"""
from ._lib import DEVICE, GCOUNT, HOST, PNCOUNT, TLOG, TREG, TYPE_NAMES, UJSON  # noqa: F401

__all__ = ["GCOUNT", "PNCOUNT", "TREG", "TLOG", "UJSON", "TYPE_NAMES", "HOST", "DEVICE"]
