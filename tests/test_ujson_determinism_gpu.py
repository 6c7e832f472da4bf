"""The UJSON converge is a function of its inputs: the config-5-shaped
sequence (Zipf hot documents whose clouds span many tiles, converges
pipelined without host synchronisation) repeated on fresh engines must leave
the same store every time.  Round 3 found U3's long-document folds reading
the version-vector row twice while other waves raised it; that race showed
at config 5 (tools/uj_repro.py, 1M documents: 3 distinct stores in 5 runs,
profiles/r03_ujrepro.log) but not at this test's 64K documents, so this is
a guard of the property at test scale, and uj_repro the reproduction."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(st, dl):
    import torch
    from bench_modes import _to_dev
    from jylis_amd._lib import UJSON
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    dev = torch.device("cuda", 0)
    eng = Engine(device=0)
    try:
        repo = RepoUJSON(eng)
        repo.converge_deltas(st)
        batches = []
        for b in dl:
            slots = eng.lookup(UJSON, (b["key_bytes"], b["key_offs"]))
            eo, vo, co = (np.asarray(b[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
            dots, elems = repo._sort_segments(eo, repo._pack(b["dot_ids"], b["dot_seqs"]), np.asarray(b["elems"]))
            (vv,) = repo._sort_segments(vo, repo._pack(b["vv_ids"], b["vv_seqs"]))
            (cloud,) = repo._sort_segments(co, repo._pack(b["cloud_ids"], b["cloud_seqs"]))
            batches.append(tuple(_to_dev(a, dev) for a in (slots, eo, dots, elems, vo, vv, co, cloud)))
        eng.sync()
        for b in batches:  # pipelined: no synchronisation between converges
            eng.ujson_converge(*b)
        eng.sync()
        h = hashlib.sha1()
        for a in eng.ujson_read(np.arange(eng.nkeys(UJSON), dtype=np.uint32)):
            h.update(np.ascontiguousarray(a).tobytes())
        return h.hexdigest(), eng.ujson_stats()
    finally:
        eng.close()


def test_pipelined_converges_are_deterministic():
    from jylis_amd import synth as S
    st, dl = S.ujson_tables(1 << 16, seed=S.BASE_SEED + 31, rounds=10, R=16)
    runs = [_run(st, dl) for _ in range(4)]
    assert runs[0][1]["touched_cloud"] > 0
    assert len({h for h, _ in runs}) == 1, [h for h, _ in runs]
