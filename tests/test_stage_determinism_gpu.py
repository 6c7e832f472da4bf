"""Determinism of the host-staged converge path at config-5 scale: the same
UJSON state and delta batches, handed over as HOST tables (chunked parallel
pinned staging, host_copy.hip), converged on two engines, must give two
identical stores -- document by document, elements, version vectors and
clouds.  (A staging race would corrupt some chunk of one engine's inputs.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dump(eng, n):
    from jylis_amd._lib import UJSON
    slots = np.arange(n, dtype=np.uint32)
    return eng.ujson_read(slots)


def test_host_staged_ujson_identical_on_two_engines():
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    D = 1 << 19
    st, dl = S.ujson_tables(D, seed=S.BASE_SEED + 77, rounds=3, R=16)
    engs = [Engine(device=0), Engine(device=0)]
    try:
        for e in engs:
            r = RepoUJSON(e)
            r.converge_deltas(st)
            for b in dl:
                r.converge_deltas(b)
            e.sync()
        n = engs[0].nkeys(4)
        assert n == engs[1].nkeys(4) == D
        a, b = _dump(engs[0], n), _dump(engs[1], n)
        for x, y, name in zip(a, b, ("el_offs", "dots", "elems", "vv", "cloud_offs", "cloud")):
            assert np.array_equal(x, y), f"{name} differs between two engines fed the same host batches"
    finally:
        for e in engs:
            e.close()
