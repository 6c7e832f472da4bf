"""The chunked parallel host staging (host_copy.hip) under repetition: long
TREG values packed from host memory go host -> pinned (worker threads, 1-MiB
chunks) -> device (one DMA per chunk, issued as each chunk lands) -> arena,
and are read back whole.  Every byte must survive, on every repetition, for
sizes that end in a partial chunk."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_staged_bytes_survive_repetition(engine):
    from jylis_amd._lib import TREG
    rng = np.random.default_rng(11)
    for rep in range(24):
        n = int(rng.integers(150_000, 400_000))
        lens = rng.integers(9, 200, n)  # every value long: its bytes go through the arena
        offs = np.zeros(n + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        vb = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
        pre, lr = engine.pack_values(TREG, (vb, offs))
        at = (lr >> np.uint64(24)).astype(np.int64)
        lo, hi = int(at[0]), int(at[-1] + lens[-1])
        got = np.frombuffer(engine.arena_read(TREG, lo, hi - lo), np.uint8)
        # every value, vectorised: the packed arena is the values back to back on 8-byte granules
        pad = (lens + 7) // 8 * 8
        starts = at - lo
        idx = np.repeat(starts, lens) + (np.arange(int(lens.sum())) - np.repeat(offs[:-1].astype(np.int64), lens))
        assert np.array_equal(got[idx], vb), f"rep {rep}: staged bytes differ"
        assert (starts[1:] - starts[:-1] == pad[:-1]).all()


def test_readback_survives_repetition(engine):
    """device -> pinned -> host through the copy pool (jy_readback): the slots
    of large host key batches (4 B a key, several MiB) read back on every
    repetition, against the first-occurrence slots of a dict"""
    from jylis_amd._lib import GCOUNT
    from jylis_amd.engine import encode_keys
    rng = np.random.default_rng(12)
    n = 1_500_003
    universe = 2_000_000
    table = {}
    for rep in range(12):
        ids = rng.integers(0, universe, n)
        kb, ko = encode_keys([b"r%08d" % i for i in ids.tolist()])
        want = np.empty(n, np.uint32)
        for j, i in enumerate(ids.tolist()):
            want[j] = table.setdefault(i, len(table))
        got = engine.intern(GCOUNT, (kb, ko))
        assert np.array_equal(got, want), f"rep {rep}: {np.count_nonzero(got != want)} slots differ"
        got2 = engine.lookup(GCOUNT, (kb, ko))
        assert np.array_equal(got2, want), f"rep {rep} (lookup)"
