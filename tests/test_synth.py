"""The synthetic stream generators (jylis_amd/synth.py) are test and bench
infrastructure: the vectorised UJSON round reproduces the per-op form it
replaced bit for bit, so the config-5 sequence (and its full-size golden
digests, tests/golden/fullsize_digests.json) did not change with it."""
import numpy as np
import pytest


@pytest.mark.parametrize("D,seed,rounds", [(500, 1, 4), (3000, 2, 3), (20000, 3, 2), (1 << 20, 0x4A594C4953 + 5, 1)])
def test_ujson_round_vectorised_matches_per_op(D, seed, rounds):
    from jylis_amd import synth as S
    st, dl = S.ujson_tables(D, seed=seed, rounds=rounds, R=16)
    # the reference: the same state draws, then per-op rounds
    import jylis_amd.synth as mod
    saved = mod._ujson_round
    try:
        mod._ujson_round = mod._ujson_round_ref
        st2, dl2 = S.ujson_tables(D, seed=seed, rounds=rounds, R=16)
    finally:
        mod._ujson_round = saved
    for k in st:
        np.testing.assert_array_equal(st[k], st2[k])
    assert len(dl) == len(dl2)
    for a, b in zip(dl, dl2):
        assert set(a) == set(b)
        for k in a:
            np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)
