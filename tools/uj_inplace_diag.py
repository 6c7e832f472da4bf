"""UJSON in-place layout diagnostics: the config-5 stream converged one batch
at a time (synchronised), with the engine's counters per converge
(jy_ujson_stats_ext) and the wall time of each converge.

usage: python tools/uj_inplace_diag.py [DOCS] [ROUNDS] [LONG_MIN]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    from jylis_amd import synth as S
    from jylis_amd.engine import Engine
    from jylis_amd.repo import RepoUJSON
    from jylis_amd._lib import UJSON
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    lm = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    st, dl = S.ujson_tables(D, seed=S.BASE_SEED + 5, rounds=rounds, R=16)
    eng = Engine(device=0, ujson_columns=16)
    eng.ujson_set_inplace(lm)
    repo = RepoUJSON(eng)
    repo.converge_deltas(st)
    eng.sync()
    prev = eng.ujson_stats()
    for r, b in enumerate(dl):
        slots = eng.lookup(UJSON, (b["key_bytes"], b["key_offs"]))
        eo, vo, co = (np.asarray(b[k], np.uint64) for k in ("el_offs", "vv_offs", "cloud_offs"))
        dots, elems = repo._sort_segments(eo, repo._pack(b["dot_ids"], b["dot_seqs"]), np.asarray(b["elems"]))
        (vv,) = repo._sort_segments(vo, repo._pack(b["vv_ids"], b["vv_seqs"]))
        (cloud,) = repo._sort_segments(co, repo._pack(b["cloud_ids"], b["cloud_seqs"]))
        t0 = time.perf_counter()
        eng.ujson_converge(slots, eo, dots, elems, vo, vv, co, cloud)
        eng.sync()
        t1 = time.perf_counter()
        cur = eng.ujson_stats()
        d = {k: cur[k] - prev[k] for k in cur}
        prev = cur
        print(f"round {r}: {1e3 * (t1 - t0):7.3f} ms  " + " ".join(f"{k}={v}" for k, v in d.items() if v), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
