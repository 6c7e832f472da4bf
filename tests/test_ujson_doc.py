"""The UJSON path / JSON layer (jylis_amd/ujson_doc.py) and GET render.

* the reference's own example session (docs/_docs/types/ujson.md:107-132,
  tests/golden/kat_docs.json "ujson_doc") replayed on the oracle backend
  (CPU) and on the GPU engine, GET renders compared canonically (sets and
  maps are unordered in UJSON);
* the same session written on replica A and converged through A's flushed
  deltas into a fresh replica B (GPU), whose GETs must match the doc;
* random path-command streams on the GPU and on the oracle backend: equal
  renders and equal flushed deltas (the layer is shared, so this pins the
  engine's INS / RM / CLR under path-scoped CLR and SET);
* render / flatten / canonical unit cases from the primer (ujson.md:134-170).
"""
import json
import os

import numpy as np
import pytest

from jylis_amd import ujson_doc as U

HERE = os.path.dirname(__file__)
IDENT_A = 0x5EED_0000_0000_00A1
IDENT_B = 0x5EED_0000_0000_00B2


class OracleDocs:
    """backend adapter: the oracle's UJSON on opaque handles"""

    def __init__(self, repo):
        self.r = repo

    def write(self, cmds, identity):
        for c in cmds:
            if c[0] == "INS":
                self.r.ujson_ins(c[1], c[2])
            elif c[0] == "RM":
                self.r.ujson_rm(c[1], c[2])
            elif c[0] == "CLR":
                self.r.ujson_clr(c[1])
            else:
                self.r.ujson_touch(c[1])

    def _docs(self):
        t = self.r.state()
        ko, kb = np.asarray(t["key_offs"], np.uint64), np.asarray(t["key_bytes"], np.uint8)
        eo, el = np.asarray(t["el_offs"], np.uint64), np.asarray(t["elems"], np.uint64)
        return {bytes(kb[int(ko[i]):int(ko[i + 1])]).decode(): el[int(eo[i]):int(eo[i + 1])].tolist()
                for i in range(len(ko) - 1)}

    def exists(self, key):
        return key in self._docs()

    def elements(self, keys):
        d = self._docs()
        return {k: d[k] for k in keys if k in d}


def _session():
    return json.load(open(os.path.join(HERE, "golden", "kat_docs.json")))["ujson_doc"]["steps"]


def _replay(docs, steps, check=True):
    for st in steps:
        op, key, path = st[0], st[1], tuple(st[2])
        if op == "SET":
            docs.set(key, path, st[3])
        elif op == "INS":
            docs.ins(key, path, st[3])
        elif op == "RM":
            docs.rm(key, path, st[3])
        elif op == "CLR":
            docs.clr(key, path)
        elif op == "GET" and check:
            got = docs.get(key, path)
            assert U.canonical(got) == U.canonical(st[3]), (st, got)


# ---- CPU: the layer on the oracle backend -----------------------------------

def test_doc_session_oracle(oracle_mod):
    O = oracle_mod
    docs = U.UJSONDocs(OracleDocs(O.Repo(O.UJSON, IDENT_A)), IDENT_A)
    _replay(docs, _session())


def test_render_primer():
    # one value bare; several a set; a map merged into a set; empty vanishes
    assert U.render([((), '"a"')]) == '"a"'
    assert U.canonical(U.render([((), '"a"'), ((), "1")])) == U.canonical('[1,"a"]')
    leaves = [(("k",), "true"), ((), "null"), (("m", "x"), "2"), (("m", "y"), "3")]
    assert U.canonical(U.render(leaves)) == U.canonical('[null,{"k":true,"m":{"x":2,"y":3}}]')
    assert U.render([]) == ""
    # sets flatten; several maps in a set merge (ujson.md:160-170)
    assert U.flatten('[[1,2],[2,{"a":1}],{"b":2}]') == {((), "1"), ((), "2"), (("a",), "1"), (("b",), "2")}
    assert U.flatten("{}") == set()
    assert U.canonical('[{"a":1},{"b":2}]') == U.canonical('{"a":1,"b":2}')


def test_leaf_handles_stable():
    a, b = U.LeafTable(), U.LeafTable()
    assert a.handle(("x", "y"), '"v"') == b.handle(("x", "y"), '"v"')
    assert a.handle(("x", "y"), '"v"') != a.handle(("xy",), '"v"')
    assert a.handle((), "0") != 0


# ---- GPU ---------------------------------------------------------------------

@pytest.mark.gpu
def test_doc_session_gpu(engine):
    from jylis_amd.repo import RepoUJSON
    docs = U.UJSONDocs(U.GpuDocs(RepoUJSON(engine)), IDENT_A)
    _replay(docs, _session())


@pytest.mark.gpu
def test_doc_session_converge_path(engine):
    """A writes the session and flushes after every command (a node that
    gossips each write); a fresh replica B converges A's deltas in order and
    renders what the doc shows at every GET.  (Flushing per command matters:
    the pending delta takes an RM's dots into its context only, as the
    restated reference does, so an element inserted and removed inside one
    flush interval still travels in that delta's map -- see DESIGN.md.)"""
    import jylis_amd.engine as E
    from jylis_amd.repo import RepoUJSON
    leaves = U.LeafTable()
    A = U.UJSONDocs(U.GpuDocs(RepoUJSON(engine)), IDENT_A, leaves)
    engB = E.Engine(key_capacity=1 << 10, ujson_columns=engine.ujson_columns)
    B = U.UJSONDocs(U.GpuDocs(RepoUJSON(engB)), IDENT_B, leaves)
    for st in _session():
        if st[0] == "GET":
            assert U.canonical(B.get(st[1], tuple(st[2]))) == U.canonical(st[3]), st
            continue
        _replay(A, [st], check=False)
        B.b.r.converge_deltas(A.b.r.flush_deltas())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_path_commands_gpu_vs_oracle(oracle_mod, engine, seed):
    from jylis_amd.repo import RepoUJSON
    from test_ujson_write_gpu import _canon_ujson
    O = oracle_mod
    rng = np.random.default_rng(500 + seed)
    leaves = U.LeafTable()
    want_repo = O.Repo(O.UJSON, IDENT_A)
    got_repo = RepoUJSON(engine)
    want = U.UJSONDocs(OracleDocs(want_repo), IDENT_A, leaves)
    got = U.UJSONDocs(U.GpuDocs(got_repo), IDENT_A, leaves)
    keys = [f"u{i}" for i in range(5)]
    paths = [(), ("a",), ("a", "b"), ("c",), ("a", "c")]
    vals = ['"x"', '"y"', "1", "true", "null", '{"p":1}', '{"p":[1,2],"q":"z"}', "[3,4]"]
    for step in range(60):
        k = keys[int(rng.integers(0, len(keys)))]
        p = paths[int(rng.integers(0, len(paths)))]
        x = rng.random()
        v = vals[int(rng.integers(0, len(vals)))]
        for d in (want, got):
            if x < 0.35:
                if not v.startswith(("{", "[")):
                    d.ins(k, p, v)
            elif x < 0.55:
                if not v.startswith(("{", "[")):
                    d.rm(k, p, v)
            elif x < 0.75:
                d.set(k, p, v)
            else:
                d.clr(k, p)
        if step % 7 == 6:
            for q in paths:
                assert [U.canonical(t) for t in got.get_many(keys, q)] == \
                       [U.canonical(t) for t in want.get_many(keys, q)]
            assert got_repo.deltas_size() == want_repo.deltas_size()
            if rng.random() < 0.5:
                assert _canon_ujson(got_repo.flush_deltas()) == _canon_ujson(want_repo.flush().table())
    assert _canon_ujson(got_repo.flush_deltas()) == _canon_ujson(want_repo.flush().table())
