"""The Pony glue (pony/jylis_gpu/*.pony) cannot be compiled here (no ponyc,
SURVEY.md 8c), so its FFI surface is checked against the boundary it binds:
every `use @jy_...` declaration names a symbol include/jylis_gpu.h declares,
with the same number of parameters, and the library exports it; every
`@jy_...` call in the glue is declared; the GPU repos share ONE node per
process (jy_node_acquire_local, database.pony:18-22's five RepoManagers) and
bracket their engine use with the node lock.  Runs without a GPU."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PONY = os.path.join(ROOT, "pony", "jylis_gpu")
HEADER = os.path.join(ROOT, "include", "jylis_gpu.h")


def _split_top(s):
    """parameters split at top-level commas (brackets and parentheses nest)"""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def header_arity():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(jy_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else len(_split_top(params))
    return out


def pony_decls():
    text = open(os.path.join(PONY, "ffi.pony")).read()
    text = re.sub(r"//[^\n]*", "", text)
    out = {}
    for m in re.finditer(r"use\s+@(jy_[a-z0-9_]+)\[[^\n]*?\]\((.*?)\)\s*(?=\n\S|\Z)", text, flags=re.S):
        params = " ".join(m.group(2).split())
        out[m.group(1)] = 0 if not params else len(_split_top(params))
    return out


def test_every_declaration_matches_the_header():
    hdr, decl = header_arity(), pony_decls()
    assert len(decl) > 50
    unknown = sorted(set(decl) - set(hdr))
    assert not unknown, f"ffi.pony declares symbols the header does not: {unknown}"
    wrong = {s: (decl[s], hdr[s]) for s in decl if decl[s] != hdr[s]}
    assert not wrong, f"parameter counts differ (pony, header): {wrong}"


def test_every_call_is_declared_and_exported():
    import ctypes as C
    lib = C.CDLL(os.path.join(ROOT, "jylis_amd", "libjylis_gpu.so"))
    decl = pony_decls()
    used = set()
    for f in os.listdir(PONY):
        if f.endswith(".pony") and f != "ffi.pony":
            body = re.sub(r"//[^\n]*", "", open(os.path.join(PONY, f)).read())
            body = re.sub(r"^use @[^\n]*", "", body, flags=re.M)
            used |= set(re.findall(r"@(jy_[a-z0-9_]+)\(", body))
    assert used, "the glue makes no FFI call"
    missing = sorted(used - set(decl))
    assert not missing, f"called but not declared in ffi.pony: {missing}"
    assert all(hasattr(lib, s) for s in decl)


def test_one_node_per_process_and_locked_engine_use():
    eng = open(os.path.join(PONY, "engine.pony")).read()
    assert "@jy_node_acquire_local" in eng and "@jy_node_release" in eng
    assert "@jy_node_create_local" not in eng  # (round 4 made one node, one communicator, per type)
    for f in ("repo_counters_gpu.pony", "repo_logs_gpu.pony", "repo_ujson_gpu.pony"):
        body = open(os.path.join(PONY, f)).read()
        assert "_Lock(_node)" not in body  # every lock names the jobs it waits for (jy_node_lock_type)
        locks = re.findall(r"_Lock\(_node, (Jy\w+)\(\)\)", body)
        assert len(locks) == body.count("_Unlock(_node)") - body.count("_Unlock(_node); error")
        assert set(locks) <= {"JyNoFence", "JyGCOUNT", "JyPNCOUNT", "JyTREG", "JyTLOG", "JyUJSON"}
        # a drain only enqueues (round 6, verdict r5 #3): no lock, no arena
        # collection on the scheduler thread -- the node's worker reclaims arenas
        for m in re.finditer(r"\n  fun ref _drain\(", body):
            nxt = body.find("\n  fun ", m.end())
            seg = body[m.end():nxt if nxt > 0 else len(body)]
            for bad in ("lock(", "_Lock(", "maybe_collect", "@jy_node_sync", "@jy_node_fence"):
                assert bad not in seg, f"{f}: _drain calls {bad}"
        # a method that touches an owner shard is a locked wrapper's inner half
        for m in re.finditer(r"\n  fun ref (\w+)\(", body):
            name = m.group(1)
            nxt = body.find("\n  fun ", m.end())
            seg = body[m.end():nxt if nxt > 0 else len(body)]
            if "n.owner(" in seg or "@jy_treg_deltas_size" in seg or "node.shards" in seg:
                assert name.startswith("_"), f"{f}: {name} uses the engines outside the node lock"


def test_typed_locks_and_worker_side_arena_gc():
    """reads and writes wait for their own type's queued converges only;
    deltas_size / flush for none; the node's worker reclaims arenas; a
    replica id -> column lookup is cached per repo"""
    eng = open(os.path.join(PONY, "engine.pony")).read()
    assert "@jy_node_lock_type(ptr, ty)" in eng and "@jy_node_arena_gc(ptr, 1)" in eng
    assert "_cols(id)" in eng  # replica_col cache
    for f, ty in (("repo_counters_gpu.pony", ("JyGCOUNT", "JyPNCOUNT")), ("repo_logs_gpu.pony", ("JyTREG", "JyTLOG")),
                  ("repo_ujson_gpu.pony", ("JyUJSON",))):
        body = open(os.path.join(PONY, f)).read()
        for m in re.finditer(r"\n  fun ref (deltas_size|flush_deltas)\(", body):
            nxt = body.find("\n  fun ", m.end())
            seg = body[m.end():nxt if nxt > 0 else len(body)]
            assert "_Lock(_node, JyNoFence())" in seg, f"{f}: {m.group(1)} fences converges it does not read"
        for t in ty:
            assert f"_Lock(_node, {t}())" in body
