"""UJSON documents above the dot kernel: paths, JSON leaves and rendering.

Mirrors RepoUJSON's command surface (repo_ujson.pony:68-110) and the UJSON
data model of docs/_docs/types/ujson.md:134-170 ("the world is flat"): a
document is a set of (path, value) leaves, each an element of the engine's
observed-remove dot kernel.  The engine stores elements as opaque u64
handles; this module owns the mapping.

  GET key [path...]         render the leaves at or under path ('' if none)
  SET key [path...] ujson   CLR path, then INS every leaf of the parsed node
  CLR key [path...]         remove every leaf at or under path (no key creation)
  INS key [path...] value   add the leaf (path, value)
  RM  key [path...] value   remove the leaf (path, value) (no key creation)

Handles are a 64-bit hash (FNV-1a) of the canonical (path, value) encoding
(each path segment length-prefixed, then 0xFFFFFFFF, then the value), so every
replica derives the same handle for the same leaf (the CRDT compares elements
by handle); `LeafTable` keeps handle -> leaf for rendering and refuses a hash
collision.  Rendering follows the primer: maps render as objects, several
values at one path as an unordered set '[...]', one value bare, at most one
merged map inside a set, nothing for empty collections.  Set and map order is
not specified by the reference (pony Map iteration); this module renders keys
and set members in sorted order, and tests compare renders canonically
(`canonical`)."""
import json

import numpy as np


def canonical_value(text):
    """a UJSON primitive (UJSONParse.value) -> its canonical JSON text"""
    v = json.loads(text)
    if isinstance(v, (dict, list)):
        raise ValueError("a UJSON value is a primitive (string, number, boolean, null)")
    return _dump(v)


def _dump(v):
    if isinstance(v, bool) or v is None or isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return repr(v)
    raise ValueError(f"not a JSON primitive: {v!r}")


def flatten(text, prefix=()):
    """UJSONParse.node: a JSON document -> set of (path, canonical value)
    leaves; arrays are sets (flattened into the enclosing path)"""
    out = set()

    def walk(v, path):
        if isinstance(v, dict):
            for k, x in v.items():
                walk(x, path + (str(k),))
        elif isinstance(v, list):
            for x in v:
                walk(x, path)
        else:
            out.add((path, _dump(v)))
    walk(json.loads(text), tuple(prefix))
    return out


def _fnv1a64(b):
    h = 0xCBF29CE484222325
    for x in b:
        h = ((h ^ x) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _encode(path, value):
    b = bytearray()
    for p in path:
        e = p.encode()
        b += len(e).to_bytes(4, "little") + e
    b += b"\xff\xff\xff\xff" + value.encode()
    return bytes(b)


class LeafTable:
    """(path, value) <-> u64 handle; one table serves every replica of a process"""

    def __init__(self):
        self._leaf = {}

    def handle(self, path, value):
        path = tuple(path)
        # FNV-1a 64 of the encoding (the Pony glue computes the same handle);
        # handle 0 is reserved: "no element" (the engine's key-touching RM)
        h = _fnv1a64(_encode(path, value)) or 1
        old = self._leaf.setdefault(h, (path, value))
        if old != (path, value):
            raise RuntimeError(f"64-bit leaf handle collision: {old} vs {(path, value)}")
        return h

    def leaf(self, h):
        return self._leaf[int(h)]


def render(leaves):
    """leaves [(relative path, value)] -> UJSON text ('' when empty)"""
    if not leaves:
        return ""
    root = {"v": set(), "m": {}}
    for path, value in leaves:
        n = root
        for p in path:
            n = n["m"].setdefault(p, {"v": set(), "m": {}})
        n["v"].add(value)

    def out(n):
        items = sorted(n["v"])
        m = {k: c for k, c in n["m"].items() if _nonempty(c)}
        if m:
            items.append("{" + ",".join(json.dumps(k, ensure_ascii=False) + ":" + out(m[k]) for k in sorted(m)) + "}")
        if len(items) == 1:
            return items[0]
        return "[" + ",".join(items) + "]"
    return out(root)


def _nonempty(n):
    return bool(n["v"]) or any(_nonempty(c) for c in n["m"].values())


def canonical(text):
    """a UJSON render -> a comparable structure (sets and maps unordered)"""
    if text == "":
        return None

    def canon(v):
        if isinstance(v, dict):
            return ("map", frozenset((k, canon(x)) for k, x in v.items()))
        if isinstance(v, list):
            flat = set()
            maps = {}
            for x in v:
                c = canon(x)
                if c[0] == "set":
                    flat |= c[1]
                elif c[0] == "map":
                    maps.update(dict(c[1]))
                else:
                    flat.add(c)
            if maps:
                flat.add(("map", frozenset(maps.items())))
            return ("set", frozenset(flat)) if len(flat) != 1 else next(iter(flat))
        return ("val", _dump(v))
    return canon(json.loads(text))


class UJSONDocs:
    """RepoUJSON's commands over a dot-kernel backend (the GPU RepoUJSON, or
    the oracle in tests).  backend: write(cmds, identity) with ("INS", key,
    h) / ("RM", key, h) / ("CLR", key) / ("TOUCH", key) (create the key and
    its delta, change nothing); elements(keys) -> {key: [handles]};
    exists(key)."""

    def __init__(self, backend, identity, leaves=None):
        self.b = backend
        self.identity = identity
        self.leaves = leaves if leaves is not None else LeafTable()

    def _under(self, key, path):
        path = tuple(path)
        hs = self.b.elements([key]).get(key, [])
        out = set()
        for h in set(int(x) for x in hs):
            p, v = self.leaves.leaf(h)
            if p[:len(path)] == path:
                out.add(h)
        return out

    def get(self, key, path=()):
        """GET (repo_ujson.pony:68-72)"""
        return self.get_many([key], path)[0]

    def get_many(self, keys, path=()):
        """GET for many docs with one engine read"""
        path = tuple(path)
        els = self.b.elements(list(keys))
        out = []
        for k in keys:
            leaves = []
            for h in set(int(x) for x in els.get(k, [])):
                p, v = self.leaves.leaf(h)
                if p[:len(path)] == path:
                    leaves.append((p[len(path):], v))
            out.append(render(leaves))
        return out

    def ins(self, key, path, value):
        """INS (repo_ujson.pony:90-99)"""
        self.b.write([("INS", key, self.leaves.handle(path, canonical_value(value)))], self.identity)

    def rm(self, key, path, value):
        """RM (repo_ujson.pony:101-110): no key creation"""
        self.b.write([("RM", key, self.leaves.handle(path, canonical_value(value)))], self.identity)

    def clr(self, key, path=()):
        """CLR (repo_ujson.pony:85-88): no key creation; path-scoped"""
        if not self.b.exists(key):
            return
        if not path:
            self.b.write([("CLR", key)], self.identity)
            return
        hs = sorted(self._under(key, path))
        # nothing under the path still creates the key's delta (_delta_for)
        self.b.write([("RM", key, h) for h in hs] or [("TOUCH", key)], self.identity)

    def set(self, key, path, text):
        """SET (repo_ujson.pony:74-83): clear the path, then insert the node's leaves"""
        leaves = flatten(text, path)
        cmds = []
        if self.b.exists(key):
            if not path:
                cmds.append(("CLR", key))
            else:
                cmds += [("RM", key, h) for h in sorted(self._under(key, path))]
        cmds += [("INS", key, self.leaves.handle(p, v)) for p, v in sorted(leaves)]
        # an empty node still creates the key and its delta (_data_for, _delta_for)
        self.b.write(cmds or [("TOUCH", key)], self.identity)


class GpuDocs:
    """backend adapter: the GPU RepoUJSON"""

    def __init__(self, repo):
        self.r = repo

    def write(self, cmds, identity):
        self.r.write(cmds, identity)

    def exists(self, key):
        from . import engine as E
        return int(self.r.slots_of([key])[0]) != E._lib.JY_NO_SLOT

    def elements(self, keys):
        from . import engine as E
        slots = self.r.slots_of(keys)
        live = [(k, int(s)) for k, s in zip(keys, slots) if int(s) != E._lib.JY_NO_SLOT]
        if not live:
            return {}
        eo, dots, elems, vv, co, cloud = self.r.eng.ujson_read(np.array([s for _, s in live], np.uint32))
        return {k: elems[int(eo[i]):int(eo[i + 1])].tolist() for i, (k, _) in enumerate(live)}
