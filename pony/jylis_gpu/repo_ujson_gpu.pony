"""
GPU-backed RepoUJSON: drop-in replacement for jylis/repo_ujson.pony behind
RepoAny (jylis/repo_manager.pony:5-10).  NOT COMPILE-CHECKED: unbuilt here (no ponyc);
INTEGRATION.md.  The same layer in Python is jylis_amd/ujson_doc.py (tested).

The engine keeps each document's observed-remove dot kernel over opaque u64
element handles; this class owns the (path, value) leaves: a handle is the
FNV-1a 64 hash of the leaf's encoding (identical on every replica and in the
Python mirror), and `_leaves` maps handles back for GET.

* converge queues the pair; the next entry point converges the queue in ONE
  node call, jy_node_ujson_converge (dots, elements, vv, cloud per doc): the
  library routes every document to the GPU that owns it.  Reads and writes
  go to the key's owner shard; deltas_size and flush walk every shard.  Reading a peer UJSON
  delta's dots and context, and rebuilding one on flush, use accessors a
  vendored pony-crdt fork adds (`dots()`, `vv_pairs()`, `cloud()`,
  `from_dot()`, `from_vv()`, `from_cloud()`): upstream keeps the dot kernel
  private.
* GET renders the leaves at or under the path (maps, unordered sets, one
  merged map per set, nothing for empty collections: ujson.md:134-170).
* INS / RM / CLR / SET become jy_ujson_write commands (INS of a handle, RM of
  every element equal to a handle, CLR of a whole doc); path-scoped CLR and
  SET remove the handles under the path.  RM and CLR of a missing key do
  nothing (repo_ujson.pony:86,108); SET of an empty node still creates the
  key and its delta (an RM of handle 0, which no element holds).
"""
use "collections"
use "crdt"
use "json"
use "resp"

primitive _UjOp
  fun ins(): U8 => 0
  fun rm(): U8 => 1
  fun clr(): U8 => 2

primitive _LeafHash
  fun apply(path: Array[String] box, value: String): U64 =>
    var h: U64 = 0xCBF29CE484222325
    for p in path.values() do
      var n = p.size().u32()
      for i in Range(0, 4) do
        h = (h xor (n and 0xFF).u64()) * 0x100000001B3
        n = n >> 8
      end
      for b in p.values() do h = (h xor b.u64()) * 0x100000001B3 end
    end
    for i in Range(0, 4) do h = (h xor 0xFF) * 0x100000001B3 end
    for b in value.values() do h = (h xor b.u64()) * 0x100000001B3 end
    if h == 0 then 1 else h end

class RepoUJSONGpu
  let _identity: U64
  let _node: (_Node | None)
  embed _in: Array[(String, Any box)] = _in.create()
  embed _leaves: Map[U64, (Array[String] val, String)] = _leaves.create()

  new create(identity': U64) =>
    _identity = identity'
    _node = try _Node(identity')? else None end

  fun ref _handle(path: Array[String] val, value: String): U64 ? =>
    let h = _LeafHash(path, value)
    (let p, let v) = _leaves.insert_if_absent(h, (path, value))?
    if (v != value) or (p.size() != path.size()) or (not _Prefix(p, path)) then error end  // a collision
    h

  fun ref deltas_size(): USize =>
    """the heartbeat's call (repo_manager.pony:86-90): applies every queued
    peer pair first, so a replica with no local commands still converges
    each tick"""
    _drain()
    _Lock(_node, JyNoFence())  // the shared node's engines (jy_node_lock_type)
    let r = _deltas_size()
    _Unlock(_node)
    r

  fun ref _deltas_size(): USize =>
    var total: USize = 0
    match _node
    | let n: _Node =>
      for e in n.shards.values() do
        var k: U64 = 0
        @jy_ujson_deltas_size(e.ptr, addressof k)
        total = total + k.usize()
      end
    end
    total

  fun ref flush_deltas(): Array[(String, Any box)] box =>
    """repo_ujson.pony:22-26: every pending doc with its delta document"""
    _drain()
    _Lock(_node, JyNoFence())  // the shared node's engines (jy_node_lock_type)
    let r = _flush_deltas()
    _Unlock(_node)
    r

  fun ref _flush_deltas(): Array[(String, Any box)] box =>
    let out = Array[(String, Any box)]
    match _node
    | let node: _Node =>
      for e in node.shards.values() do try
        e.sync_names(JyUJSON())
        var nd: U64 = 0
        var ne: U64 = 0
        var nc: U64 = 0
        e.check(@jy_ujson_flush(e.ptr, 0, 0, 0, Pointer[U32], Pointer[U64], Pointer[U64], Pointer[U64],
          Pointer[U64], Pointer[U64], Pointer[U64], addressof nd, addressof ne, addressof nc, JyHost()))?
        if nd == 0 then continue end
        let r: USize = 16   // jy_config.ujson_columns
        let slots = Array[U32].init(0, nd.usize())
        let eo = Array[U64].init(0, nd.usize() + 1)
        let co = Array[U64].init(0, nd.usize() + 1)
        let dots = Array[U64].init(0, ne.usize().max(1))
        let elems = Array[U64].init(0, ne.usize().max(1))
        let cloud = Array[U64].init(0, nc.usize().max(1))
        let vv = Array[U64].init(0, nd.usize() * r)
        e.check(@jy_ujson_flush(e.ptr, nd, ne, nc, slots.cpointer(), eo.cpointer(), dots.cpointer(),
          elems.cpointer(), vv.cpointer(), co.cpointer(), cloud.cpointer(), addressof nd, addressof ne,
          addressof nc, JyHost()))?
        for i in Range(0, nd.usize()) do
          let d = UJSON(0)
          for j in Range(eo(i)?.usize(), eo(i + 1)?.usize()) do
            (let p, let v) = _leaves(elems(j)?)?
            d.from_dot(e.replica((dots(j)? >> JyDotSeqBits()).u32()), dots(j)? and 0xFFFFFFFFFFFF, p, v)
          end
          for c in Range(0, r) do
            let n = vv((i * r) + c)?
            if n != 0 then d.from_vv(e.replica(c.u32()), n) end
          end
          for j in Range(co(i)?.usize(), co(i + 1)?.usize()) do
            d.from_cloud(e.replica((cloud(j)? >> JyDotSeqBits()).u32()), cloud(j)? and 0xFFFFFFFFFFFF)
          end
          out.push((e.name(slots(i)?), d))
        end
      end end
    end
    out

  fun ref converge(key: String, delta': Any box) =>
    """RepoAny.converge, once per pair (repo_manager.pony:92-93): queue it;
    a full queue is merged at once (bounded memory between heartbeats)"""
    _in.push((key, delta'))
    if _in.size() >= _DrainBound() then _drain() end

  fun ref _drain() =>
    """every queued UJSON delta in one node call (jy_node_ujson_converge)"""
    if _in.size() == 0 then return end
    match _node
    | let e: _Node =>
      try
        let keys = Array[String]
        let eo: Array[U64] = [0]
        let vo: Array[U64] = [0]
        let co: Array[U64] = [0]
        let dots = Array[U64]
        let elems = Array[U64]
        let vv = Array[U64]
        let cloud = Array[U64]
        for (k, d') in _in.values() do
          match d'
          | let d: UJSON box =>
            keys.push(k)
            // sorted per doc by packed dot (column, seq): the engine's segment
            // order; a doc's dots are unique, so sort the dots and map back
            let ds = Array[U64]
            let hs = Map[U64, U64]
            for (id, seq, path, value) in d.dots() do
              let dot = (e.replica_col(id)?.u64() << JyDotSeqBits()) or seq
              ds.push(dot)
              hs(dot) = _handle(path, value)?
            end
            for dot in Sort[Array[U64], U64](ds).values() do
              dots.push(dot); elems.push(hs(dot)?)
            end
            eo.push(dots.size().u64())
            let vs = Array[U64]
            for (id, n) in d.vv_pairs() do vs.push((e.replica_col(id)?.u64() << JyDotSeqBits()) or n) end
            for x in Sort[Array[U64], U64](vs).values() do vv.push(x) end
            vo.push(vv.size().u64())
            let cs = Array[U64]
            for (id, seq) in d.cloud() do cs.push((e.replica_col(id)?.u64() << JyDotSeqBits()) or seq) end
            for x in Sort[Array[U64], U64](cs).values() do cloud.push(x) end
            co.push(cloud.size().u64())
          end
        end
        if keys.size() > 0 then
          let m = _Strs(keys)
          e.check(@jy_node_ujson_converge(e.ptr, keys.size().u64(), m.bytes.cpointer(), m.offs.cpointer(),
            eo.cpointer(), dots.cpointer(), elems.cpointer(), vo.cpointer(), vv.cpointer(), co.cpointer(),
            cloud.cpointer(), JyHost()))?
        end
      end
    end
    _in.clear()

  fun ref apply(r: Respond, cmd: Iterator[String]): Bool? =>
    let word = cmd.next()?
    let key = cmd.next()?
    let rest = Array[String]
    for s in cmd do rest.push(s) end
    match word
    | "GET" => get(r, key, _path(rest))
    | "CLR" => clr(r, key, _path(rest))
    | "SET" => let v = rest.pop()?; set(r, key, _path(rest), v)?
    | "INS" => let v = rest.pop()?; ins_rm(r, key, _path(rest), v, _UjOp.ins())?
    | "RM"  => let v = rest.pop()?; ins_rm(r, key, _path(rest), v, _UjOp.rm())?
    else error
    end

  fun _path(rest: Array[String] box): Array[String] val =>
    let p = recover Array[String] end
    for s in rest.values() do p.push(s) end
    consume p

  fun ref _elements(e: _Engine, key: String): Array[U64] =>
    """the doc's element handles (empty for a missing key)"""
    var slot = e.lookup(JyUJSON(), key)
    if slot == JyNoSlot() then return Array[U64] end
    var ne: U64 = 0
    var nc: U64 = 0
    @jy_ujson_read_sizes(e.ptr, 1, addressof slot, addressof ne, addressof nc)
    let eo = Array[U64].init(0, 2)   // the one doc's CSRs: [0, ne], [0, nc]
    let co = Array[U64].init(0, 2)
    try eo(1)? = ne; co(1)? = nc end
    let dots = Array[U64].init(0, ne.usize().max(1))
    let elems = Array[U64].init(0, ne.usize().max(1))
    let vv = Array[U64].init(0, 16)
    let cloud = Array[U64].init(0, nc.usize().max(1))
    @jy_ujson_read(e.ptr, 1, addressof slot, eo.cpointer(), dots.cpointer(), elems.cpointer(), vv.cpointer(),
      co.cpointer(), cloud.cpointer())
    elems.truncate(ne.usize())
    elems

  fun ref _under(e: _Engine, key: String, path: Array[String] box): Array[U64] =>
    let out = Array[U64]
    let seen = Set[U64]
    for h in _elements(e, key).values() do
      if seen.contains(h) then continue end
      seen.set(h)
      try
        (let p, _) = _leaves(h)?
        if _Prefix(path, p) then out.push(h) end
      end
    end
    out

  fun ref _write(e: _Engine, key: String, ops: Array[U8], elems: Array[U64]) ? =>
    let keys = Array[String].init(key, ops.size())
    let slots = e.intern(JyUJSON(), keys)?
    e.check(@jy_ujson_write(e.ptr, ops.size().u64(), ops.cpointer(), slots.cpointer(), elems.cpointer(),
      e.col(), JyHost()))?   // the key's owner shard

  fun ref get(resp: Respond, key: String, path: Array[String] val): Bool =>
    """repo_ujson.pony:68-72: the render, or '' for nothing"""
    _drain()
    _Lock(_node, JyUJSON())  // the shared node's engines (jy_node_lock_type)
    let r = _get(resp, key, path)
    _Unlock(_node)
    r

  fun ref _get(resp: Respond, key: String, path: Array[String] val): Bool =>
    match _node
    | let n: _Node =>
      let e = try n.owner(key)? else return _Fail(resp) end
      let leaves = Array[(Array[String] val, String)]
      for h in _under(e, key, path).values() do
        try
          (let p, let v) = _leaves(h)?
          leaves.push((recover val p.slice(path.size()) end, v))
        end
      end
      resp.string(_Render(leaves))
      false
    else _Fail(resp)
    end

  fun ref ins_rm(resp: Respond, key: String, path: Array[String] val, text: String, op: U8): Bool ? =>
    """INS / RM (repo_ujson.pony:90-110): the value parses as a UJSON primitive"""
    _drain()
    _Lock(_node, JyUJSON())  // the shared node's engines (jy_node_lock_type)
    let r = try _ins_rm(resp, key, path, text, op)? else _Unlock(_node); error end
    _Unlock(_node)
    r

  fun ref _ins_rm(resp: Respond, key: String, path: Array[String] val, text: String, op: U8): Bool ? =>
    match _node
    | let n: _Node =>
      let e = try n.owner(key)? else return _Fail(resp) end
      if (op == _UjOp.rm()) and (e.lookup(JyUJSON(), key) == JyNoSlot()) then resp.ok(); return true end
      let h = _handle(path, _Canon.value(text)?)?
      _write(e, key, [op], [h])?
      resp.ok()
      true
    else _Fail(resp)
    end

  fun ref clr(resp: Respond, key: String, path: Array[String] val): Bool =>
    """CLR (repo_ujson.pony:85-88): no key creation"""
    _drain()
    _Lock(_node, JyUJSON())  // the shared node's engines (jy_node_lock_type)
    let r = _clr(resp, key, path)
    _Unlock(_node)
    r

  fun ref _clr(resp: Respond, key: String, path: Array[String] val): Bool =>
    match _node
    | let n: _Node =>
      let e = try n.owner(key)? else return _Fail(resp) end
      if e.lookup(JyUJSON(), key) != JyNoSlot() then
        try
          if path.size() == 0 then
            _write(e, key, [_UjOp.clr()], [0])?
          else
            let hs = _under(e, key, path)
            if hs.size() == 0 then hs.push(0) end      // still creates the key's delta
            _write(e, key, Array[U8].init(_UjOp.rm(), hs.size()), hs)?
          end
        end
      end
      resp.ok()
      true
    else _Fail(resp)
    end

  fun ref set(resp: Respond, key: String, path: Array[String] val, text: String): Bool ? =>
    """SET (repo_ujson.pony:74-83): clear the path, insert the node's leaves"""
    _drain()
    _Lock(_node, JyUJSON())  // the shared node's engines (jy_node_lock_type)
    let r = try _set(resp, key, path, text)? else _Unlock(_node); error end
    _Unlock(_node)
    r

  fun ref _set(resp: Respond, key: String, path: Array[String] val, text: String): Bool ? =>
    match _node
    | let n: _Node =>
      let e = try n.owner(key)? else return _Fail(resp) end
      let ops = Array[U8]
      let hs = Array[U64]
      if e.lookup(JyUJSON(), key) != JyNoSlot() then
        if path.size() == 0 then
          ops.push(_UjOp.clr()); hs.push(0)
        else
          for h in _under(e, key, path).values() do ops.push(_UjOp.rm()); hs.push(h) end
        end
      end
      for (p, v) in _Canon.flatten(text, path)?.values() do
        ops.push(_UjOp.ins()); hs.push(_handle(p, v)?)
      end
      if ops.size() == 0 then ops.push(_UjOp.rm()); hs.push(0) end   // an empty node: key + delta
      _write(e, key, ops, hs)?
      resp.ok()
      true
    else _Fail(resp)
    end

primitive _Quote
  """a JSON string literal"""
  fun apply(s: String box): String =>
    let out = String(s.size() + 2)
    out.push('"')
    for b in s.values() do
      match b
      | '"' => out.append("\\\"")
      | '\\' => out.append("\\\\")
      | '\n' => out.append("\\n")
      | '\r' => out.append("\\r")
      | '\t' => out.append("\\t")
      else
        if b < 0x20 then
          out.append("\\u00")
          out.push("0123456789abcdef".at_offset((b >> 4).isize()) as U8)
          out.push("0123456789abcdef".at_offset((b and 0xF).isize()) as U8)
        else
          out.push(b)
        end
      end
    end
    out.push('"')
    out.clone()

primitive _Prefix
  fun apply(prefix: Array[String] box, path: Array[String] box): Bool =>
    if prefix.size() > path.size() then return false end
    for (i, s) in prefix.pairs() do
      try if path(i)? != s then return false end else return false end
    end
    true

primitive _Canon
  """UJSONParse.value / .node: JSON text -> canonical primitive text / leaves"""
  fun value(text: String): String ? =>
    let doc = JsonDoc
    doc.parse(text)?
    _dump(doc.data)?

  fun _dump(v: JsonType box): String ? =>
    match v
    | let s: String box => _Quote(s)
    | let n: I64 => n.string()
    | let f: F64 => f.string()
    | let b: Bool => b.string()
    | None => "null"
    else error   // objects and arrays are not primitives
    end

  fun flatten(text: String, prefix: Array[String] val): Array[(Array[String] val, String)] ? =>
    let doc = JsonDoc
    doc.parse(text)?
    let out = Array[(Array[String] val, String)]
    _walk(doc.data, prefix, out)?
    out

  fun _walk(v: JsonType box, path: Array[String] val, out: Array[(Array[String] val, String)]) ? =>
    match v
    | let o: JsonObject box =>
      for (k, x) in o.data.pairs() do
        let p = recover val path.clone() .> push(k) end
        _walk(x, p, out)?
      end
    | let a: JsonArray box =>
      for x in a.data.values() do _walk(x, path, out)? end     // sets flatten
    else
      out.push((path, _dump(v)?))
    end

primitive _Render
  """leaves (relative path, canonical value) -> UJSON text ('' when empty)"""
  fun apply(leaves: Array[(Array[String] val, String)] box): String =>
    if leaves.size() == 0 then return "" end
    let root = _JsonNode
    for (p, v) in leaves.values() do
      var n = root
      for s in p.values() do n = n.child(s) end
      n.values.set(v)
    end
    root.render()

class _JsonNode
  embed values: Set[String] = values.create()
  embed map: Map[String, _JsonNode] = map.create()

  fun ref child(k: String): _JsonNode =>
    try map(k)? else let c = _JsonNode; map(k) = c; c end

  fun nonempty(): Bool =>
    if values.size() > 0 then return true end
    for c in map.values() do if c.nonempty() then return true end end
    false

  fun render(): String =>
    let items = Array[String]
    for v in values.values() do items.push(v) end
    let keys = Array[String]
    for (k, c) in map.pairs() do if c.nonempty() then keys.push(k) end end
    if keys.size() > 0 then
      let m = String
      m.append("{")
      for (i, k) in Sort[Array[String], String](keys).pairs() do
        if i > 0 then m.append(",") end
        m.append(_Quote(k))
        m.append(":")
        m.append(try map(k)?.render() else "" end)
      end
      m.append("}")
      items.push(m.clone())
    end
    if items.size() == 1 then return try items(0)? else "" end end
    let s = String
    s.append("[")
    for (i, x) in Sort[Array[String], String](items).pairs() do
      if i > 0 then s.append(",") end
      s.append(x)
    end
    s.append("]")
    s.clone()
