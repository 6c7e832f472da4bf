"""
GPU-backed RepoGCOUNT / RepoPNCOUNT: drop-in replacements for
jylis/repo_gcount.pony and jylis/repo_pncount.pony behind RepoAny
(jylis/repo_manager.pony:5-10).  NOT COMPILE-CHECKED: unbuilt here (no ponyc); INTEGRATION.md.

* converge (repo_gcount.pony:50-51) queues the pair; the next entry point
  merges every queued pair in ONE node call (RepoManagerCore.converge_deltas
  at repo_manager.pony:92-93 calls converge once per pair of a decoded peer
  batch, then returns): jy_node_counter_converge takes the key strings and
  each key's cells, and the library routes every key to the GPU that owns it.
* INC / DEC go to the owner shard's jy_counter_write: the engine adds to this
  replica's own column with wrapping and records the post-write total as the
  key's pending delta -- GCounter.increment's assignment semantics, so an own
  entry that wraps is never max-merged back to its old value.
* deltas_size sums the shards; flush_deltas rebuilds pony-crdt deltas from
  every shard's pending totals.
* Reading a peer GCounter's per-replica entries uses `pairs()` (PNCounter:
  `pos_pairs()` / `neg_pairs()`), accessors a vendored pony-crdt fork adds if
  upstream keeps the map private (INTEGRATION.md "pony-crdt accessors").
"""
use "collections"
use "crdt"
use "resp"

class RepoGCOUNTGpu
  let _identity: U64
  let _node: (_Node | None)
  embed _in: Array[(String, Any box)] = _in.create()

  new create(identity': U64) =>
    _identity = identity'
    _node = try _Node(identity')? else None end

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
    _CounterPending(_node, JyGCOUNT())

  fun ref flush_deltas(): Array[(String, Any box)] box =>
    """repo_gcount.pony:18-23: every pending key with its post-write total"""
    _drain()
    _Lock(_node, JyNoFence())  // the shared node's engines (jy_node_lock_type)
    let r = _flush_deltas()
    _Unlock(_node)
    r

  fun ref _flush_deltas(): Array[(String, Any box)] box =>
    let out = Array[(String, Any box)]
    match _node
    | let n: _Node =>
      for e in n.shards.values() do
        try
          e.sync_names(JyGCOUNT())
          let f = _CounterFlush(e, JyGCOUNT())?
          for (i, s) in f.slots.pairs() do
            let d = GCounter(_identity)
            d.increment(f.vals(i)?)
            out.push((e.name(s), d))
          end
        end
      end
    end
    out

  fun ref converge(key: String, delta': Any box) =>
    """RepoAny.converge, once per pair (repo_manager.pony:92-93): queue it;
    a full queue is merged at once (bounded memory between heartbeats)"""
    _in.push((key, delta'))
    if _in.size() >= _DrainBound() then _drain() end

  fun ref _drain() =>
    if _in.size() == 0 then return end
    match _node
    | let n: _Node => try _CounterIn(n, JyGCOUNT(), _in)? end
    end
    _in.clear()

  fun ref apply(r: Respond, cmd: Iterator[String]): Bool? =>
    match cmd.next()?
    | "GET" => get(r, cmd.next()?)
    | "INC" => inc(r, cmd.next()?, cmd.next()?.u64()?)
    else error
    end

  fun ref get(resp: Respond, key: String): Bool =>
    """repo_gcount.pony:53-55: a missing key reads 0"""
    _drain()
    _Lock(_node, JyGCOUNT())  // the shared node's engines (jy_node_lock_type)
    let r = _get(resp, key)
    _Unlock(_node)
    r

  fun ref _get(resp: Respond, key: String): Bool =>
    match _node
    | let n: _Node =>
      try
        let e = n.owner(key)?
        var slot = e.lookup(JyGCOUNT(), key)
        var v: U64 = 0
        if slot != JyNoSlot() then @jy_gcount_get(e.ptr, 1, addressof slot, addressof v, JyHost()) end
        resp.u64(v)
        false
      else _Fail(resp)
      end
    else _Fail(resp)
    end

  fun ref inc(resp: Respond, key: String, value: U64): Bool =>
    """repo_gcount.pony:57-60, on the key's owner shard"""
    _drain()
    _Lock(_node, JyGCOUNT())  // the shared node's engines (jy_node_lock_type)
    let r = _inc(resp, key, value)
    _Unlock(_node)
    r

  fun ref _inc(resp: Respond, key: String, value: U64): Bool =>
    match _node
    | let n: _Node =>
      try
        let e = n.owner(key)?
        let slots = e.intern(JyGCOUNT(), [key])?
        var v = value
        n.check(@jy_counter_write(e.ptr, JyGCOUNT(), 0, n.col(), 1, slots.cpointer(), addressof v,
          JyHost()))?
        resp.ok()
        true
      else _Fail(resp)
      end
    else _Fail(resp)
    end

class RepoPNCOUNTGpu
  let _identity: U64
  let _node: (_Node | None)
  embed _in: Array[(String, Any box)] = _in.create()

  new create(identity': U64) =>
    _identity = identity'
    _node = try _Node(identity')? else None end

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
    _CounterPending(_node, JyPNCOUNT())

  fun ref flush_deltas(): Array[(String, Any box)] box =>
    """repo_pncount.pony:19-24"""
    _drain()
    _Lock(_node, JyNoFence())  // the shared node's engines (jy_node_lock_type)
    let r = _flush_deltas()
    _Unlock(_node)
    r

  fun ref _flush_deltas(): Array[(String, Any box)] box =>
    let out = Array[(String, Any box)]
    match _node
    | let n: _Node =>
      for e in n.shards.values() do
        try
          e.sync_names(JyPNCOUNT())
          let f = _CounterFlush(e, JyPNCOUNT())?
          for (i, s) in f.slots.pairs() do
            let d = PNCounter(_identity)
            let m = f.mask(i)?
            if (m and 1) != 0 then d.increment(f.vals(i)?) end
            if (m and 2) != 0 then d.decrement(f.vals(f.cap + i)?) end
            out.push((e.name(s), d))
          end
        end
      end
    end
    out

  fun ref converge(key: String, delta': Any box) =>
    """RepoAny.converge, once per pair (repo_manager.pony:92-93): queue it;
    a full queue is merged at once (bounded memory between heartbeats)"""
    _in.push((key, delta'))
    if _in.size() >= _DrainBound() then _drain() end

  fun ref _drain() =>
    if _in.size() == 0 then return end
    match _node
    | let n: _Node => try _CounterIn(n, JyPNCOUNT(), _in)? end
    end
    _in.clear()

  fun ref apply(r: Respond, cmd: Iterator[String]): Bool? =>
    match cmd.next()?
    | "GET" => get(r, cmd.next()?)
    | "INC" => write(r, cmd.next()?, cmd.next()?.i64()?, 0)
    | "DEC" => write(r, cmd.next()?, cmd.next()?.i64()?, 1)
    else error
    end

  fun ref get(resp: Respond, key: String): Bool =>
    """repo_pncount.pony:55-57: (sum P - sum N) as i64; a missing key reads 0"""
    _drain()
    _Lock(_node, JyPNCOUNT())  // the shared node's engines (jy_node_lock_type)
    let r = _get(resp, key)
    _Unlock(_node)
    r

  fun ref _get(resp: Respond, key: String): Bool =>
    match _node
    | let n: _Node =>
      try
        let e = n.owner(key)?
        var slot = e.lookup(JyPNCOUNT(), key)
        var v: I64 = 0
        if slot != JyNoSlot() then @jy_pncount_get(e.ptr, 1, addressof slot, addressof v, JyHost()) end
        resp.i64(v)
        false
      else _Fail(resp)
      end
    else _Fail(resp)
    end

  fun ref write(resp: Respond, key: String, value: I64, sign: I32): Bool =>
    """INC / DEC (repo_pncount.pony:59-67): the i64 argument bit-cast to u64"""
    _drain()
    _Lock(_node, JyPNCOUNT())  // the shared node's engines (jy_node_lock_type)
    let r = _write(resp, key, value, sign)
    _Unlock(_node)
    r

  fun ref _write(resp: Respond, key: String, value: I64, sign: I32): Bool =>
    match _node
    | let n: _Node =>
      try
        let e = n.owner(key)?
        let slots = e.intern(JyPNCOUNT(), [key])?
        var v = value.u64()
        n.check(@jy_counter_write(e.ptr, JyPNCOUNT(), sign, n.col(), 1, slots.cpointer(), addressof v,
          JyHost()))?
        resp.ok()
        true
      else _Fail(resp)
      end
    else _Fail(resp)
    end

primitive _CounterPending
  """deltas_size over every shard of the node"""
  fun apply(node: (_Node | None), ty: I32): USize =>
    var total: USize = 0
    match node
    | let n: _Node =>
      for e in n.shards.values() do
        var k: U64 = 0
        @jy_counter_deltas_size(e.ptr, ty, addressof k)
        total = total + k.usize()
      end
    end
    total

class _CounterFlush
  """jy_counter_flush of one shard: pending slots, totals [sign][cap],
  written-sign masks"""
  let slots: Array[U32]
  let vals: Array[U64]
  let mask: Array[U32]
  let cap: USize

  new create(e: _Engine, ty: I32) ? =>
    var n: U64 = 0
    e.check(@jy_counter_deltas_size(e.ptr, ty, addressof n))?
    cap = n.usize().max(1)
    slots = Array[U32].init(0, cap)
    vals = Array[U64].init(0, 2 * cap)
    mask = Array[U32].init(0, cap)
    var got: U64 = 0
    e.check(@jy_counter_flush(e.ptr, ty, cap.u64(), slots.cpointer(), vals.cpointer(), mask.cpointer(),
      addressof got, JyHost()))?
    slots.truncate(got.usize())

primitive _CounterIn
  """a batch of peer counter deltas in ONE node call: the key strings and,
  per key, its cells (sign, replica column, value) -- jy_node_counter_converge
  routes each key to its owner GPU, interns it there and max-merges"""
  fun apply(n: _Node, ty: I32, pairs: Array[(String, Any box)] box) ? =>
    let keys = Array[String]
    let offs: Array[U64] = [0]
    let sg = Array[U8]
    let cc = Array[U16]
    let cv = Array[U64]
    for (k, d') in pairs.values() do
      // the reference's downcast (`delta' as GCounter box`); failures skip
      match d'
      | let d: GCounter box if ty == JyGCOUNT() =>
        keys.push(k)
        for (id, v) in d.pairs() do cc.push(n.replica_col(id)?); cv.push(v) end
        offs.push(cv.size().u64())
      | let d: PNCounter box if ty == JyPNCOUNT() =>
        keys.push(k)
        for (id, v) in d.pos_pairs() do sg.push(0); cc.push(n.replica_col(id)?); cv.push(v) end
        for (id, v) in d.neg_pairs() do sg.push(1); cc.push(n.replica_col(id)?); cv.push(v) end
        offs.push(cv.size().u64())
      end
    end
    if keys.size() == 0 then return end
    let m = _Strs(keys)
    let sp = if ty == JyGCOUNT() then Pointer[U8] else sg.cpointer() end
    n.check(@jy_node_counter_converge(n.ptr, ty, keys.size().u64(), m.bytes.cpointer(), m.offs.cpointer(),
      offs.cpointer(), sp, cc.cpointer(), cv.cpointer(), JyHost()))?
