"""
The engine handle and the marshalling every GPU repo shares (package jylis).
NOT COMPILE-CHECKED: unbuilt here (no ponyc); see INTEGRATION.md.

A GPU repo holds `(_Node | None)`: `RepoAny.create` (repo_manager.pony:6)
is not partial, so a missing GPU is reported per call (`_Fail`), not at
construction.  Every repo's `_Node` wraps the process's one library node
(jy_node_acquire_local / jy_node_release).
"""
use "collections"
use "resp"

class _Node
  """Every GPU of this Jylis process behind one handle (jy_node_*).  ONE node
  per process, shared by the five GPU repos (database.pony:18-22 makes one
  RepoManager actor per type): jy_node_acquire_local hands every repo the
  same library node, so one RCCL communicator and one engine per GPU serve
  every CRDT type.  Keys are hash-sharded over the GPUs (jy_node_shard_of).
  A decoded peer batch goes out in ONE call (jy_node_*_converge) that only
  enqueues: the node's worker thread regroups, exchanges and merges, one job
  at a time in call order, so the five actors' calls never interleave on the
  communicator and no scheduler thread waits for the GPU.  Reads, local
  writes and flushes use the key's owner shard (`owner`, `shards`) between
  `lock(ty)` and `unlock`: jy_node_lock_type waits only for the jobs of the
  repo's own type queued before it (a TREG read never waits for queued UJSON
  converges), JyNoFence for none (deltas_size and flush read state no
  converge changes).  The value arenas are reclaimed by the node's worker
  after TREG / TLOG jobs (jy_node_arena_gc), so a drain only enqueues.
  Never call a jy_node_* entry point while holding the lock."""
  let ptr: Pointer[None] tag
  let shards: Array[_Engine] = shards.create()   // one view per GPU, index = shard
  let _col: U32                                   // this replica's column (the same on every shard)
  embed _cols: Map[U64, U16] = _cols.create()     // replica id -> column, cached per repo

  new create(identity: U64) ? =>
    let cfg = JyConfig
    @jy_config_default(cfg)
    var p = Pointer[None]
    if @jy_node_acquire_local(cfg, addressof p) != 0 then error end
    ptr = p
    var c: U32 = 0
    if @jy_node_replica_col(ptr, identity, addressof c) != 0 then error end
    _col = c
    @jy_node_arena_gc(ptr, 1)
    for s in Range[U32](0, @jy_node_nshards(ptr)) do shards.push(_Engine.view(@jy_node_engine(ptr, s), c)) end

  fun col(): U32 => _col

  fun check(rc: I32) ? => if rc != 0 then error end

  fun lock(ty: I32) => @jy_node_lock_type(ptr, ty)
  fun unlock() => @jy_node_unlock(ptr)

  fun owner(key: String): _Engine ? =>
    """the shard that owns `key` (jy_key_owner over the node's GPUs)"""
    shards(@jy_node_shard_of(ptr, key.cpointer(), key.size().u64()).usize())?

  fun ref replica_col(id: U64): U16 ? =>
    """a peer's column, registered on every shard in one order; cached here,
    so a drain's per-cell lookups stay on the scheduler thread (the library
    answers a known id without waiting for the worker as well)"""
    try return _cols(id)? end
    var c: U32 = 0
    check(@jy_node_replica_col(ptr, id, addressof c))?
    _cols(id) = c.u16()
    c.u16()

  fun _final() => @jy_node_release(ptr)

primitive _Lock
  """the shared node's engines, exclusively, after the jobs of type `ty`
  queued before (JyNoFence: none); a repo holds no node: no-op"""
  fun apply(node: (_Node box | None), ty: I32) => match node | let n: _Node box => n.lock(ty) end

primitive _Unlock
  fun apply(node: (_Node box | None)) => match node | let n: _Node box => n.unlock() end

class _Engine
  """One shard's engine (one GPU): a view the node owns.  Slot -> key names
  are kept per shard for flushes and GETs."""
  let ptr: Pointer[None] tag
  let _names: Array[String] = _names.create()    // slot -> key (slots are dense)
  let _col: U32                                   // this replica's column
  var _arena_live: Array[U64] = Array[U64].init(0, 5)  // bytes kept by the last collect, per type

  new view(p: Pointer[None] tag, col': U32) =>
    ptr = p
    _col = col'

  fun col(): U32 => _col

  fun check(rc: I32) ? => if rc != 0 then error end

  fun ref intern(ty: I32, keys: Array[String] box): Array[U32] ? =>
    """slots of `keys`, creating missing ones (Repo._data_for)"""
    sync_names(ty)  // keys a one-call converge interned on the device
    let m = _Strs(keys)
    let slots = Array[U32].init(0, keys.size())
    check(@jy_keys_intern(ptr, ty, keys.size().u64(), m.bytes.cpointer(), m.offs.cpointer(),
      slots.cpointer()))?
    for (i, s) in slots.pairs() do
      while _names.size() <= s.usize() do _names.push("") end
      _names(s.usize())? = keys(i)?
    end
    slots

  fun lookup(ty: I32, key: String): U32 =>
    """slot of `key`, or JyNoSlot (Repo._data(key)? failing)"""
    let m = _Strs([key])
    var s: U32 = JyNoSlot()
    @jy_keys_lookup(ptr, ty, 1, m.bytes.cpointer(), m.offs.cpointer(), addressof s)
    s

  fun name(slot: U32): String => try _names(slot.usize())? else "" end

  fun ref sync_names(ty: I32) =>
    """names of keys interned on the device (jy_counter_converge_keys) come
    back from the directory (jy_keys_export) before a flush needs them"""
    let n = @jy_keys_count(ptr, ty)
    let have = _names.size().u64()
    if n <= have then return end
    let offs = Array[U64].init(0, (n - have).usize() + 1)
    @jy_keys_export(ptr, ty, have, n - have, offs.cpointer(), Pointer[U8], 0)  // sizes first
    let total = try offs(offs.size() - 1)? else 0 end
    let bytes = Array[U8].init(0, total.usize())
    if @jy_keys_export(ptr, ty, have, n - have, offs.cpointer(), bytes.cpointer(), total) != 0 then return end
    var i: USize = 0
    while (i + 1) < offs.size() do
      try
        let a = offs(i)?.usize()
        let b = offs(i + 1)?.usize()
        let k = recover String(b - a) end
        for j in Range(a, b) do k.push(bytes(j)?) end
        _names.push(consume k)
      end
      i = i + 1
    end

  fun replica(col': U32): U64 =>
    var id: U64 = 0
    @jy_replica_id(ptr, col', addressof id)
    id


  fun ref pack(ty: I32, values: Array[String] box): (Array[U64], Array[U64]) ? =>
    """value strings -> (pre, lr) handles (long values into the arena)"""
    let m = _Strs(values)
    let pre = Array[U64].init(0, values.size())
    let lr = Array[U64].init(0, values.size())
    check(@jy_values_pack(ptr, ty, values.size().u64(), m.bytes.cpointer(), m.offs.cpointer(),
      pre.cpointer(), lr.cpointer()))?
    (pre, lr)

  fun unpack(ty: I32, pre: U64, lr: U64): String =>
    """(pre, lr) -> the value string: <= 8 bytes live in pre (big-endian),
    longer ones in the arena at lr >> 24"""
    let len = (lr and 0xFFFFFF).usize()
    let out = recover String(len) end
    if len <= 8 then
      var i: USize = 0
      while i < len do
        out.push(((pre >> (56 - (8 * i.u64()))) and 0xFF).u8())
        i = i + 1
      end
    else
      let buf = Array[U8].init(0, len)
      @jy_arena_read(ptr, ty, lr >> 24, len.u64(), buf.cpointer())
      for b in buf.values() do out.push(b) end
    end
    consume out

  fun ref maybe_collect(ty: I32) =>
    """Reclaim the TREG / TLOG value arena once dead bytes pass twice the
    live ones (the policy of jylis_amd/repo.py _ArenaGC).  Call only after a
    converge / SET / INS that consumed every handle it packed: collection
    rewrites live handles and invalidates packed-but-unmerged ones."""
    var n: U64 = 0
    var cap: U64 = 0
    if @jy_arena_usage(ptr, ty, addressof n, addressof cap) != 0 then return end
    let live = try _arena_live(ty.usize())? else 0 end
    if n > ((2 * live) + (1 << 20)) then
      var kept: U64 = 0
      if @jy_arena_collect(ptr, ty, addressof kept) == 0 then
        try _arena_live(ty.usize())? = kept end
      end
    end

class _Strs
  """strings marshalled as bytes + offsets (the C-ABI's key / value columns)"""
  let bytes: Array[U8] = bytes.create()
  let offs: Array[U64] = offs.create()

  new create(strs: Array[String] box) =>
    offs.push(0)
    for k in strs.values() do
      bytes.append(k)
      offs.push(bytes.size().u64())
    end

class _Vals
  """value strings marshalled as bytes + offsets, built as they come"""
  let bytes: Array[U8] = bytes.create()
  let offs: Array[U64] = [0]

  fun ref push(v: String box) =>
    bytes.append(v)
    offs.push(bytes.size().u64())

primitive _Fail
  fun apply(resp: Respond): Bool =>
    resp.err("GPU engine unavailable")
    false
