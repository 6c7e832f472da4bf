"""
GPU-backed RepoGCOUNT / RepoPNCOUNT: drop-in replacements for
jylis/repo_gcount.pony and jylis/repo_pncount.pony behind RepoAny
(jylis/repo_manager.pony:5-10).  NOT COMPILE-CHECKED: unbuilt here (no ponyc); INTEGRATION.md.

* converge (repo_gcount.pony:50-51) queues the pair; the next entry point
  merges every queued pair in ONE engine call (RepoManagerCore.converge_deltas
  at repo_manager.pony:92-93 calls converge once per pair of a decoded peer
  batch, then returns): COO cells for sparse batches, one dense column block
  (jy_*_converge_block) when the batch covers most cells of a slot run (a
  full-state sync).
* INC / DEC go to jy_counter_write: the engine adds to this replica's own
  column with wrapping and records the post-write total as the key's pending
  delta -- GCounter.increment's assignment semantics, so an own entry that
  wraps is never max-merged back to its old value.
* flush_deltas rebuilds pony-crdt deltas from the engine's pending totals.
* Reading a peer GCounter's per-replica entries uses `pairs()`, an accessor a
  vendored pony-crdt fork adds if upstream keeps the map private.
"""
use "collections"
use "crdt"
use "resp"

class RepoGCOUNTGpu
  let _identity: U64
  let _eng: (_Engine | None)
  embed _in: Array[(String, Any box)] = _in.create()

  new create(identity': U64) =>
    _identity = identity'
    _eng = try _Engine(identity')? else None end

  fun ref deltas_size(): USize =>
    """the heartbeat's call (repo_manager.pony:86-90): applies every queued
    peer pair first, so a replica with no local commands still converges
    each tick"""
    _drain()
    match _eng
    | let e: _Engine =>
      var n: U64 = 0
      @jy_counter_deltas_size(e.ptr, JyGCOUNT(), addressof n)
      n.usize()
    else 0
    end

  fun ref flush_deltas(): Array[(String, Any box)] box =>
    """repo_gcount.pony:18-23: every pending key with its post-write total"""
    _drain()
    let out = Array[(String, Any box)]
    match _eng
    | let e: _Engine =>
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
    out

  fun ref converge(key: String, delta': Any box) =>
    """RepoAny.converge, once per pair (repo_manager.pony:92-93): queue it;
    a full queue is merged at once (bounded memory between heartbeats)"""
    _in.push((key, delta'))
    if _in.size() >= _DrainBound() then _drain() end

  fun ref _drain() =>
    if _in.size() == 0 then return end
    match _eng
    | let e: _Engine => try _CounterIn(e, JyGCOUNT(), _in)? end
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
    match _eng
    | let e: _Engine =>
      var slot = e.lookup(JyGCOUNT(), key)
      var v: U64 = 0
      if slot != JyNoSlot() then @jy_gcount_get(e.ptr, 1, addressof slot, addressof v, JyHost()) end
      resp.u64(v)
      false
    else _Fail(resp)
    end

  fun ref inc(resp: Respond, key: String, value: U64): Bool =>
    """repo_gcount.pony:57-60"""
    _drain()
    match _eng
    | let e: _Engine =>
      try
        let slots = e.intern(JyGCOUNT(), [key])?
        var v = value
        e.check(@jy_counter_write(e.ptr, JyGCOUNT(), 0, e.col(), 1, slots.cpointer(), addressof v,
          JyHost()))?
        resp.ok()
        true
      else _Fail(resp)
      end
    else _Fail(resp)
    end

class RepoPNCOUNTGpu
  let _identity: U64
  let _eng: (_Engine | None)
  embed _in: Array[(String, Any box)] = _in.create()

  new create(identity': U64) =>
    _identity = identity'
    _eng = try _Engine(identity')? else None end

  fun ref deltas_size(): USize =>
    """the heartbeat's call (repo_manager.pony:86-90): applies every queued
    peer pair first, so a replica with no local commands still converges
    each tick"""
    _drain()
    match _eng
    | let e: _Engine =>
      var n: U64 = 0
      @jy_counter_deltas_size(e.ptr, JyPNCOUNT(), addressof n)
      n.usize()
    else 0
    end

  fun ref flush_deltas(): Array[(String, Any box)] box =>
    """repo_pncount.pony:19-24"""
    _drain()
    let out = Array[(String, Any box)]
    match _eng
    | let e: _Engine =>
      try
        e.sync_names(JyPNCOUNT())
        let f = _CounterFlush(e, JyPNCOUNT())?
        for (i, s) in f.slots.pairs() do
          let d = PNCounter(_identity)
          let m = f.mask(i)?
          if (m and 1) != 0 then d.increment(f.vals(i)?) end
          if (m and 2) != 0 then d.decrement(f.vals(f.slots.size() + i)?) end
          out.push((e.name(s), d))
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
    match _eng
    | let e: _Engine => try _CounterIn(e, JyPNCOUNT(), _in)? end
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
    match _eng
    | let e: _Engine =>
      var slot = e.lookup(JyPNCOUNT(), key)
      var v: I64 = 0
      if slot != JyNoSlot() then @jy_pncount_get(e.ptr, 1, addressof slot, addressof v, JyHost()) end
      resp.i64(v)
      false
    else _Fail(resp)
    end

  fun ref write(resp: Respond, key: String, value: I64, sign: I32): Bool =>
    """INC / DEC (repo_pncount.pony:59-67): the i64 argument bit-cast to u64"""
    _drain()
    match _eng
    | let e: _Engine =>
      try
        let slots = e.intern(JyPNCOUNT(), [key])?
        var v = value.u64()
        e.check(@jy_counter_write(e.ptr, JyPNCOUNT(), sign, e.col(), 1, slots.cpointer(), addressof v,
          JyHost()))?
        resp.ok()
        true
      else _Fail(resp)
      end
    else _Fail(resp)
    end

class _CounterFlush
  """jy_counter_flush: pending slots, totals [sign][cap], written-sign masks"""
  let slots: Array[U32]
  let vals: Array[U64]
  let mask: Array[U32]

  new create(e: _Engine, ty: I32) ? =>
    var n: U64 = 0
    e.check(@jy_counter_deltas_size(e.ptr, ty, addressof n))?
    let cap = n.usize().max(1)
    slots = Array[U32].init(0, cap)
    vals = Array[U64].init(0, 2 * cap)
    mask = Array[U32].init(0, cap)
    var got: U64 = 0
    e.check(@jy_counter_flush(e.ptr, ty, cap.u64(), slots.cpointer(), vals.cpointer(), mask.cpointer(),
      addressof got, JyHost()))?
    slots.truncate(got.usize())

primitive _CounterIn
  """one engine call for a batch of peer counter deltas"""
  fun apply(e: _Engine, ty: I32, pairs: Array[(String, Any box)] box) ? =>
    let keys = Array[String]
    let ds = Array[Any box]
    for (k, d') in pairs.values() do
      // the reference's downcast (`delta' as GCounter box`); failures skip
      match d'
      | let d: GCounter box if ty == JyGCOUNT() => keys.push(k); ds.push(d)
      | let d: PNCounter box if ty == JyPNCOUNT() => keys.push(k); ds.push(d)
      end
    end
    if keys.size() == 0 then return end
    // A sparse batch (the usual flushed peer delta: a few replica entries per
    // key) goes out in ONE call with its key strings: interned on the device,
    // merged with the device slots, no slot back to the host.  A batch that
    // carries about every replica of every key (a full-state sync) is
    // interned first, so its slot run can take the dense column-block path.
    var ncell: USize = 0
    for d' in ds.values() do
      match d'
      | let d: GCounter box => for _ in d.pairs() do ncell = ncell + 1 end
      | let d: PNCounter box =>
        for _ in d.pos_pairs() do ncell = ncell + 1 end
        for _ in d.neg_pairs() do ncell = ncell + 1 end
      end
    end
    let nrep = @jy_replica_count(e.ptr).usize().max(1)
    if (ncell * 2) < (keys.size() * nrep) then
      let m = _Strs(keys)
      let ck = Array[U32]
      let sg = Array[U8]
      let cc = Array[U16]
      let cv = Array[U64]
      for (i, d') in ds.pairs() do
        match d'
        | let d: GCounter box =>
          for (id, v) in d.pairs() do ck.push(i.u32()); cc.push(e.replica_col(id)?); cv.push(v) end
        | let d: PNCounter box =>
          for (id, v) in d.pos_pairs() do ck.push(i.u32()); sg.push(0); cc.push(e.replica_col(id)?); cv.push(v) end
          for (id, v) in d.neg_pairs() do ck.push(i.u32()); sg.push(1); cc.push(e.replica_col(id)?); cv.push(v) end
        end
      end
      let sp = if ty == JyGCOUNT() then Pointer[U8] else sg.cpointer() end
      e.check(@jy_counter_converge_keys(e.ptr, ty, keys.size().u64(), m.bytes.cpointer(), m.offs.cpointer(),
        ck.size().u64(), ck.cpointer(), sp, cc.cpointer(), cv.cpointer(), JyHost()))?
      return
    end
    let slots = e.intern(ty, keys)?
    // cells per sign: (slot, column, value)
    let cs = [Array[U32]; Array[U32]]
    let cc = [Array[U16]; Array[U16]]
    let cv = [Array[U64]; Array[U64]]
    for (i, d') in ds.pairs() do
      match d'
      | let d: GCounter box =>
        for (id, v) in d.pairs() do
          cs(0)?.push(slots(i)?); cc(0)?.push(e.replica_col(id)?); cv(0)?.push(v)
        end
      | let d: PNCounter box =>
        for (id, v) in d.pos_pairs() do
          cs(0)?.push(slots(i)?); cc(0)?.push(e.replica_col(id)?); cv(0)?.push(v)
        end
        for (id, v) in d.neg_pairs() do
          cs(1)?.push(slots(i)?); cc(1)?.push(e.replica_col(id)?); cv(1)?.push(v)
        end
      end
    end
    // dense enough for one column block over the slot run?
    var lo: U32 = U32.max_value()
    var hi: U32 = 0
    let colset = Set[U16]
    var ncells: USize = 0
    for sg in Range(0, 2) do
      for (j, s) in cs(sg)?.pairs() do
        lo = lo.min(s); hi = hi.max(s); colset.set(cc(sg)?(j)?)
      end
      ncells = ncells + cs(sg)?.size()
    end
    if ncells == 0 then return end
    let span = (hi - lo).usize() + 1
    let nsg: USize = if ty == JyGCOUNT() then 1 else 2 end
    if (span * colset.size() * nsg) <= (2 * ncells) then
      let cols = Array[U16]
      let ci = Map[U16, USize]
      for c in colset.values() do ci(c) = cols.size(); cols.push(c) end
      let blk = [Array[U64].init(0, cols.size() * span); Array[U64].init(0, cols.size() * span)]
      for sg in Range(0, nsg) do
        for (j, s) in cs(sg)?.pairs() do
          let at = (ci(cc(sg)?(j)?)? * span) + (s - lo).usize()
          blk(sg)?(at)? = blk(sg)?(at)?.max(cv(sg)?(j)?)   // zeros are neutral under max
        end
      end
      if ty == JyGCOUNT() then
        e.check(@jy_gcount_converge_block(e.ptr, cols.size().u32(), cols.cpointer(), lo, span.u32(),
          blk(0)?.cpointer(), JyHost()))?
      else
        e.check(@jy_pncount_converge_block(e.ptr, cols.size().u32(), cols.cpointer(), lo, span.u32(),
          blk(0)?.cpointer(), blk(1)?.cpointer(), JyHost()))?
      end
    elseif ty == JyGCOUNT() then
      e.check(@jy_gcount_converge(e.ptr, cs(0)?.size().u64(), cs(0)?.cpointer(), cc(0)?.cpointer(),
        cv(0)?.cpointer(), JyHost()))?
    else
      e.check(@jy_pncount_converge(e.ptr,
        cs(0)?.size().u64(), cs(0)?.cpointer(), cc(0)?.cpointer(), cv(0)?.cpointer(),
        cs(1)?.size().u64(), cs(1)?.cpointer(), cc(1)?.cpointer(), cv(1)?.cpointer(), JyHost()))?
    end
