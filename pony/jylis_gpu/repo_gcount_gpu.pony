"""
GPU-backed RepoGCOUNT / RepoTREG: drop-in replacements for
jylis/repo_gcount.pony and jylis/repo_treg.pony behind RepoAny
(jylis/repo_manager.pony:5-10), plus the one added batch method that
RepoManagerCore.converge_deltas (repo_manager.pony:92-93) calls.

UNBUILT here (no ponyc).  The write path (INC/SET -> `_deltas`, flush_deltas)
is unchanged host code; only converge and GET move to the engine.  Reading a
stock pony-crdt delta's per-replica entries needs an accessor that the
upstream GCounter may keep private -- `pairs()` below stands for it (a
vendored pony-crdt fork adds it if upstream lacks one).
"""
use "collections"
use "crdt"
use "resp"

class RepoGCOUNTGpu
  let _identity: U64
  let _eng: _Engine
  let _data: Map[String, GCounter] = _data.create()   // local writes only
  let _deltas: Map[String, GCounter] = _deltas.create()

  new create(identity': U64) ? =>
    (_identity, _eng) = (identity', _Engine(0)?)

  fun ref deltas_size(): USize => _deltas.size()
  fun ref flush_deltas(): Array[(String, Any box)] box =>
    let out = Array[(String, Any box)](_deltas.size())
    for (k, d) in _deltas.pairs() do out.push((k, d)) end
    _deltas.clear()
    out

  fun ref converge(key: String, delta': Any box) =>
    """single pair (repo_gcount.pony:50-51): a batch of one"""
    converge_batch(recover val [as (String, Any box): (key, delta')] end)

  fun ref converge_batch(deltas: Array[(String, Any box)] val) =>
    """the whole decoded MsgPushDeltas payload in ONE engine call"""
    let keys = _Keys(deltas)
    let slots = Array[U32].init(0, deltas.size())
    try _eng.check(@jy_keys_intern(_eng.ptr, JyGCOUNT(), deltas.size().u64(),
      keys.bytes.cpointer(), keys.offs.cpointer(), slots.cpointer()))? end
    let cell_slot = Array[U32]
    let cell_col = Array[U16]
    let cell_val = Array[U64]
    for (i, (k, d')) in deltas.pairs() do
      try
        let d = d' as GCounter box     // the reference's downcast; failures skip
        for (id, v) in d.pairs() do
          var col: U32 = 0
          _eng.check(@jy_replica_col(_eng.ptr, id, addressof col))?
          cell_slot.push(slots(i)?)
          cell_col.push(col.u16())
          cell_val.push(v)
        end
      end
    end
    try _eng.check(@jy_gcount_converge(_eng.ptr, cell_slot.size().u64(),
      cell_slot.cpointer(), cell_col.cpointer(), cell_val.cpointer(), JyHost()))? end

  fun ref apply(r: Respond, cmd: Iterator[String]): Bool? =>
    match cmd.next()?
    | "GET" => get(r, cmd.next()?)
    | "INC" => inc(r, cmd.next()?, cmd.next()?.u64()?)
    else error
    end

  fun get(resp: Respond, key: String): Bool =>
    """GCOUNT GET (repo_gcount.pony:53-55): missing key -> 0"""
    let kb = key.array()
    let ko: Array[U64] = [0; kb.size().u64()]
    var slot: U32 = 0
    var v: U64 = 0
    if (@jy_keys_lookup(_eng.ptr, JyGCOUNT(), 1, kb.cpointer(), ko.cpointer(), addressof slot) == 0)
      and (slot != U32.max_value()) then
      @jy_gcount_get(_eng.ptr, 1, addressof slot, addressof v, JyHost())
    end
    resp.u64(v)
    false

  fun ref inc(resp: Respond, key: String, value: U64): Bool =>
    """write path unchanged: local counter + delta; the local delta is also
    converged into the engine so GET sees it"""
    let d = try _deltas(key)? else let d' = GCounter(0); _deltas(key) = d'; d' end
    let data = try _data(key)? else let d' = GCounter(_identity); _data(key) = d'; d' end
    data.increment(value, d)
    converge(key, d)
    resp.ok()
    true
