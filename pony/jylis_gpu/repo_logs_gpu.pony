"""
GPU-backed RepoTREG / RepoTLOG: drop-in replacements for jylis/repo_treg.pony
and jylis/repo_tlog.pony behind RepoAny (jylis/repo_manager.pony:5-10).
NOT COMPILE-CHECKED: unbuilt here (no ponyc); INTEGRATION.md.

converge queues the pair and the next entry point merges the whole queue in
ONE node call (jy_node_treg_converge / jy_node_tlog_converge: key strings,
timestamps and value strings as bytes + offsets; the library routes every
key to the GPU that owns it, where its value bytes land in that shard's
arena).  Writes and reads go to the key's owner shard (jy_treg_set / _read,
jy_tlog_write / _read); deltas_size and flush_deltas walk every shard, and
flush rebuilds the pony-crdt deltas from the pending registers / logs.
Values travel as (pre, lr) handles on a shard (jy_values_pack); reads turn
them back into Strings.
"""
use "collections"
use "crdt"
use "resp"

class RepoTREGGpu
  let _node: (_Node | None)
  embed _in: Array[(String, Any box)] = _in.create()

  new create(identity': U64) =>
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
    var total: USize = 0
    match _node
    | let n: _Node =>
      for e in n.shards.values() do
        var k: U64 = 0
        @jy_treg_deltas_size(e.ptr, addressof k)
        total = total + k.usize()
      end
    end
    total

  fun ref flush_deltas(): Array[(String, Any box)] box =>
    """repo_treg.pony:18-22: every pending key with its delta register"""
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
        e.sync_names(JyTREG())
        var n: U64 = 0
        e.check(@jy_treg_deltas_size(e.ptr, addressof n))?
        let cap = n.usize().max(1)
        let slots = Array[U32].init(0, cap)
        let ts = Array[U64].init(0, cap)
        let pre = Array[U64].init(0, cap)
        let lr = Array[U64].init(0, cap)
        var got: U64 = 0
        e.check(@jy_treg_flush(e.ptr, cap.u64(), slots.cpointer(), ts.cpointer(), pre.cpointer(),
          lr.cpointer(), addressof got, JyHost()))?
        for i in Range(0, got.usize()) do
          let d = TRegString
          d.update(e.unpack(JyTREG(), pre(i)?, lr(i)?), ts(i)?)
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
    if _in.size() == 0 then return end
    match _node
    | let n: _Node =>
      try
        let keys = Array[String]
        let vals = _Vals
        let ts = Array[U64]
        for (k, d') in _in.values() do
          match d'
          | let d: TRegString box => keys.push(k); vals.push(d.value()); ts.push(d.timestamp())
          end
        end
        if keys.size() > 0 then
          let m = _Strs(keys)
          n.check(@jy_node_treg_converge(n.ptr, keys.size().u64(), m.bytes.cpointer(), m.offs.cpointer(),
            ts.cpointer(), vals.bytes.cpointer(), vals.offs.cpointer(), JyHost()))?
        end
      end
    end
    _in.clear()

  fun ref apply(r: Respond, cmd: Iterator[String]): Bool? =>
    match cmd.next()?
    | "GET" => get(r, cmd.next()?)
    | "SET" => set(r, cmd.next()?, cmd.next()?, cmd.next()?.u64()?)
    else error
    end

  fun ref get(resp: Respond, key: String): Bool =>
    """repo_treg.pony:54-63: [value, timestamp], or null for a missing key"""
    _drain()
    _Lock(_node, JyTREG())  // the shared node's engines (jy_node_lock_type)
    let r = _get(resp, key)
    _Unlock(_node)
    r

  fun ref _get(resp: Respond, key: String): Bool =>
    match _node
    | let n: _Node =>
      let e = try n.owner(key)? else return _Fail(resp) end
      var slot = e.lookup(JyTREG(), key)
      if slot == JyNoSlot() then resp.null(); return false end
      var ts: U64 = 0
      var pre: U64 = 0
      var lr: U64 = 0
      @jy_treg_read(e.ptr, 1, addressof slot, addressof ts, addressof pre, addressof lr)
      resp.array_start(2)
      resp.string(e.unpack(JyTREG(), pre, lr))
      resp.u64(ts)
      false
    else _Fail(resp)
    end

  fun ref set(resp: Respond, key: String, value: String, timestamp: U64): Bool =>
    """repo_treg.pony:65-68"""
    _drain()
    _Lock(_node, JyTREG())  // the shared node's engines (jy_node_lock_type)
    let r = _set(resp, key, value, timestamp)
    _Unlock(_node)
    r

  fun ref _set(resp: Respond, key: String, value: String, timestamp: U64): Bool =>
    match _node
    | let n: _Node =>
      try
        let e = n.owner(key)?
        let slots = e.intern(JyTREG(), [key])?
        (let pre, let lr) = e.pack(JyTREG(), [value])?
        var ts = timestamp
        e.check(@jy_treg_set(e.ptr, 1, slots.cpointer(), addressof ts, pre.cpointer(), lr.cpointer(),
          JyHost()))?
        e.maybe_collect(JyTREG())
        resp.ok()
        true
      else _Fail(resp)
      end
    else _Fail(resp)
    end

primitive _TlogOp
  fun ins(): U8 => 0
  fun trimat(): U8 => 1
  fun trim(): U8 => 2
  fun clr(): U8 => 3

class RepoTLOGGpu
  let _node: (_Node | None)
  embed _in: Array[(String, Any box)] = _in.create()

  new create(identity': U64) =>
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
    var total: USize = 0
    match _node
    | let n: _Node =>
      for e in n.shards.values() do
        var k: U64 = 0
        @jy_tlog_deltas_size(e.ptr, addressof k)
        total = total + k.usize()
      end
    end
    total

  fun ref flush_deltas(): Array[(String, Any box)] box =>
    """repo_tlog.pony:21-25: every pending key with its delta log"""
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
        e.sync_names(JyTLOG())
        var nk: U64 = 0
        var ne: U64 = 0
        e.check(@jy_tlog_flush(e.ptr, 0, 0, Pointer[U32], Pointer[U64], Pointer[U64], Pointer[U64],
          Pointer[U64], Pointer[U64], addressof nk, addressof ne, JyHost()))?
        if nk == 0 then continue end
        let slots = Array[U32].init(0, nk.usize())
        let cut = Array[U64].init(0, nk.usize())
        let offs = Array[U64].init(0, nk.usize() + 1)
        let ts = Array[U64].init(0, ne.usize().max(1))
        let pre = Array[U64].init(0, ne.usize().max(1))
        let lr = Array[U64].init(0, ne.usize().max(1))
        e.check(@jy_tlog_flush(e.ptr, nk, ne, slots.cpointer(), cut.cpointer(), offs.cpointer(),
          ts.cpointer(), pre.cpointer(), lr.cpointer(), addressof nk, addressof ne, JyHost()))?
        for i in Range(0, nk.usize()) do
          let d = TLog[String]
          d.raise_cutoff(cut(i)?)
          for j in Range(offs(i)?.usize(), offs(i + 1)?.usize()) do
            d.write(e.unpack(JyTLOG(), pre(j)?, lr(j)?), ts(j)?)
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
    """every queued TLog delta in one node call (CSR of entries, values as
    bytes + offsets; jy_node_tlog_converge routes each log to its owner)"""
    if _in.size() == 0 then return end
    match _node
    | let n: _Node =>
      try
        let keys = Array[String]
        let cut = Array[U64]
        let offs: Array[U64] = [0]
        let vals = _Vals
        let ts = Array[U64]
        for (k, d') in _in.values() do
          match d'
          | let d: TLog[String] box =>
            keys.push(k)
            cut.push(d.cutoff())
            for (v, t) in d.entries() do vals.push(v); ts.push(t) end   // newest first
            offs.push(ts.size().u64())
          end
        end
        if keys.size() > 0 then
          let m = _Strs(keys)
          n.check(@jy_node_tlog_converge(n.ptr, keys.size().u64(), m.bytes.cpointer(), m.offs.cpointer(),
            cut.cpointer(), offs.cpointer(), ts.cpointer(), vals.bytes.cpointer(), vals.offs.cpointer(),
            JyHost()))?
        end
      end
    end
    _in.clear()

  fun ref apply(r: Respond, cmd: Iterator[String]): Bool? =>
    match cmd.next()?
    | "GET"    => get(r, cmd.next()?, try cmd.next()?.usize()? else USize.max_value() end)
    | "INS"    =>
      let k = cmd.next()?
      let v = cmd.next()?
      write(r, k, _TlogOp.ins(), v, cmd.next()?.u64()?, 0)?
    | "SIZE"   => size(r, cmd.next()?, false)
    | "CUTOFF" => size(r, cmd.next()?, true)
    | "TRIMAT" => write(r, cmd.next()?, _TlogOp.trimat(), "", cmd.next()?.u64()?, 0)?
    | "TRIM"   => write(r, cmd.next()?, _TlogOp.trim(), "", 0, cmd.next()?.u64()?)?
    | "CLR"    => write(r, cmd.next()?, _TlogOp.clr(), "", 0, 0)?
    else error
    end

  fun ref write(resp: Respond, key: String, op: U8, value: String, ts': U64, count: U64): Bool ? =>
    """INS key value ts / TRIMAT key ts / TRIM key count / CLR key
    (repo_tlog.pony:85-111): one jy_tlog_write command"""
    _drain()
    _Lock(_node, JyTLOG())  // the shared node's engines (jy_node_lock_type)
    let r = try _write(resp, key, op, value, ts', count)? else _Unlock(_node); error end
    _Unlock(_node)
    r

  fun ref _write(resp: Respond, key: String, op: U8, value: String, ts': U64, count: U64): Bool ? =>
    var ts = ts'
    match _node
    | let n: _Node =>
      let e = n.owner(key)?
      let slots = e.intern(JyTLOG(), [key])?
      (let pre, let lr) = e.pack(JyTLOG(), [value])?
      var o = op
      var c = count
      e.check(@jy_tlog_write(e.ptr, 1, addressof o, slots.cpointer(), addressof ts, addressof c,
        pre.cpointer(), lr.cpointer(), JyHost()))?
      e.maybe_collect(JyTLOG())
      resp.ok()
      true
    else _Fail(resp)
    end

  fun ref get(resp: Respond, key: String, count: USize): Bool =>
    """repo_tlog.pony:69-83: at most `count` entries, newest first"""
    _drain()
    _Lock(_node, JyTLOG())  // the shared node's engines (jy_node_lock_type)
    let r = _get(resp, key, count)
    _Unlock(_node)
    r

  fun ref _get(resp: Respond, key: String, count: USize): Bool =>
    match _node
    | let n: _Node =>
      let e = try n.owner(key)? else return _Fail(resp) end
      var slot = e.lookup(JyTLOG(), key)
      if slot == JyNoSlot() then resp.array_start(0); return false end
      var len: U64 = 0
      var cut: U64 = 0
      @jy_tlog_read_sizes(e.ptr, 1, addressof slot, addressof len, addressof cut)
      let offs = Array[U64].init(0, 2)   // the one slot's CSR: [0, len]
      try offs(1)? = len end
      let ts = Array[U64].init(0, len.usize().max(1))
      let pre = Array[U64].init(0, len.usize().max(1))
      let lr = Array[U64].init(0, len.usize().max(1))
      @jy_tlog_read(e.ptr, 1, addressof slot, offs.cpointer(), ts.cpointer(), pre.cpointer(), lr.cpointer())
      let total = len.usize().min(count)
      resp.array_start(total)
      for i in Range(0, total) do
        resp.array_start(2)
        resp.string(try e.unpack(JyTLOG(), pre(i)?, lr(i)?) else "" end)
        resp.u64(try ts(i)? else 0 end)
      end
      false
    else _Fail(resp)
    end

  fun ref size(resp: Respond, key: String, cutoff: Bool): Bool =>
    """SIZE / CUTOFF (repo_tlog.pony:90-96): 0 for a missing key"""
    _drain()
    _Lock(_node, JyTLOG())  // the shared node's engines (jy_node_lock_type)
    let r = _size(resp, key, cutoff)
    _Unlock(_node)
    r

  fun ref _size(resp: Respond, key: String, cutoff: Bool): Bool =>
    match _node
    | let n: _Node =>
      let e = try n.owner(key)? else return _Fail(resp) end
      var slot = e.lookup(JyTLOG(), key)
      var len: U64 = 0
      var cut: U64 = 0
      if slot != JyNoSlot() then
        @jy_tlog_read_sizes(e.ptr, 1, addressof slot, addressof len, addressof cut)
      end
      resp.u64(if cutoff then cut else len end)
      false
    else _Fail(resp)
    end
