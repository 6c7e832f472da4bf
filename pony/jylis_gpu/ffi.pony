"""
FFI declarations of the MI355X converge engine (include/jylis_gpu.h).

UNBUILT in this repository: the image has no ponyc and jemc/pony-crdt is not
vendored (DESIGN.md "Oracle").  Written against the reference's interfaces
(jylis/repo_manager.pony:5-10) for a maintainer to drop into package jylis.
Every @-call returns an I32 status (0 ok); pointers are borrowed for the call.
"""

use "lib:jylis_gpu"

use @jy_config_default[None](cfg: Pointer[JyConfig] tag)
use @jy_engine_create[I32](cfg: Pointer[JyConfig] tag, out: Pointer[Pointer[None] tag])
use @jy_engine_destroy[None](eng: Pointer[None] tag)
use @jy_last_error[Pointer[U8] val](eng: Pointer[None] tag)
use @jy_skipped[U64](eng: Pointer[None] tag)
use @jy_sync[I32](eng: Pointer[None] tag)

use @jy_replica_col[I32](eng: Pointer[None] tag, id: U64, col: Pointer[U32] tag)
use @jy_keys_intern[I32](eng: Pointer[None] tag, ty: I32, n: U64,
  key_bytes: Pointer[U8] tag, key_offs: Pointer[U64] tag, slots: Pointer[U32] tag)
use @jy_keys_lookup[I32](eng: Pointer[None] tag, ty: I32, n: U64,
  key_bytes: Pointer[U8] tag, key_offs: Pointer[U64] tag, slots: Pointer[U32] tag)
use @jy_values_pack[I32](eng: Pointer[None] tag, ty: I32, n: U64,
  bytes: Pointer[U8] tag, offs: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag)
use @jy_arena_read[I32](eng: Pointer[None] tag, ty: I32, off: U64, len: U64, dst: Pointer[U8] tag)

use @jy_gcount_converge[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  col: Pointer[U16] tag, value: Pointer[U64] tag, mem: I32)
use @jy_gcount_get[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  out: Pointer[U64] tag, mem: I32)
use @jy_pncount_converge[I32](eng: Pointer[None] tag,
  np: U64, pslot: Pointer[U32] tag, pcol: Pointer[U16] tag, pval: Pointer[U64] tag,
  nn: U64, nslot: Pointer[U32] tag, ncol: Pointer[U16] tag, nval: Pointer[U64] tag, mem: I32)
use @jy_pncount_get[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  out: Pointer[I64] tag, mem: I32)
use @jy_treg_converge[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag, mem: I32)
use @jy_treg_read[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag)
// local writes + flush_deltas (RepoGCOUNT.inc / RepoPNCOUNT.inc,dec /
// RepoTREG.set and flush_deltas, repo_gcount.pony:18-23,57-60)
use @jy_counter_write[I32](eng: Pointer[None] tag, ty: I32, sign: I32, col: U32, n: U64,
  slot: Pointer[U32] tag, value: Pointer[U64] tag, mem: I32)
use @jy_counter_deltas_size[I32](eng: Pointer[None] tag, ty: I32, n_out: Pointer[U64] tag)
use @jy_counter_flush[I32](eng: Pointer[None] tag, ty: I32, cap: U64, slot_out: Pointer[U32] tag,
  vals_out: Pointer[U64] tag, mask_out: Pointer[U32] tag, n_out: Pointer[U64] tag, mem: I32)
use @jy_treg_set[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag, mem: I32)
use @jy_treg_deltas_size[I32](eng: Pointer[None] tag, n_out: Pointer[U64] tag)
use @jy_treg_flush[I32](eng: Pointer[None] tag, cap: U64, slot_out: Pointer[U32] tag,
  ts_out: Pointer[U64] tag, pre_out: Pointer[U64] tag, lr_out: Pointer[U64] tag,
  n_out: Pointer[U64] tag, mem: I32)
use @jy_tlog_converge[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  cutoff: Pointer[U64] tag, ent_offs: Pointer[U64] tag, nent: U64,
  ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag, mem: I32)
use @jy_ujson_converge[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  el_offs: Pointer[U64] tag, nel: U64, dots: Pointer[U64] tag, elems: Pointer[U64] tag,
  vv_offs: Pointer[U64] tag, nvv: U64, vv: Pointer[U64] tag,
  cloud_offs: Pointer[U64] tag, ncloud: U64, cloud: Pointer[U64] tag, mem: I32)

primitive JyHost fun apply(): I32 => 0
primitive JyGCOUNT fun apply(): I32 => 0
primitive JyPNCOUNT fun apply(): I32 => 1
primitive JyTREG fun apply(): I32 => 2
primitive JyTLOG fun apply(): I32 => 3
primitive JyUJSON fun apply(): I32 => 4

struct JyConfig
  var device: I32 = 0
  var counter_columns: U32 = 16
  var ujson_columns: U32 = 16
  var reserved: U32 = 0
  embed key_capacity: _U64x5 = _U64x5
  embed entry_capacity: _U64x5 = _U64x5
  embed arena_capacity: _U64x5 = _U64x5

struct _U64x5
  var a: U64 = 1024
  var b: U64 = 1024
  var c: U64 = 1024
  var d: U64 = 1024
  var e: U64 = 1024

class _Engine
  """One engine per Database (one GPU, one key shard); owned by one actor."""
  let ptr: Pointer[None] tag

  new create(device: I32 = 0) ? =>
    let cfg = JyConfig
    @jy_config_default(cfg)
    cfg.device = device
    var p = Pointer[None]
    if @jy_engine_create(cfg, addressof p) != 0 then error end
    ptr = p

  fun check(rc: I32) ? => if rc != 0 then error end

  fun _final() => @jy_engine_destroy(ptr)

class _Keys
  """Array[(String, Any box)] keys marshalled as bytes + offsets."""
  let bytes: Array[U8] = bytes.create()
  let offs: Array[U64] = offs.create()

  new create(deltas: Array[(String, Any box)] val) =>
    offs.push(0)
    for (k, _) in deltas.values() do
      bytes.append(k)
      offs.push(bytes.size().u64())
    end
