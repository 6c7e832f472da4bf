"""
FFI declarations of the MI355X engine (include/jylis_gpu.h), for package
jylis.  NOT COMPILE-CHECKED: UNBUILT in this repository: the image has no ponyc and jemc/pony-crdt
is not vendored (DESIGN.md "Oracle").  Every @-call returns an I32 status
(0 ok, negative JY_E*); pointers are borrowed for the duration of the call
(JyHost memory: the engine stages host buffers itself).
"""

use "lib:jylis_gpu"

// ---- lifecycle ---------------------------------------------------------------
use @jy_config_default[None](cfg: JyConfig tag)
use @jy_engine_create[I32](cfg: JyConfig tag, out: Pointer[Pointer[None] tag] tag)
use @jy_engine_destroy[None](eng: Pointer[None] tag)
use @jy_last_error[Pointer[U8] val](eng: Pointer[None] tag)
use @jy_skipped[U64](eng: Pointer[None] tag)
use @jy_sync[I32](eng: Pointer[None] tag)

// ---- replicas, keys, values ---------------------------------------------------
use @jy_replica_col[I32](eng: Pointer[None] tag, id: U64, col: Pointer[U32] tag)
use @jy_replica_id[I32](eng: Pointer[None] tag, col: U32, id: Pointer[U64] tag)
use @jy_keys_intern[I32](eng: Pointer[None] tag, ty: I32, n: U64,
  key_bytes: Pointer[U8] tag, key_offs: Pointer[U64] tag, slots: Pointer[U32] tag)
use @jy_keys_lookup[I32](eng: Pointer[None] tag, ty: I32, n: U64,
  key_bytes: Pointer[U8] tag, key_offs: Pointer[U64] tag, slots: Pointer[U32] tag)
use @jy_values_pack[I32](eng: Pointer[None] tag, ty: I32, n: U64,
  bytes: Pointer[U8] tag, offs: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag)
use @jy_arena_read[I32](eng: Pointer[None] tag, ty: I32, off: U64, len: U64, dst: Pointer[U8] tag)
use @jy_arena_usage[I32](eng: Pointer[None] tag, ty: I32, len_out: Pointer[U64] tag, cap_out: Pointer[U64] tag)
use @jy_arena_collect[I32](eng: Pointer[None] tag, ty: I32, live_out: Pointer[U64] tag)

// ---- GCOUNT / PNCOUNT ---------------------------------------------------------
use @jy_gcount_converge[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  col: Pointer[U16] tag, value: Pointer[U64] tag, mem: I32)
use @jy_gcount_converge_block[I32](eng: Pointer[None] tag, ncols: U32, cols: Pointer[U16] tag,
  slot0: U32, nslots: U32, vals: Pointer[U64] tag, mem: I32)
use @jy_counter_converge_keys[I32](eng: Pointer[None] tag, ty: I32, nkeys: U64,
  key_bytes: Pointer[U8] tag, key_offs: Pointer[U64] tag, ncells: U64, cell_key: Pointer[U32] tag,
  sign: Pointer[U8] tag, col: Pointer[U16] tag, value: Pointer[U64] tag, mem: I32)
use @jy_replica_count[U32](eng: Pointer[None] tag)
use @jy_keys_count[U64](eng: Pointer[None] tag, ty: I32)
use @jy_keys_export[I32](eng: Pointer[None] tag, ty: I32, slot0: U64, n: U64, offs: Pointer[U64] tag,
  bytes: Pointer[U8] tag, cap: U64)
use @jy_gcount_get[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  out: Pointer[U64] tag, mem: I32)
use @jy_pncount_converge[I32](eng: Pointer[None] tag,
  np: U64, pslot: Pointer[U32] tag, pcol: Pointer[U16] tag, pval: Pointer[U64] tag,
  nn: U64, nslot: Pointer[U32] tag, ncol: Pointer[U16] tag, nval: Pointer[U64] tag, mem: I32)
use @jy_pncount_converge_block[I32](eng: Pointer[None] tag, ncols: U32, cols: Pointer[U16] tag,
  slot0: U32, nslots: U32, vals_p: Pointer[U64] tag, vals_n: Pointer[U64] tag, mem: I32)
use @jy_pncount_get[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  out: Pointer[I64] tag, mem: I32)
use @jy_counter_write[I32](eng: Pointer[None] tag, ty: I32, sign: I32, col: U32, n: U64,
  slot: Pointer[U32] tag, value: Pointer[U64] tag, mem: I32)
use @jy_counter_deltas_size[I32](eng: Pointer[None] tag, ty: I32, n_out: Pointer[U64] tag)
use @jy_counter_flush[I32](eng: Pointer[None] tag, ty: I32, cap: U64, slot_out: Pointer[U32] tag,
  vals_out: Pointer[U64] tag, mask_out: Pointer[U32] tag, n_out: Pointer[U64] tag, mem: I32)

// ---- TREG ----------------------------------------------------------------------
use @jy_treg_converge[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag, mem: I32)
use @jy_treg_read[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag)
use @jy_treg_set[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag, mem: I32)
use @jy_treg_deltas_size[I32](eng: Pointer[None] tag, n_out: Pointer[U64] tag)
use @jy_treg_flush[I32](eng: Pointer[None] tag, cap: U64, slot_out: Pointer[U32] tag,
  ts_out: Pointer[U64] tag, pre_out: Pointer[U64] tag, lr_out: Pointer[U64] tag,
  n_out: Pointer[U64] tag, mem: I32)

// ---- TLOG ----------------------------------------------------------------------
use @jy_tlog_converge[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  cutoff: Pointer[U64] tag, ent_offs: Pointer[U64] tag, nent: U64,
  ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag, mem: I32)
use @jy_tlog_read_sizes[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  len_out: Pointer[U64] tag, cutoff_out: Pointer[U64] tag)
use @jy_tlog_read[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  out_offs: Pointer[U64] tag, ts: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag)
use @jy_tlog_write[I32](eng: Pointer[None] tag, n: U64, op: Pointer[U8] tag, slot: Pointer[U32] tag,
  ts: Pointer[U64] tag, arg: Pointer[U64] tag, pre: Pointer[U64] tag, lr: Pointer[U64] tag, mem: I32)
use @jy_tlog_deltas_size[I32](eng: Pointer[None] tag, n_out: Pointer[U64] tag)
use @jy_tlog_flush[I32](eng: Pointer[None] tag, cap_keys: U64, cap_ent: U64,
  slot_out: Pointer[U32] tag, cutoff_out: Pointer[U64] tag, ent_offs_out: Pointer[U64] tag,
  ts_out: Pointer[U64] tag, pre_out: Pointer[U64] tag, lr_out: Pointer[U64] tag,
  nkeys_out: Pointer[U64] tag, nent_out: Pointer[U64] tag, mem: I32)

// ---- UJSON ---------------------------------------------------------------------
use @jy_ujson_converge[I32](eng: Pointer[None] tag, n: U64, slot: Pointer[U32] tag,
  el_offs: Pointer[U64] tag, nel: U64, dots: Pointer[U64] tag, elems: Pointer[U64] tag,
  vv_offs: Pointer[U64] tag, nvv: U64, vv: Pointer[U64] tag,
  cloud_offs: Pointer[U64] tag, ncloud: U64, cloud: Pointer[U64] tag, mem: I32)
use @jy_ujson_read_sizes[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  nel_out: Pointer[U64] tag, ncloud_out: Pointer[U64] tag)
use @jy_ujson_read[I32](eng: Pointer[None] tag, n: U64, slots: Pointer[U32] tag,
  el_offs: Pointer[U64] tag, dots: Pointer[U64] tag, elems: Pointer[U64] tag, vv: Pointer[U64] tag,
  cloud_offs: Pointer[U64] tag, cloud: Pointer[U64] tag)
use @jy_ujson_write[I32](eng: Pointer[None] tag, n: U64, op: Pointer[U8] tag, slot: Pointer[U32] tag,
  elem: Pointer[U64] tag, col: U32, mem: I32)
use @jy_ujson_deltas_size[I32](eng: Pointer[None] tag, n_out: Pointer[U64] tag)
use @jy_ujson_flush[I32](eng: Pointer[None] tag, cap_docs: U64, cap_el: U64, cap_cloud: U64,
  slot_out: Pointer[U32] tag, el_offs_out: Pointer[U64] tag, dots_out: Pointer[U64] tag,
  elems_out: Pointer[U64] tag, vv_out: Pointer[U64] tag, cloud_offs_out: Pointer[U64] tag,
  cloud_out: Pointer[U64] tag, ndocs_out: Pointer[U64] tag, nel_out: Pointer[U64] tag,
  ncloud_out: Pointer[U64] tag, mem: I32)

// ---- the node: every GPU of this Jylis node (jy_node.hip) ---------------------
use @jy_device_count[I32]()
use @jy_node_create_local[I32](nshards: U32, devices: Pointer[I32] tag, fabric: U32, cfg: JyConfig tag,
  out: Pointer[Pointer[None] tag] tag)
use @jy_node_destroy[None](node: Pointer[None] tag)
use @jy_node_last_error[Pointer[U8] val](node: Pointer[None] tag)
use @jy_node_engine[Pointer[None] tag](node: Pointer[None] tag, shard: U32)
use @jy_node_shard_of[U32](node: Pointer[None] tag, key: Pointer[U8] tag, len: U64)
use @jy_node_replica_col[I32](node: Pointer[None] tag, id: U64, col: Pointer[U32] tag)
use @jy_node_sync[I32](node: Pointer[None] tag)
use @jy_node_nshards[U32](node: Pointer[None] tag)
// one node per process, shared by the five repos; the calls enqueue
use @jy_node_acquire_local[I32](cfg: JyConfig tag, out: Pointer[Pointer[None] tag] tag)
use @jy_node_release[None](node: Pointer[None] tag)
use @jy_node_fence[I32](node: Pointer[None] tag)
use @jy_node_lock[I32](node: Pointer[None] tag)
use @jy_node_unlock[None](node: Pointer[None] tag)
use @jy_node_lock_type[I32](node: Pointer[None] tag, ty: I32)
use @jy_node_pending[I32](node: Pointer[None] tag, ty: I32, n_out: Pointer[U64] tag)
use @jy_node_arena_gc[I32](node: Pointer[None] tag, enable: U32)
use @jy_node_counter_converge[I32](node: Pointer[None] tag, ty: I32, n: U64, key_bytes: Pointer[U8] tag,
  key_offs: Pointer[U64] tag, cell_offs: Pointer[U64] tag, sign: Pointer[U8] tag, col: Pointer[U16] tag,
  value: Pointer[U64] tag, mem: I32)
use @jy_node_treg_converge[I32](node: Pointer[None] tag, n: U64, key_bytes: Pointer[U8] tag,
  key_offs: Pointer[U64] tag, ts: Pointer[U64] tag, val_bytes: Pointer[U8] tag, val_offs: Pointer[U64] tag,
  mem: I32)
use @jy_node_tlog_converge[I32](node: Pointer[None] tag, n: U64, key_bytes: Pointer[U8] tag,
  key_offs: Pointer[U64] tag, cutoff: Pointer[U64] tag, ent_offs: Pointer[U64] tag, ts: Pointer[U64] tag,
  val_bytes: Pointer[U8] tag, val_offs: Pointer[U64] tag, mem: I32)
use @jy_node_ujson_converge[I32](node: Pointer[None] tag, n: U64, key_bytes: Pointer[U8] tag,
  key_offs: Pointer[U64] tag, el_offs: Pointer[U64] tag, dots: Pointer[U64] tag, elems: Pointer[U64] tag,
  vv_offs: Pointer[U64] tag, vv: Pointer[U64] tag, cloud_offs: Pointer[U64] tag, cloud: Pointer[U64] tag,
  mem: I32)

primitive JyFabricRccl fun apply(): U32 => 0
primitive JyHost fun apply(): I32 => 0
primitive JyGCOUNT fun apply(): I32 => 0
primitive JyPNCOUNT fun apply(): I32 => 1
primitive JyTREG fun apply(): I32 => 2
primitive JyTLOG fun apply(): I32 => 3
primitive JyUJSON fun apply(): I32 => 4
primitive JyNoSlot fun apply(): U32 => U32.max_value()
primitive JyNoFence fun apply(): I32 => -1
primitive JyDotSeqBits fun apply(): U64 => 48
// queued converge pairs that force a drain before the next entry point
primitive _DrainBound fun apply(): USize => 65536

// struct jy_config (include/jylis_gpu.h): field order and widths match
struct JyConfig
  var device: I32 = 0
  var counter_columns: U32 = 16
  var ujson_columns: U32 = 16
  var flags: U32 = 0
  embed key_capacity: _U64x5 = _U64x5
  embed entry_capacity: _U64x5 = _U64x5
  embed arena_capacity: _U64x5 = _U64x5

struct _U64x5
  var a: U64 = 1024
  var b: U64 = 1024
  var c: U64 = 1024
  var d: U64 = 1024
  var e: U64 = 1024
