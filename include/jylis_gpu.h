/* jylis_gpu.h -- C ABI of the MI355X CRDT delta-convergence engine.
 *
 * Drop-in point: RepoManagerCore.converge_deltas (jylis/repo_manager.pony:92-93)
 * loops `_repo.converge(k, d)` over one decoded MsgPushDeltas batch
 * (jylis/msg.pony:20-24).  A GPU-backed Repo* marshals that whole
 * Array[(String, Any box)] into structure-of-arrays once and makes ONE call
 * here per batch (see INTEGRATION.md for the Pony FFI declarations).
 *
 * Conventions
 *   - every entry returns int32 status: 0 ok, < 0 error (detail in
 *     jy_last_error).  Pony FFI has no exceptions; the reference swallows
 *     converge failures (`try ... end`, repo_gcount.pony:51), so malformed
 *     entries are skipped and counted, never fatal (jy_skipped()).
 *   - pointers are borrowed for the duration of the call only.  `mem` says
 *     where they live: JY_HOST (copied through pinned staging) or JY_DEVICE
 *     (HBM-resident; read asynchronously on the engine stream, keep them
 *     alive until jy_sync).
 *   - one engine = one GPU = one key shard.  An engine handle is not
 *     thread-safe: the caller serialises calls (one RepoManager actor per
 *     type, repo_manager.pony:18).  No thread-local HIP state is assumed.
 *   - keys are interned to dense per-type slots (u32); replica identities
 *     (u64 Address.hash64, jylis/address.pony:29-33) to dense columns (u16).
 *   - within ONE converge call every slot appears at most once (a batch
 *     comes from the sender's `_deltas` Map, repo_gcount.pony:14,19-23).
 *     Host-pointer calls enforce this by splitting into rounds; device
 *     batches must honour it (routed batches are converged per source).
 */
#ifndef JYLIS_GPU_H
#define JYLIS_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JY_OK 0
#define JY_EINVAL (-1)
#define JY_ENOMEM (-2)
#define JY_EHIP (-3)
#define JY_ERANGE (-4)
#define JY_ETYPE (-5)

#define JY_NO_SLOT 0xFFFFFFFFu

/* CRDT types: the RepoManager names of database.pony:18-22 */
enum { JY_GCOUNT = 0, JY_PNCOUNT = 1, JY_TREG = 2, JY_TLOG = 3, JY_UJSON = 4, JY_NTYPES = 5 };
enum { JY_HOST = 0, JY_DEVICE = 1 };

typedef struct jy_engine jy_engine;

/* jy_config.flags: test switches that force a kernel form the engine would
 * otherwise pick by state size (the parity tests reach every form) */
#define JY_CFG_TREG_WHOLE_LINES 1u /* k_treg_lww<true>: every handle line rewritten */
#define JY_CFG_TREG_DUP_TEST 2u    /* a fixed 64-record TREG duplicate list the host never folds
                                      ahead of time: a test overflows it and expects JY_ERANGE */

typedef struct jy_config {
  int32_t device;            /* HIP device ordinal                                   */
  uint32_t counter_columns;  /* initial replica-column capacity of GCOUNT/PNCOUNT    */
  uint32_t ujson_columns;    /* version-vector width of UJSON contexts (fixed)       */
  uint32_t flags;            /* JY_CFG_* switches; 0 in production                   */
  uint64_t key_capacity[JY_NTYPES];   /* initial slots per type (grows by doubling)  */
  uint64_t entry_capacity[JY_NTYPES]; /* initial TLOG entries / UJSON dots            */
  uint64_t arena_capacity[JY_NTYPES]; /* initial string arena bytes (TREG, TLOG)      */
} jy_config;

/* ---- engine lifecycle (replaces RepoXXX.create(identity), repo_manager.pony:6) ---- */
void jy_config_default(jy_config* cfg);
int32_t jy_engine_create(const jy_config* cfg, jy_engine** out);
void jy_engine_destroy(jy_engine* eng);
const char* jy_last_error(const jy_engine* eng);
uint64_t jy_skipped(const jy_engine* eng);      /* malformed entries skipped so far  */
int32_t jy_set_stream(jy_engine* eng, void* hip_stream); /* NULL: engine-owned stream */
void* jy_get_stream(jy_engine* eng);
int32_t jy_sync(jy_engine* eng);
/* measurement (not on the reference's surface; bench.py and rocprof
 * cross-checks): while enabled, every merge call brackets its device work
 * (first to last launch, host staging excluded) with HIP events on the
 * engine stream.  jy_timing_read waits for them, writes up to `cap`
 * per-call durations in ms, returns the count in *n_out and clears them. */
int32_t jy_timing_enable(jy_engine* eng, int32_t on);
int32_t jy_timing_read(jy_engine* eng, uint64_t cap, double* ms_out, uint64_t* n_out);

/* ---- replica dictionary: u64 identity <-> dense column ---- */
int32_t jy_replica_col(jy_engine* eng, uint64_t replica_id, uint32_t* col_out);
int32_t jy_replica_id(const jy_engine* eng, uint32_t col, uint64_t* id_out);
uint32_t jy_replica_count(const jy_engine* eng);

/* ---- key interning: `_data_for(key)` (repo_gcount.pony:36-41) creates on miss,
 *      `_data(key)?` (repo_gcount.pony:53-55) only looks up (JY_NO_SLOT) ---- */
int32_t jy_keys_intern(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* key_bytes,
                       const uint64_t* key_offs, uint32_t* slots_out);
int32_t jy_keys_lookup(const jy_engine* eng, int32_t type, uint64_t n, const uint8_t* key_bytes,
                       const uint64_t* key_offs, uint32_t* slots_out);
/* The key directory lives in HBM (hash table + key bytes, k_keys.hip); the
 * host-pointer calls above consult a host cache first and send the misses to
 * it.  The _mem forms take key_bytes / key_offs / slots_out in HBM when
 * mem = JY_DEVICE (bulk interning with no host round trip per key).  Slots
 * are dense, per type, handed out in order of first occurrence. */
int32_t jy_keys_intern_mem(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* key_bytes,
                           const uint64_t* key_offs, uint32_t* slots_out, int32_t mem);
int32_t jy_keys_lookup_mem(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* key_bytes,
                           const uint64_t* key_offs, uint32_t* slots_out, int32_t mem);
uint64_t jy_keys_count(const jy_engine* eng, int32_t type);
/* the key strings of slots [slot0, slot0 + n) (host out): offs_out u64[n + 1];
 * bytes_out is written when cap_bytes >= offs_out[n] (else sizes only).
 * Keys interned on the device (jy_keys_intern_mem, jy_keys_intern_lens) get
 * their names back this way.  Blocks. */
int32_t jy_keys_export(jy_engine* eng, int32_t type, uint64_t slot0, uint64_t n, uint64_t* offs_out,
                       uint8_t* bytes_out, uint64_t cap_bytes);
int32_t jy_keys_reserve(jy_engine* eng, int32_t type, uint64_t key_capacity);
/* owner shard of a key when keys are hash-sharded over `nshards` engines */
uint32_t jy_key_owner(const uint8_t* key, uint64_t len, uint32_t nshards);

/* ---- string arena of TREG / TLOG values (value bytes beyond the 8-byte prefix) ----
 * A value is held as (prefix u64 = first 8 bytes big-endian, zero padded;
 * lr u64 = arena_offset << 24 | length).  Values of <= 8 bytes never touch
 * the arena.  jy_values_pack appends long values (each on an 8-byte
 * boundary) and fills pre/lr. */
int32_t jy_values_pack(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* bytes,
                       const uint64_t* offs, uint64_t* pre_out, uint64_t* lr_out);

/* arena bytes in use / reserved (host counters, no GPU work) */
int32_t jy_arena_usage(jy_engine* eng, int32_t type, uint64_t* len_out, uint64_t* cap_out);
/* Reclaim the arena (TREG, TLOG): copy the values every live register, log
 * entry and pending delta still references back to back into a fresh arena
 * and rewrite their handles; *live_out = the bytes kept.  Handles packed by
 * jy_values_pack but not yet merged become INVALID: call between converge /
 * write calls (the reference frees a replaced value, repo_treg.pony:51-52).
 * Blocks. */
int32_t jy_arena_collect(jy_engine* eng, int32_t type, uint64_t* live_out);

/* ---- GCOUNT: GCounter.converge (repo_gcount.pony:50-51) / value (:53-55) ----
 * COO form: n cells (slot, col, value): s[slot][col] = max(s, value). */
int32_t jy_gcount_converge(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint16_t* col,
                           const uint64_t* val, int32_t mem);
/* Column-block form: ncols peer columns over the slot run [slot0, slot0+nslots);
 * vals is [ncols][nslots] (one flushed peer batch per column, in slot order). */
int32_t jy_gcount_converge_block(jy_engine* eng, uint32_t ncols, const uint16_t* cols_host,
                                 uint32_t slot0, uint32_t nslots, const uint64_t* vals, int32_t mem);
int32_t jy_gcount_get(jy_engine* eng, uint64_t n, const uint32_t* slots, uint64_t* out, int32_t mem);

/* ---- GCOUNT / PNCOUNT: one decoded peer batch WITH its key strings ----
 * RepoManagerCore.converge_deltas (repo_manager.pony:92-93) of a counter
 * batch including each key's _data_for (repo_gcount.pony:36-41,
 * repo_pncount.pony:38-43: create on miss) in ONE call: the nkeys key strings
 * (key_bytes / key_offs, as jy_keys_intern) are interned on the device and
 * the ncells cells merged with their device slots -- no slot crosses to the
 * host (jy_keys_intern + jy_gcount_converge move every slot down and up).
 * Cell i belongs to key cell_key[i] (NULL: cell i is key i, ncells == nkeys)
 * and, for PNCOUNT, to sign[i] (0 = P, 1 = N; NULL: all P); GCOUNT takes
 * sign NULL.  s[slot][col] = max(s, val).  mem applies to every array (with
 * JY_DEVICE the key bytes / offsets are in HBM too). */
int32_t jy_counter_converge_keys(jy_engine* eng, int32_t type, uint64_t nkeys, const uint8_t* key_bytes,
                                 const uint64_t* key_offs, uint64_t ncells, const uint32_t* cell_key,
                                 const uint8_t* sign, const uint16_t* col, const uint64_t* val, int32_t mem);

/* ---- PNCOUNT: two GCounters (repo_pncount.pony:52-57); GET = (sum P - sum N) as i64 ---- */
int32_t jy_pncount_converge(jy_engine* eng, uint64_t np, const uint32_t* pslot, const uint16_t* pcol,
                            const uint64_t* pval, uint64_t nn, const uint32_t* nslot,
                            const uint16_t* ncol, const uint64_t* nval, int32_t mem);
/* vals_p / vals_n are each [ncols][nslots] */
int32_t jy_pncount_converge_block(jy_engine* eng, uint32_t ncols, const uint16_t* cols_host,
                                  uint32_t slot0, uint32_t nslots, const uint64_t* vals_p,
                                  const uint64_t* vals_n, int32_t mem);
int32_t jy_pncount_get(jy_engine* eng, uint64_t n, const uint32_t* slots, int64_t* out, int32_t mem);

/* counter state dump for parity checks: out is [nsigns][ncols][nslots] over
 * columns [0, ncols) and slots [slot0, slot0+nslots) (host memory) */
int32_t jy_counter_export(jy_engine* eng, int32_t type, uint32_t ncols, uint32_t slot0,
                          uint32_t nslots, uint64_t* out);

/* ---- counter write path: the local writes that produce deltas ----
 * jy_counter_write: n writes of THIS replica, whose column is `col`
 * (= jy_replica_col(identity)): GCOUNT INC (sign 0, RepoGCOUNT.inc
 * repo_gcount.pony:57-60), PNCOUNT INC (sign 0) / DEC (sign 1)
 * (RepoPNCOUNT.inc/dec repo_pncount.pony:59-67; the i64 argument bit-cast to
 * u64).  s[slot][col] += v (wrapping); each key's pending delta records its
 * post-write total (GCounter.increment).  Keys may repeat within a batch. */
int32_t jy_counter_write(jy_engine* eng, int32_t type, int32_t sign, uint32_t col, uint64_t n,
                         const uint32_t* slot, const uint64_t* val, int32_t mem);
/* deltas_size() (repo_gcount.pony:16): keys with a pending delta.  Blocks. */
int32_t jy_counter_deltas_size(jy_engine* eng, int32_t type, uint64_t* n_out);
/* flush_deltas() (repo_gcount.pony:18-23): every pending key, ascending slot:
 * slot_out[i]; vals_out[sign * cap + i] = the recorded total (0 where that
 * sign was not written); mask_out[i] bit s set iff sign s was written.  Clears
 * the pending set.  *n_out = the count; JY_ERANGE (nothing cleared, *n_out =
 * the count needed) if cap is smaller.  Blocks. */
int32_t jy_counter_flush(jy_engine* eng, int32_t type, uint64_t cap, uint32_t* slot_out,
                         uint64_t* vals_out, uint32_t* mask_out, uint64_t* n_out, int32_t mem);

/* ---- TREG: TRegString.converge (repo_treg.pony:51-52), LWW by (ts, value) ----
 * An entry whose slot is JY_NO_SLOT is skipped (a key not interned). */
int32_t jy_treg_converge(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint64_t* ts,
                         const uint64_t* pre, const uint64_t* lr, int32_t mem);
/* The same join for a BLOCK batch: entry i is the delta of slot slot0 + i
 * (a full-state delta, or a shard's batch regrouped in slot order), so no
 * slot stream is read and no slot can repeat.  [slot0, slot0 + n) must be
 * interned (JY_ERANGE otherwise). */
int32_t jy_treg_converge_block(jy_engine* eng, uint32_t slot0, uint64_t n, const uint64_t* ts,
                               const uint64_t* pre, const uint64_t* lr, int32_t mem);
/* read (ts, pre, lr) for n slots (host out) and fetch arena bytes */
int32_t jy_treg_read(jy_engine* eng, uint64_t n, const uint32_t* slots, uint64_t* ts_out,
                     uint64_t* pre_out, uint64_t* lr_out);
int32_t jy_arena_read(jy_engine* eng, int32_t type, uint64_t offset, uint64_t len, uint8_t* dst);

/* ---- TREG write path: RepoTREG.set (repo_treg.pony:65-68) ----
 * n local SETs (slot, ts, value handle from jy_values_pack): a SET that wins
 * against the state (LWW as converge) changes it and is LWW-merged into the
 * key's pending delta; the key's delta exists even when the SET loses
 * (_delta_for is evaluated either way).  Host batches may repeat keys (applied
 * in order); a device batch holds one entry per key. */
int32_t jy_treg_set(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint64_t* ts,
                    const uint64_t* pre, const uint64_t* lr, int32_t mem);
int32_t jy_treg_deltas_size(jy_engine* eng, uint64_t* n_out);  /* deltas_size(); blocks */
/* flush_deltas() (repo_treg.pony:18-22): every pending key, ascending slot,
 * with its delta register (ts, pre, lr; a losing-only key reads ("", 0)), then
 * clears them.  JY_ERANGE (nothing cleared, *n_out = needed) if cap is short. */
int32_t jy_treg_flush(jy_engine* eng, uint64_t cap, uint32_t* slot_out, uint64_t* ts_out,
                      uint64_t* pre_out, uint64_t* lr_out, uint64_t* n_out, int32_t mem);

/* ---- TLOG: TLog[String].converge (repo_tlog.pony:66-67) ----
 * nkeys delta logs, CSR: entries of key i are [ent_offs[i], ent_offs[i+1]),
 * canonical (later ts first, then greater value; unique; ts >= cutoff[i]).
 * Non-canonical segments are skipped (counted in jy_skipped). */
int32_t jy_tlog_converge(jy_engine* eng, uint64_t nkeys, const uint32_t* slot, const uint64_t* cutoff,
                         const uint64_t* ent_offs, uint64_t nent, const uint64_t* ts,
                         const uint64_t* pre, const uint64_t* lr, int32_t mem);
/* ---- TLOG write path: RepoTLOG.ins / trimat / trim / clr (repo_tlog.pony:85-111) ----
 * n commands applied in order: op[i] is JY_TLOG_INS (value handle pre/lr from
 * jy_values_pack at ts[i]), JY_TLOG_TRIMAT (ts[i]), JY_TLOG_TRIM (arg[i] =
 * count) or JY_TLOG_CLR.  Each changes the state as TLog.write / raise_cutoff
 * / trim / clear do, and where it changed the state the same change goes into
 * the key's pending delta log; every command marks its key pending.  Host
 * batches may repeat keys (applied in order); a device batch holds one
 * command per key.  Unused columns may be null. */
#define JY_TLOG_INS 0
#define JY_TLOG_TRIMAT 1
#define JY_TLOG_TRIM 2
#define JY_TLOG_CLR 3
int32_t jy_tlog_write(jy_engine* eng, uint64_t n, const uint8_t* op, const uint32_t* slot, const uint64_t* ts,
                      const uint64_t* arg, const uint64_t* pre, const uint64_t* lr, int32_t mem);
int32_t jy_tlog_deltas_size(jy_engine* eng, uint64_t* n_out);  /* deltas_size(); blocks */
/* flush_deltas() (repo_tlog.pony:21-25): every pending key, ascending slot,
 * with its delta log (cutoff, entries newest first as a CSR); then clears
 * them.  With cap_keys / cap_ent too small nothing is written or cleared and
 * *nkeys_out / *nent_out report the sizes needed (JY_OK). */
int32_t jy_tlog_flush(jy_engine* eng, uint64_t cap_keys, uint64_t cap_ent, uint32_t* slot_out,
                      uint64_t* cutoff_out, uint64_t* ent_offs_out, uint64_t* ts_out, uint64_t* pre_out,
                      uint64_t* lr_out, uint64_t* nkeys_out, uint64_t* nent_out, int32_t mem);
/* Threading: a TLOG converge only enqueues.  Where a merge's rebuilt logs do
 * not fit the entry pool, the device leaves those keys as they were and keeps
 * their deltas; they are re-merged after a pool compaction by the next call
 * that finds the merge finished, or by any call that reads TLOG state (reads,
 * write commands, flush, jy_arena_collect, jy_sync), which waits for it.  A
 * call that fails midway may have applied part of its batch; retrying it is
 * safe (the join is idempotent). */
/* telemetry of the state store (not on the reference's surface): [0] merges
 * issued, [1] merges whose rebuilt logs were spilled and re-merged, [2] pool
 * compactions, [3] pool capacity in entries */
int32_t jy_tlog_stats(jy_engine* eng, uint64_t* out4);
/* two-phase read: sizes (n entries per slot + cutoffs), then entries */
int32_t jy_tlog_read_sizes(jy_engine* eng, uint64_t n, const uint32_t* slots, uint64_t* len_out,
                           uint64_t* cutoff_out);
int32_t jy_tlog_read(jy_engine* eng, uint64_t n, const uint32_t* slots, const uint64_t* out_offs,
                     uint64_t* ts_out, uint64_t* pre_out, uint64_t* lr_out);

/* ---- UJSON: UJSON.converge (repo_ujson.pony:65-66), dot-kernel join ----
 * dots are packed (col << 48 | seq), seq in [1, 2^48).  Per doc i:
 *   elements [el_offs[i], el_offs[i+1]) of (dots, elems), dots ascending;
 *   context  version vector [vv_offs[i], vv_offs[i+1]) of packed (col << 48 | n)
 *            meaning "every seq <= n of col seen", plus
 *            cloud [cloud_offs[i], cloud_offs[i+1]) of packed dots, ascending. */
int32_t jy_ujson_converge(jy_engine* eng, uint64_t ndocs, const uint32_t* slot, const uint64_t* el_offs,
                          uint64_t nel, const uint64_t* dots, const uint64_t* elems,
                          const uint64_t* vv_offs, uint64_t nvv, const uint64_t* vv,
                          const uint64_t* cloud_offs, uint64_t ncloud, const uint64_t* cloud,
                          int32_t mem);
/* two-phase read: per slot element / cloud counts, then contents; vv_out is
 * [n][ujson_columns] dense */
int32_t jy_ujson_read_sizes(jy_engine* eng, uint64_t n, const uint32_t* slots, uint64_t* nel_out,
                            uint64_t* ncloud_out);
int32_t jy_ujson_read(jy_engine* eng, uint64_t n, const uint32_t* slots, const uint64_t* el_offs,
                      uint64_t* dots_out, uint64_t* elems_out, uint64_t* vv_out,
                      const uint64_t* cloud_offs, uint64_t* cloud_out);

/* ---- UJSON write path: RepoUJSON.ins / rm / clr (repo_ujson.pony:74-110) ----
 * Elements are opaque handles (the host interns (path, value) leaves; path-
 * scoped CLR and SET are host compositions of RM / INS).  n commands applied
 * in order: JY_UJSON_INS elem[i] under a fresh dot of replica column col
 * (seq = the doc's vv[col] + 1); JY_UJSON_RM removes every element equal to
 * elem[i] (observed remove); JY_UJSON_CLR removes every element of the doc.
 * Each command's delta is converged into the state and into the doc's pending
 * delta; every command marks its doc pending (issue RM / CLR only for docs
 * that exist: repo_ujson.pony:86,108 create nothing).  Host batches may repeat
 * docs (applied in order); a device batch holds one command per doc. */
#define JY_UJSON_INS 0
#define JY_UJSON_RM 1
#define JY_UJSON_CLR 2
int32_t jy_ujson_write(jy_engine* eng, uint64_t n, const uint8_t* op, const uint32_t* slot, const uint64_t* elem,
                       uint32_t col, int32_t mem);
int32_t jy_ujson_deltas_size(jy_engine* eng, uint64_t* n_out);  /* deltas_size(); blocks */
/* flush_deltas() (repo_ujson.pony:22-26): every pending doc, ascending slot,
 * with its delta document (elements CSR, dense vv [ndocs][ujson_columns],
 * cloud CSR), then clears them.  Caps too small: sizes only (JY_OK). */
int32_t jy_ujson_flush(jy_engine* eng, uint64_t cap_docs, uint64_t cap_el, uint64_t cap_cloud, uint32_t* slot_out,
                       uint64_t* el_offs_out, uint64_t* dots_out, uint64_t* elems_out, uint64_t* vv_out,
                       uint64_t* cloud_offs_out, uint64_t* cloud_out, uint64_t* ndocs_out, uint64_t* nel_out,
                       uint64_t* ncloud_out, int32_t mem);

/* cumulative converge counters since the engine was made (synchronising):
 * [0] touched state elements, [1] touched state cloud dots, [2] elements
 * written, [3] cloud dots written, [4] delta elements, [5] delta cloud dots,
 * [6] delta documents, [7] converge calls.  Bench / telemetry only: the
 * bytes a converge really moved.  [0..3] count the regular merge path only. */
int32_t jy_ujson_stats(jy_engine* eng, uint64_t* out8);
/* the same eight, then the in-place layout of long documents:
 * [8] delta docs converged in place, [9] / [10] their state elements / cloud
 * dots (examined by the join, never read), [11] / [12] elements / cloud dots
 * appended, [13] cloud dots folded into the vv, [14] documents promoted to
 * the per-column layout, [15] documents demoted to the regular path */
int32_t jy_ujson_stats_ext(jy_engine* eng, uint64_t* out16);
/* UJSON in-place layout (an engine choice, invisible in every result): a
 * document whose merged state holds at least min_elems elements keeps one
 * element run and one cloud run per replica column with room behind it, so
 * a delta whose dots all lie above what the document's column holds (the
 * usual case: fresh inserts) is appended where it lies instead of rewriting
 * the document.  0 stops promotions (documents already in the layout stay).
 * Default 512 (env JY_UJ_LONG_MIN); needs ujson_columns <= 64. */
int32_t jy_ujson_set_inplace(jy_engine* eng, uint32_t min_elems);

/* ---- multi-GPU routing: the exchange step of a key-hash-sharded node ----
 * Replaces nothing in the reference (every node holds every key there); it is
 * the intra-node analogue of Cluster.broadcast_deltas (cluster.pony:209-213).
 * Runs have a FIXED capacity per destination, so the all-to-all is an
 * equal-split collective and the counts travel on the device with the data:
 * no host round trip per batch.
 *
 * Sender: jy_treg_route_part partitions n ingested TREG entries (owner
 * shard, slot on the owner, ts, pre, lr) into nshards runs:
 *   recs_dev  u64[nshards][cap][4] {slot, ts, pre, lr'}, 16-B aligned; lr' of a
 *             value > 8 bytes addresses the run's own bytes (8-byte granules)
 *   bytes_dev u8[nshards][cap_byte], cap_byte a multiple of 8
 *   hdr_dev   u64[nshards][2]: records / value bytes placed per destination
 *             (written by the call); entries keep their input order in a run
 *             and the placed ones are a prefix of each destination's sequence
 *   ovf_dev   u32[1 + n]: [0] = entries that did not fit (ZERO on entry), then
 *             their input indices -- the caller sends those in a later round.
 * Receiver: jy_treg_converge_routed merges nsrc received runs (the same
 * layout, source-major, each source's hdr row) in one launch; a key named by
 * several sources is exact (LWW join).  All pointers are device memory
 * except the `mem`-tagged inputs; both calls only enqueue. */
void jy_keys_owner(uint64_t n, const uint8_t* key_bytes, const uint64_t* key_offs, uint32_t nshards,
                   uint32_t* owner_out);
int32_t jy_treg_route_part(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot,
                           const uint64_t* ts, const uint64_t* pre, const uint64_t* lr, uint32_t nshards,
                           uint64_t cap, uint64_t cap_byte, int32_t mem, uint64_t* recs_dev, uint8_t* bytes_dev,
                           uint64_t* hdr_dev, uint32_t* ovf_dev);
/* The same partition on the shard `self` (< nshards) that owns part of its
 * own batch: the entries with owner == self are merged into eng's registers
 * where they lie (the keyed LWW merge, enqueued before the partition) and
 * never enter a run; run `self` stays empty (hdr row 0), its overflow list
 * never names them.  The receivers' merge is unchanged (an empty run costs
 * one launch that reads its count), and at nshards == 1 the caller may skip
 * it and the run buffers altogether. */
int32_t jy_treg_route_part_self(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot,
                                const uint64_t* ts, const uint64_t* pre, const uint64_t* lr, uint32_t nshards,
                                uint32_t self, uint64_t cap, uint64_t cap_byte, int32_t mem, uint64_t* recs_dev,
                                uint8_t* bytes_dev, uint64_t* hdr_dev, uint32_t* ovf_dev);
int32_t jy_treg_converge_routed(jy_engine* eng, uint32_t nsrc, uint64_t cap, uint64_t cap_byte,
                                const uint64_t* recs_dev, const uint8_t* bytes_dev, const uint64_t* hdr_dev);
/* The same merge when the byte runs were received straight into this
 * engine's arena: jy_arena_reserve(eng, JY_TREG, nsrc * cap_byte, &dst,
 * &rebase) hands out the arena's tail (dst stays valid until the next call
 * that grows that arena), the exchange (or, for the sender's own run,
 * jy_treg_route_part with bytes_dev = dst) writes there, and
 * jy_treg_converge_routed_at merges with the runs at arena offset `rebase`
 * -- no append copy of the byte runs. */
int32_t jy_arena_reserve(jy_engine* eng, int32_t type, uint64_t bytes, uint8_t** dev_out, uint64_t* rebase_out);
int32_t jy_treg_converge_routed_at(jy_engine* eng, uint32_t nsrc, uint64_t cap, uint64_t cap_byte,
                                   const uint64_t* recs_dev, const uint64_t* hdr_dev, uint64_t rebase);

/* ---- cross-shard key resolution (k_keyroute.hip): `_data_for(key)`
 * (repo_treg.pony:37-42, every repo_*.pony) when the key's slot lives on
 * another GPU.  All pointers are device memory; the calls only enqueue.
 * Sender: jy_keys_route_part computes every key's owner (jy_key_owner, on the
 * device) and regroups the keys by owner for a variable all-to-all:
 *   owner_out u32[n], pos_out u32[n] (each key's index in owner order),
 *   send_lens u64[n] and send_bytes u8[total key bytes] in owner order,
 *   counts_out u64[2 * nshards]: keys per owner, then bytes per owner.
 * Owner: jy_keys_intern_lens interns the n received keys (lengths + bytes)
 *   in its directory -- create on miss, like jy_keys_intern_mem -- and
 *   writes their slots (it synchronises, as interning does).
 * Sender, once the slots came back in its owner order:
 *   jy_keys_route_back writes slots_out[i] = answers[pos[i]]. */
int32_t jy_keys_route_part(jy_engine* eng, uint64_t n, const uint8_t* key_bytes, const uint64_t* key_offs,
                           uint32_t nshards, uint32_t* owner_out, uint32_t* pos_out, uint64_t* send_lens,
                           uint8_t* send_bytes, uint64_t* counts_out);
int32_t jy_keys_intern_lens(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* bytes, const uint64_t* lens,
                            uint32_t* slots_out);
int32_t jy_keys_route_back(jy_engine* eng, uint64_t n, const uint32_t* pos, const uint32_t* answers,
                           uint32_t* slots_out);

/* ---- routing TLOG logs and UJSON documents (k_route_csr.hip) ----
 * The CSR counterpart of the TREG pair above: a key travels with its whole
 * log / document.  Each destination gets one RUN of jy_route_words(type,
 * cap_k, caps) u64 words, a complete converge batch of cap_k records (TLOG
 * caps = {cap_e}; UJSON caps = {cap_e, cap_v, cap_c} for elements, vv
 * entries, cloud dots); runs_dev is u64[nshards][words], 16-B aligned.
 * Keys keep their input order in a run; the first key of a destination that
 * does not fit (records, entries or long-value bytes) and every later one go
 * to ovf_dev (u32[1 + n]: [0] the count, ZERO before the first call; calls
 * append key_base + their input index, so the chunks of one batch -- key
 * ranges passed as offset pointers with the full entry arrays -- share one
 * list); unused records are holes the receiver skips.  hdr_dev
 * u64[nshards][8] receives per run the keys, the entries per CSR and (TLOG)
 * the value bytes placed (zeroed by the call).  Offsets are absolute: a
 * chunk's ent_offs[0] may be > 0 and nent bounds the entries it names.  TLOG value bytes go to bytes_dev
 * (u8[nshards][cap_byte], cap_byte a multiple of 8); UJSON runs need
 * cap_k >= 2 (the last record is a hole spanning the unused capacity).
 * Receiver: nsrc received runs, source-major; each source's run is merged
 * in turn (TLOG rewrites the runs' value handles in place).  Device-memory
 * pointers except the `mem`-tagged inputs; the calls only enqueue.  A
 * device batch with an owner >= nshards drops that key (counted in
 * jy_skipped). */
uint64_t jy_route_words(int32_t type, uint64_t cap_k, const uint64_t* caps);
int32_t jy_tlog_route_part(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot,
                           const uint64_t* cutoff, const uint64_t* ent_offs, uint64_t nent, const uint64_t* ts,
                           const uint64_t* pre, const uint64_t* lr, uint32_t nshards, uint64_t cap_k, uint64_t cap_e,
                           uint64_t cap_byte, uint64_t key_base, int32_t mem, uint64_t* runs_dev, uint8_t* bytes_dev,
                           uint64_t* hdr_dev, uint32_t* ovf_dev);
int32_t jy_tlog_converge_routed(jy_engine* eng, uint32_t nsrc, uint64_t cap_k, uint64_t cap_e, uint64_t cap_byte,
                                uint64_t* runs_dev, const uint8_t* bytes_dev);
int32_t jy_ujson_route_part(jy_engine* eng, uint64_t n, const uint32_t* owner, const uint32_t* slot,
                            const uint64_t* el_offs, uint64_t nel, const uint64_t* dots, const uint64_t* elems,
                            const uint64_t* vv_offs, uint64_t nvv, const uint64_t* vv, const uint64_t* cloud_offs,
                            uint64_t ncloud, const uint64_t* cloud, uint32_t nshards, uint64_t cap_k, uint64_t cap_e,
                            uint64_t cap_v, uint64_t cap_c, uint64_t key_base, int32_t mem, uint64_t* runs_dev,
                            uint64_t* hdr_dev, uint32_t* ovf_dev);
int32_t jy_ujson_converge_routed(jy_engine* eng, uint32_t nsrc, uint64_t cap_k, uint64_t cap_e, uint64_t cap_v,
                                 uint64_t cap_c, const uint64_t* runs_dev);

/* ---- the node: every GPU of one Jylis node behind one handle (jy_node.hip) ----
 * Replaces, for the whole node, Database.converge_deltas (jylis/database.pony:50-51)
 * -> RepoManager.converge_deltas -> RepoManagerCore.converge_deltas
 * (jylis/repo_manager.pony:30-31,92-93): ONE call per decoded peer batch, its
 * keys hash-sharded over the node's GPUs (owner = jy_key_owner(key, S)).  The
 * reference has no sharding (every node holds every key); the exchange step
 * is the intra-node analogue of Cluster.broadcast_deltas (cluster.pony:205-213).
 *
 * A node has S shards (one engine each).  One process may drive all of them
 * (the Pony host: nlocal = S) or several processes one each (nlocal = 1,
 * rank0 = the process's rank, one ncclUniqueId shared by all of them).
 * Per converge call, per shard: the batch the process passed is cut into
 * nlocal contiguous key ranges, one per local shard (its ingest); each ingest
 * shard hashes its keys on the device and regroups keys and payload by owner;
 * the per-owner counts are exchanged (RCCL, or a host transposition for the
 * copy fabric) and read back once; the payload moves with grouped
 * ncclSend/ncclRecv over xGMI (or device copies); each owner interns the keys
 * it received in its device directory (_data_for, create on miss) and
 * merges them -- TREG and counters all sources in one launch (LWW / max are
 * joins, repeats are exact), TLOG and UJSON one source after another (a key
 * two peers sent is merged twice, exactly).  No slot crosses the host and
 * no key is resolved by a round trip: the key bytes travel with their delta.
 *
 * Every process of a multi-process node makes the same node calls in the
 * same order (they are collectives), each with its own batch (possibly
 * empty).  Errors: JY_* codes, detail in jy_node_last_error.  Reads, local
 * writes and flushes go to the owner's engine (jy_node_engine).
 *
 * One node per process, shared by every CRDT type (round 5).  The converge
 * calls ENQUEUE: a call checks its arguments, copies host inputs into a
 * pinned block the node owns (JY_HOST inputs are free to reuse when it
 * returns) and queues a job; one worker thread per node runs the jobs in call
 * order -- the count exchange, the key directory's miss count and every other
 * host wait of a converge happen there, never on the caller's thread (a Pony
 * scheduler thread).  The five RepoManager actors may call from five threads
 * at once: their jobs run one at a time, so the node's ONE communicator sees
 * one group at a time, issued from one thread (database.pony:18-23 makes the
 * five actors; cluster.pony:205-213 is the broadcast this replaces).  A
 * queued job's failure is returned by the node's next call (converge, fence,
 * lock, sync, stats) and its detail by jy_node_last_error.
 * JY_DEVICE inputs are read by the worker later, and on streams of the node's
 * own (the read-back stream reads offsets, value lengths and value heads
 * beside the engine stream): they must be complete device-wide before the
 * call (no pending write on any stream) and stay valid and unchanged until
 * jy_node_fence (every queued job issued to its streams) AND the GPU work
 * reading them has finished -- jy_node_sync returns after both.  The engines of a node (jy_node_engine) are shared
 * with the worker: use them between jy_node_lock and jy_node_unlock (the
 * lock first waits for every job queued before it), or after jy_node_sync
 * with no node call in flight. */
typedef struct jy_node jy_node;
#define JY_NODE_MAX_SHARDS 64
#define JY_FABRIC_RCCL 0 /* RCCL communicator over the shards' GPUs (one GPU per shard)   */
#define JY_FABRIC_COPY 1 /* device copies: one process, shards may share a GPU (tests)      */
typedef struct jy_node_config {
  uint32_t nshards;                     /* S: key shards of the node                        */
  uint32_t nlocal;                      /* shards this process drives: rank0 .. rank0+nlocal-1 */
  uint32_t rank0;                       /* first local shard                               */
  uint32_t fabric;                      /* JY_FABRIC_*                                     */
  int32_t devices[JY_NODE_MAX_SHARDS];  /* HIP device of each local shard                  */
  uint8_t unique_id[128];               /* RCCL: one ncclUniqueId for every process of the
                                           node (jy_node_unique_id on one of them); with
                                           nlocal == nshards an all-zero id means "make one" */
  jy_config engine;                     /* each shard's engine (device overridden)         */
} jy_node_config;

int32_t jy_node_unique_id(uint8_t* id_out /* 128 bytes */);
int32_t jy_node_create(const jy_node_config* cfg, jy_node** out);
/* the one-process node of an FFI host without struct layouts (the Pony
 * host): nshards shards on devices[0..nshards), every one local, an RCCL
 * communicator of its own (fabric JY_FABRIC_RCCL) or device copies */
int32_t jy_node_create_local(uint32_t nshards, const int32_t* devices, uint32_t fabric, const jy_config* engine,
                             jy_node** out);
/* The process's shared node (round 5): the first call makes a one-process
 * node over every visible GPU (jy_node_create_local, RCCL, `engine` for each
 * shard); later calls return the same node.  Reference counted: the last
 * jy_node_release destroys it.  The five GPU repos of a Jylis process (one
 * RepoManager actor each, database.pony:18-22) share it, so one communicator
 * and one engine per GPU serve every CRDT type. */
int32_t jy_node_acquire_local(const jy_config* engine, jy_node** out);
void jy_node_release(jy_node* node);
/* GPUs visible to this process (0 without a GPU or HIP runtime) */
int32_t jy_device_count(void);
void jy_node_destroy(jy_node* node);
/* the detail of the calling thread's last failed node call (per thread, like
 * errno: the repos call one node from their own threads) */
const char* jy_node_last_error(const jy_node* node);
uint32_t jy_node_nshards(const jy_node* node);
/* the engine of local shard `shard` (global index), NULL if not local */
jy_engine* jy_node_engine(jy_node* node, uint32_t shard);
uint32_t jy_node_shard_of(const jy_node* node, const uint8_t* key, uint64_t len);
/* register a replica identity on every local shard (the same column on all:
 * every process registers the cluster's identities in one order).  A known
 * identity is answered without waiting for the worker; a new one takes the
 * node's lock (not a fence) */
int32_t jy_node_replica_col(jy_node* node, uint64_t replica_id, uint32_t* col_out);
/* every queued job issued and its GPU work finished on every shard's streams
 * (blocks); then a queued job's failure, if any -- the streams are drained on
 * that path too, so JY_DEVICE inputs may be freed once it returns */
int32_t jy_node_sync(jy_node* node);
/* every job queued before this call issued to the GPU streams (blocks until
 * the worker took them, not for the GPU); device inputs of those calls are
 * no longer read by the host side, and the GPU reads them in stream order */
int32_t jy_node_fence(jy_node* node);
/* exclusive use of the node's engines: waits for the jobs queued before it
 * (as jy_node_fence), then holds the node's lock until jy_node_unlock.  The
 * lock is held even when an earlier job's failure is returned. */
int32_t jy_node_lock(jy_node* node);
void jy_node_unlock(jy_node* node);
/* the same, waiting only for the jobs of CRDT type `type` queued before it
 * (round 6): the types' engine states are disjoint and every engine call the
 * holder makes is ordered after the issued jobs on the engine stream, so a
 * TREG read does not wait for queued UJSON converges.  JY_NODE_NOFENCE waits
 * for no job (a read of state no converge changes: deltas_size, flush).  The
 * lock is held even when a job's failure is returned. */
#define JY_NODE_NOFENCE (-1)
int32_t jy_node_lock_type(jy_node* node, int32_t type);
/* jobs queued or running: of CRDT type `type`, or all with type < 0 */
int32_t jy_node_pending(jy_node* node, int32_t type, uint64_t* n_out);
/* the worker reclaims a shard's TREG / TLOG value arena after that type's
 * jobs once its dead bytes pass twice the live ones (+ 1 MiB): the policy the
 * Pony glue ran after every drain under the lock.  Off by default; callers
 * that pack value handles must consume them under the lock. */
int32_t jy_node_arena_gc(jy_node* node, uint32_t enable);
/* The payload schedule one shard of the exchange issues (host logic only, no
 * GPU; the node's exchange runs exactly this): for S shards, shard `rank`,
 * W count granules, nwires wire columns (granule, element bytes) and the
 * shard's per-peer element counts send_cnt / recv_cnt [S][W], the ordered
 * operations ops_out[i] = {kind (0 own part copied, 1 send, 2 receive), wire,
 * peer, source offset, destination offset, bytes}, at most cap of them;
 * *nops_out = how many there are.  Tests check it for S = 2..8 (every send
 * meets a receive of the same size, one peer order on every rank). */
int32_t jy_node_exchange_plan(uint32_t S, uint32_t rank, uint32_t W, uint32_t nwires, const int32_t* wire_gran,
                              const int32_t* wire_esize, const uint64_t* send_cnt, const uint64_t* recv_cnt,
                              uint64_t cap, uint64_t* ops_out, uint64_t* nops_out);

/* Converge one decoded peer batch (per process).  Keys: n strings (key_bytes,
 * key_offs[n + 1]).  `mem` = JY_HOST (staged per ingest shard) or JY_DEVICE
 * (readable by every local shard's GPU).  Offsets may start above 0.
 *   counters: key i's cells are [cell_offs[i], cell_offs[i+1]) of (sign 0 = P /
 *             1 = N, NULL: all P; col = jy_node_replica_col; val): s = max(s, val)
 *   TREG:     (ts[i], value bytes [val_offs[i], val_offs[i+1]))
 *   TLOG:     cutoff[i]; entries [ent_offs[i], ent_offs[i+1]) of (ts, value bytes
 *             [val_offs[e], val_offs[e+1])), canonical order (as jy_tlog_converge)
 *   UJSON:    as jy_ujson_converge, per document (dots carry node columns) */
int32_t jy_node_counter_converge(jy_node* node, int32_t type, uint64_t n, const uint8_t* key_bytes,
                                 const uint64_t* key_offs, const uint64_t* cell_offs, const uint8_t* sign,
                                 const uint16_t* col, const uint64_t* val, int32_t mem);
int32_t jy_node_treg_converge(jy_node* node, uint64_t n, const uint8_t* key_bytes, const uint64_t* key_offs,
                              const uint64_t* ts, const uint8_t* val_bytes, const uint64_t* val_offs, int32_t mem);
int32_t jy_node_tlog_converge(jy_node* node, uint64_t n, const uint8_t* key_bytes, const uint64_t* key_offs,
                              const uint64_t* cutoff, const uint64_t* ent_offs, const uint64_t* ts,
                              const uint8_t* val_bytes, const uint64_t* val_offs, int32_t mem);
int32_t jy_node_ujson_converge(jy_node* node, uint64_t n, const uint8_t* key_bytes, const uint64_t* key_offs,
                               const uint64_t* el_offs, const uint64_t* dots, const uint64_t* elems,
                               const uint64_t* vv_offs, const uint64_t* vv, const uint64_t* cloud_offs,
                               const uint64_t* cloud, int32_t mem);
/* Dense counter blocks arriving MIXED (the bench's routed PNCOUNT step, and a
 * peer that shards like this node: it flushes shard by shard).  This process
 * ingests ncols peer columns for the keys of every owner: vals_p / vals_n
 * are device arrays [ncols][S][nslots] (vals_n NULL for GCOUNT), block
 * [c][d] holding owner d's slots [slot0, slot0 + nslots).  cols_all[r * ncols
 * + c] is the column of shard r's c-th peer (every process passes the whole
 * table).  Column c of every shard crosses in one exchange; the owner merges
 * the S received columns with one block converge while column c + 1 is in
 * flight on a second stream.  Device memory only. */
int32_t jy_node_counter_converge_block(jy_node* node, int32_t type, uint32_t ncols, const uint16_t* cols_all,
                                       uint32_t slot0, uint32_t nslots, const uint64_t* vals_p,
                                       const uint64_t* vals_n);
/* telemetry of the node's last converge call (not on the reference's
 * surface): [0] keys ingested, [1] keys received, [2] bytes sent, [3] bytes
 * received (this process's local shards), [4] exchange calls so far */
int32_t jy_node_stats(jy_node* node, uint64_t* out5);

#ifdef __cplusplus
}
#endif
#endif /* JYLIS_GPU_H */
