// engine.hip -- engine lifecycle, interning, staging and the C ABI wrappers.
//
// Boundary: RepoManagerCore.converge_deltas (jylis/repo_manager.pony:92-93)
// and the per-type Repo*.converge / get entry points (repo_gcount.pony:50-55,
// repo_pncount.pony:52-57, repo_treg.pony:51-63, repo_tlog.pony:66-96,
// repo_ujson.pony:65-72).  See include/jylis_gpu.h for the contract.

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "jy_internal.hpp"
#include "jy_scan.hpp"

namespace {

u64 round_up(u64 x, u64 a) { return (x + a - 1) / a * a; }

int32_t check_type(jy_engine* eng, int32_t type) {
  if (type < 0 || type >= JY_NTYPES) return eng->fail(JY_ETYPE, "unknown CRDT type");
  return JY_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// memory helpers

// Engine buffers come from the stream-ordered allocator: growing a buffer
// never waits for queued kernels that still read the old one (they finish
// before the stream-ordered free takes effect), so the host can enqueue the
// next merge while the GPU runs the previous one.
int32_t jy_dev_alloc(jy_engine* eng, void** p, u64 bytes, const char* what) {
  hipError_t e = hipMallocFromPoolAsync(p, bytes ? bytes : 8, eng->pool, eng->stream);
  if (e != hipSuccess) {
    *p = nullptr;
    return eng->fail(JY_ENOMEM, std::string(what) + " hipMallocAsync(" + std::to_string(bytes) + "): " +
                                    hipGetErrorString(e));
  }
  return JY_OK;
}
void jy_dev_free(jy_engine* eng, void* p) {
  if (p) hipFreeAsync(p, eng->stream);
}

int32_t jy_realloc(jy_engine* eng, void** p, u64 old_bytes, u64 new_bytes, bool zero_tail) {
  if (new_bytes <= old_bytes && *p) return JY_OK;
  void* np = nullptr;
  JY_TRY(jy_dev_alloc(eng, &np, new_bytes, "realloc"));
  if (*p && old_bytes) JY_HIP(eng, hipMemcpyAsync(np, *p, old_bytes, hipMemcpyDeviceToDevice, eng->stream));
  if (zero_tail && new_bytes > old_bytes)
    JY_HIP(eng, hipMemsetAsync(static_cast<uint8_t*>(np) + old_bytes, 0, new_bytes - old_bytes, eng->stream));
  jy_dev_free(eng, *p);
  *p = np;
  return JY_OK;
}

int32_t jy_dscan_ctx(jy_engine* eng, u64 ntiles, u64** status, u32** tick, u32* epoch) {
  if (!eng->dscan_tick) {
    JY_TRY(jy_dev_alloc(eng, reinterpret_cast<void**>(&eng->dscan_tick), 64, "scan tickets"));
    JY_HIP(eng, hipMemsetAsync(eng->dscan_tick, 0, 64, eng->stream));
  }
  DevArray& a = eng->dscan_st;
  if (a.bytes < ntiles * 8) {
    const u64 nb = std::max<u64>(round_up(2 * ntiles * 8, 256), 4096);
    JY_TRY(jy_realloc(eng, &a.p, a.bytes, nb, true));
    JY_HIP(eng, hipMemsetAsync(a.p, 0, nb, eng->stream));  // old words may carry any epoch
    a.bytes = nb;
  }
  eng->dscan_epoch++;
  if ((eng->dscan_epoch & ((1u << jyscan::kEpochBits) - 1)) == 0) {  // wrap: no stale word may match
    eng->dscan_epoch = 1;
    JY_HIP(eng, hipMemsetAsync(a.p, 0, a.bytes, eng->stream));
  }
  *status = static_cast<u64*>(a.p);
  *tick = eng->dscan_tick;
  *epoch = eng->dscan_epoch;
  return JY_OK;
}

int32_t jy_scratch(jy_engine* eng, int idx, u64 bytes, void** out) {
  DevArray& a = eng->scratch[idx];
  if (a.bytes < bytes) {
    JY_TRACE("scratch %d grows %llu -> %llu", idx, (unsigned long long)a.bytes, (unsigned long long)bytes);
    // grow by at least 2x: growing states should not realloc every call
    u64 nb = std::max<u64>(round_up(std::max<u64>(bytes + bytes / 4, 2 * a.bytes), 256), 4096);
    jy_dev_free(eng, a.p);
    a.p = nullptr;
    a.bytes = 0;
    JY_TRY(jy_dev_alloc(eng, &a.p, nb, "scratch"));
    a.bytes = nb;
  }
  *out = a.p;
  return JY_OK;
}

static int32_t stage_begin(jy_engine* eng) {
  eng->pin_used = false;
  return JY_OK;
}
static int32_t stage_end(jy_engine* eng) {
  if (eng->pin_used) JY_HIP(eng, hipEventRecord(eng->pins[eng->pin_slot].ready, eng->stream));
  return JY_OK;
}

int32_t jy_stage_begin(jy_engine* eng) { return stage_begin(eng); }
int32_t jy_stage_end(jy_engine* eng) { return stage_end(eng); }

int32_t jy_stage(jy_engine* eng, int idx, const void* src, u64 bytes, int32_t mem, const void** dev_out) {
  if (mem == JY_DEVICE || bytes == 0) {
    *dev_out = src;
    if (bytes == 0 && mem != JY_DEVICE) {
      void* d;
      JY_TRY(jy_scratch(eng, idx, 8, &d));
      *dev_out = d;
    }
    return JY_OK;
  }
  if (mem != JY_HOST) return eng->fail(JY_EINVAL, "mem must be JY_HOST or JY_DEVICE");
  void* d;
  JY_TRY(jy_scratch(eng, idx, bytes, &d));
  if (!eng->pin_used) {
    // next region of the ring: its copies (kPinRing calls ago) must have drained
    eng->pin_slot = (eng->pin_slot + 1) % jy_engine::kPinRing;
    const double tw = jy_tracing() ? jy_now_us() : 0;
    JY_HIP(eng, hipEventSynchronize(eng->pins[eng->pin_slot].ready));
    if (jy_tracing() && jy_now_us() - tw > 20) JY_TRACE("pinned ring slot %d: waited %.1f us", eng->pin_slot, jy_now_us() - tw);
    eng->pin_cursor = 0;
    eng->pin_used = true;
  }
  jy_engine::PinSlot& ps = eng->pins[eng->pin_slot];
  u64 need = round_up(eng->pin_cursor, 256) + bytes;
  if (need > ps.bytes) {
    // grow this region: drain everything that may read it.  Every other
    // region of the ring that is smaller grows with it (all are idle after
    // the drain), so a larger batch shape costs one pinned allocation pause
    // (hipHostMalloc of tens of MB takes milliseconds), not one per region
    // as the ring comes round.
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    const u64 nb = std::max<u64>(need * 2, 1ull << 20);
    for (int r = 0; r < jy_engine::kPinRing; r++) {
      jy_engine::PinSlot& q = eng->pins[r];
      if (q.bytes >= nb) continue;
      void* np = nullptr;
      JY_HIP(eng, hipHostMalloc(&np, nb, hipHostMallocDefault));
      if (q.p) {
        if (r == eng->pin_slot) std::memcpy(np, q.p, eng->pin_cursor);  // earlier inputs of this call stay valid
        JY_HIP(eng, hipHostFree(q.p));
      }
      q.p = np;
      q.bytes = nb;
    }
    JY_TRACE("pinned ring grown to %llu B per region", (unsigned long long)nb);
  }
  u64 at = round_up(eng->pin_cursor, 256);
  // chunked: large copies run on the copy pool, each chunk's DMA issued as it lands
  JY_TRY(jy_copy_h2d_staged(eng, d, static_cast<uint8_t*>(ps.p) + at, src, bytes));
  eng->pin_cursor = at + bytes;
  *dev_out = d;
  return JY_OK;
}

int32_t jy_readback(jy_engine* eng, void* dst, const void* dev, u64 bytes) {
  if (bytes < (1ull << 20)) {
    JY_HIP(eng, hipMemcpyAsync(dst, dev, bytes, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    return JY_OK;
  }
  if (eng->pin_rb_bytes < bytes) {
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    if (eng->pin_rb) JY_HIP(eng, hipHostFree(eng->pin_rb));
    eng->pin_rb = nullptr;
    eng->pin_rb_bytes = 0;
    const u64 nb = std::max<u64>(bytes + bytes / 2, 4ull << 20);
    JY_HIP(eng, hipHostMalloc(&eng->pin_rb, nb, hipHostMallocDefault));
    eng->pin_rb_bytes = nb;
  }
  JY_HIP(eng, hipMemcpyAsync(eng->pin_rb, dev, bytes, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  jy_copy_host(dst, eng->pin_rb, bytes);
  return JY_OK;
}

// Device copy of a block merge's column list, cached by content (a routed
// step cycles through a few lists); a new list is uploaded asynchronously
// from a pinned copy kept with it, so no call waits for the stream.
static int32_t cols_to_device(jy_engine* eng, u32 ncols, const u16* cols, const u16** out) {
  std::vector<u16> key(cols, cols + ncols);
  auto it = eng->cols_cache.find(key);
  if (it != eng->cols_cache.end()) {
    *out = it->second.dev;
    return JY_OK;
  }
  if (eng->cols_cache.size() >= 256) {  // rare: drop the cache once its uploads and readers are done
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
    for (auto& kv : eng->cols_cache) {
      hipFree(kv.second.dev);
      hipHostFree(kv.second.pin);
    }
    eng->cols_cache.clear();
  }
  jy_engine::ColList c;
  JY_HIP(eng, hipHostMalloc(reinterpret_cast<void**>(&c.pin), std::max<u64>(ncols, 1) * 2, hipHostMallocDefault));
  std::memcpy(c.pin, cols, (u64)ncols * 2);
  if (hipMalloc(reinterpret_cast<void**>(&c.dev), std::max<u64>(ncols, 1) * 2) != hipSuccess) {
    hipHostFree(c.pin);
    return eng->fail(JY_ENOMEM, "column list allocation");
  }
  JY_HIP(eng, hipMemcpyAsync(c.dev, c.pin, (u64)ncols * 2, hipMemcpyHostToDevice, eng->stream));
  eng->cols_cache.emplace(std::move(key), c);
  *out = c.dev;
  return JY_OK;
}

int32_t jy_ensure_slots(jy_engine* eng, int32_t type, u64 n) {
  switch (type) {
    case JY_GCOUNT: return jy_counter_grow(eng, 0, 0, n);
    case JY_PNCOUNT: return jy_counter_grow(eng, 1, 0, n);
    case JY_TREG: return jy_treg_grow(eng, n);
    case JY_TLOG: return jy_tlog_grow(eng, n);
    case JY_UJSON: return jy_ujson_grow(eng, n);
  }
  return eng->fail(JY_ETYPE, "unknown CRDT type");
}

// ---------------------------------------------------------------------------
// C ABI

extern "C" {

void jy_config_default(jy_config* cfg) {
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->device = 0;
  cfg->counter_columns = 16;
  cfg->ujson_columns = 16;
  for (int t = 0; t < JY_NTYPES; t++) {
    cfg->key_capacity[t] = 1024;
    cfg->entry_capacity[t] = 8192;
    cfg->arena_capacity[t] = 1 << 16;
  }
}

int32_t jy_engine_create(const jy_config* cfg, jy_engine** out) {
  *out = nullptr;
  jy_engine* eng = new jy_engine();
  if (cfg) eng->cfg = *cfg;
  else jy_config_default(&eng->cfg);
  if (eng->cfg.counter_columns == 0) eng->cfg.counter_columns = 16;
  if (eng->cfg.ujson_columns == 0) eng->cfg.ujson_columns = 16;
  eng->device = eng->cfg.device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    // the product path has no CPU fallback: fail loudly
    delete eng;
    return JY_EHIP;
  }
  if (hipSetDevice(eng->device) != hipSuccess ||
      hipStreamCreateWithFlags(&eng->own_stream, hipStreamNonBlocking) != hipSuccess ||

      hipEventCreateWithFlags(&eng->total_ready, hipEventDisableTiming) != hipSuccess ||
      hipMalloc(&eng->skipped_dev, 8) != hipSuccess || hipMemset(eng->skipped_dev, 0, 8) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&eng->pin_total), 64, hipHostMallocDefault) != hipSuccess) {
    delete eng;
    return JY_EHIP;
  }
  eng->stream = eng->own_stream;
  {
    // The engine's own stream-ordered pool.  It keeps what it frees: with
    // the default release threshold (0) every synchronisation hands freed
    // blocks back and the next growth of a scratch array re-maps memory
    // (0.1-1 ms of host time inside a merge call, GPU idle meanwhile:
    // round-3 UJSON trace).  Being the engine's, what it keeps is not taken
    // from torch's or RCCL's allocations (the device's default pool is shared
    // by the whole process), and jy_engine_destroy returns all of it.
    hipMemPoolProps props;
    std::memset(&props, 0, sizeof(props));
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = eng->device;
    uint64_t keep = UINT64_MAX;
    if (hipMemPoolCreate(&eng->pool, &props) != hipSuccess ||
        hipMemPoolSetAttribute(eng->pool, hipMemPoolAttrReleaseThreshold, &keep) != hipSuccess) {
      std::fprintf(stderr, "jy_engine_create: hipMemPoolCreate failed\n");
      if (eng->pool) hipMemPoolDestroy(eng->pool);
      eng->pool = nullptr;
      hipStreamDestroy(eng->own_stream);
      delete eng;
      return JY_EHIP;
    }
  }
  std::memset(eng->pin_total, 0, 64);
  for (auto& ps : eng->pins) {
    if (hipEventCreateWithFlags(&ps.ready, hipEventDisableTiming) != hipSuccess) {
      jy_engine_destroy(eng);
      return JY_EHIP;
    }
    hipEventRecord(ps.ready, eng->stream);
  }
  hipEventRecord(eng->total_ready, eng->stream);
  int32_t rc = JY_OK;
  for (int t = 0; t < JY_NTYPES && rc == JY_OK; t++) rc = jy_ensure_slots(eng, t, eng->cfg.key_capacity[t]);
  if (rc == JY_OK) rc = jy_counter_grow(eng, 0, eng->cfg.counter_columns, 0);
  if (rc == JY_OK) rc = jy_counter_grow(eng, 1, eng->cfg.counter_columns, 0);
  if (rc != JY_OK) {
    std::fprintf(stderr, "jy_engine_create: %s\n", eng->err.c_str());
    jy_engine_destroy(eng);
    return rc;
  }
  hipStreamSynchronize(eng->stream);
  *out = eng;
  return JY_OK;
}

void jy_engine_destroy(jy_engine* eng) {
  if (!eng) return;
  hipSetDevice(eng->device);
  if (eng->stream) hipStreamSynchronize(eng->stream);
  auto F = [eng](void* p) { jy_dev_free(eng, p); };
  for (int w = 0; w < 2; w++) {
    F(eng->cnt[w].slab);
    F(eng->cnt[w].dflag);
    F(eng->cnt[w].dval);
    F(eng->cnt[w].dcount);
  }
  F(eng->treg.ts);
  F(eng->treg.val);
  F(eng->treg.dts);
  F(eng->treg.dval);
  F(eng->treg.dflag);
  F(eng->treg.dcount);
  F(eng->treg.seen[0]);
  F(eng->treg.seen[1]);
  F(eng->treg.dupn);
  F(eng->treg.dups);
  F(eng->treg.dupn_alt);
  F(eng->treg.dups_alt);
  F(eng->treg.fold_claim);
  for (TlogState* t : {&eng->tlog, &eng->tlog_d}) {
    F(t->meta);
    F(t->hint);
    F(t->hist);
    F(t->pool);
    F(t->ctr);
    if (t->pin) hipHostFree(t->pin);
    for (auto& sp : t->spill) {
      F(sp.buf.p);
      if (sp.done) hipEventDestroy(sp.done);
    }
  }
  F(eng->tl_dflag);
  F(eng->tl_dcount);
  for (auto& k : eng->kdir) jy_keydir_free(eng, k);
  for (UjsonState* u : {&eng->ujson, &eng->ujson_d}) {
    F(u->vv);
    F(u->meta);
    F(u->epool);
    F(u->cpool);
    F(u->spare_e);
    F(u->spare_c);
    F(u->ctr);
    F(u->dptr);
    F(u->bad);
    F(u->vvd);
    F(u->tick);
    for (auto& a : u->st) F(a.p);
    F(u->tmap.p);
    F(u->stats);
    F(u->lpe);
    F(u->lpc);
    F(u->lcol);
    F(u->lplan);
    F(u->jobs);
    F(u->fast);
    F(u->nf);
    F(u->plist);
    if (u->pin) hipHostFree(u->pin);
    for (hipEvent_t e : u->ready)
      if (e) hipEventDestroy(e);
  }
  F(eng->uj_dflag);
  F(eng->uj_dcount);
  F(eng->dscan_st.p);
  F(eng->tl_claim.p);
  F(eng->tl_bad.p);
  F(eng->kd_done);
  F(eng->dscan_tick);
  for (auto& a : eng->arena) F(a.p);
  for (auto& s : eng->scratch) F(s.p);
  if (eng->stream) hipStreamSynchronize(eng->stream);
  if (eng->skipped_dev) hipFree(eng->skipped_dev);
  for (auto& kv : eng->cols_cache) {
    hipFree(kv.second.dev);
    hipHostFree(kv.second.pin);
  }
  for (auto& ps : eng->pins) {
    if (ps.p) hipHostFree(ps.p);
    if (ps.ready) hipEventDestroy(ps.ready);
  }
  if (eng->pin_total) hipHostFree(eng->pin_total);
  if (eng->pin_rb) hipHostFree(eng->pin_rb);
  if (eng->kd_words) hipHostFree(eng->kd_words);
  if (eng->treg.dupflag) hipHostFree(eng->treg.dupflag);
  for (auto& ev : eng->tm_ev) {
    hipEventDestroy(ev.first);
    hipEventDestroy(ev.second);
  }
  if (eng->total_ready) hipEventDestroy(eng->total_ready);
  if (eng->stream) hipStreamSynchronize(eng->stream);  // the frees above have happened
  if (eng->pool) hipMemPoolDestroy(eng->pool);          // everything it kept goes back
  if (eng->own_stream) hipStreamDestroy(eng->own_stream);
  delete eng;
}

const char* jy_last_error(const jy_engine* eng) { return eng ? eng->err.c_str() : "null engine"; }

uint64_t jy_skipped(const jy_engine* eng) {
  jy_engine* e = const_cast<jy_engine*>(eng);
  u64 dev = 0;
  hipSetDevice(e->device);
  hipStreamSynchronize(e->stream);
  hipMemcpy(&dev, e->skipped_dev, 8, hipMemcpyDeviceToHost);
  return dev + e->skipped_host;
}

int32_t jy_set_stream(jy_engine* eng, void* s) {
  JY_HIP(eng, hipSetDevice(eng->device));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  eng->stream = s ? static_cast<hipStream_t>(s) : eng->own_stream;
  // events recorded on the previous stream are complete (synchronised above)
  for (auto& ps : eng->pins) JY_HIP(eng, hipEventRecord(ps.ready, eng->stream));
  JY_HIP(eng, hipEventRecord(eng->total_ready, eng->stream));
  return JY_OK;
}
void* jy_get_stream(jy_engine* eng) { return eng->stream; }

int32_t jy_sync(jy_engine* eng) {
  JY_HIP(eng, hipSetDevice(eng->device));
  JY_TRY(jy_tlog_settle(eng));  // spilled TLOG rebuilds re-merged: every converge has landed
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

int32_t jy_timing_enable(jy_engine* eng, int32_t on) {
  JY_HIP(eng, hipSetDevice(eng->device));
  eng->timing = on != 0;
  eng->tm_used = 0;
  eng->tm_depth = 0;
  return JY_OK;
}

int32_t jy_timing_read(jy_engine* eng, uint64_t cap, double* ms_out, uint64_t* n_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  const u64 n = eng->tm_used;
  for (u64 i = 0; i < n; i++) {
    JY_HIP(eng, hipEventSynchronize(eng->tm_ev[i].second));
    float ms = 0;
    JY_HIP(eng, hipEventElapsedTime(&ms, eng->tm_ev[i].first, eng->tm_ev[i].second));
    if (i < cap && ms_out) ms_out[i] = ms;
  }
  if (n_out) *n_out = n;
  eng->tm_used = 0;
  return JY_OK;
}

// ---- replicas ----
int32_t jy_replica_col(jy_engine* eng, uint64_t id, uint32_t* col) {
  auto it = eng->rep_col.find(id);
  if (it != eng->rep_col.end()) {
    *col = it->second;
    return JY_OK;
  }
  if (eng->rep_id.size() >= 0xFFFF) return eng->fail(JY_ERANGE, "more than 65535 replica identities");
  u32 c = (u32)eng->rep_id.size();
  eng->rep_id.push_back(id);
  eng->rep_col.emplace(id, c);
  *col = c;
  return JY_OK;
}
int32_t jy_replica_id(const jy_engine* eng, uint32_t col, uint64_t* id) {
  if (col >= eng->rep_id.size()) return JY_ERANGE;
  *id = eng->rep_id[col];
  return JY_OK;
}
uint32_t jy_replica_count(const jy_engine* eng) { return (uint32_t)eng->rep_id.size(); }

// ---- keys ----
// The device key directory (k_keys.hip) is authoritative; eng->keys is a
// host cache filled by small host-pointer calls.
static constexpr u64 kCacheFill = 1 << 16;  // bulk calls do not fill the cache

static int32_t keys_created(jy_engine* eng, int32_t type, u64 created) {
  if (created == 0) return JY_OK;
  const u64 before = eng->nkeys[type], nk = before + created;
  JY_TRY(jy_ensure_slots(eng, type, nk));
  if (type == JY_TLOG) JY_TRY(jy_tlog_extend(eng, before, nk));
  if (type == JY_UJSON) JY_TRY(jy_ujson_extend(eng, before, nk));
  eng->nkeys[type] = nk;
  return JY_OK;
}

// host keys: cache first, the misses go to the device directory in one call
// host batches up to this size probe the host-side slot cache first (a
// single-key GET avoids a device round trip); larger ones go straight to the
// device directory
constexpr u64 kHostProbeMax = 1024;

static int32_t keys_host(jy_engine* eng, int32_t type, u64 n, const uint8_t* kb, const u64* ko, u32* slots,
                         bool create) {
  KeyIndex& ix = eng->keys[type];
  if (n > kHostProbeMax) {
    // a decoded peer batch: every key goes to the device directory (the host
    // cache probe costs ~25 ns a key, the device probe well under 1)
    const void *db, *dofs;
    JY_TRY(stage_begin(eng));
    JY_TRY(jy_stage(eng, 0, kb, ko[n], JY_HOST, &db));
    JY_TRY(jy_stage(eng, 1, ko, (n + 1) * 8, JY_HOST, &dofs));
    JY_TRY(stage_end(eng));
    void* ds;
    JY_TRY(jy_scratch(eng, 2, n * 4, &ds));
    u64 created = 0;
    JY_TRY(jy_keydir_run(eng, type, n, static_cast<const uint8_t*>(db), static_cast<const u64*>(dofs),
                         static_cast<u32*>(ds), create, &created));
    JY_TRY(jy_readback(eng, slots, ds, n * 4));
    return keys_created(eng, type, created);
  }
  std::vector<u64> miss;
  for (u64 i = 0; i < n; i++) {
    auto it = ix.map.find(std::string(reinterpret_cast<const char*>(kb) + ko[i], ko[i + 1] - ko[i]));
    if (it != ix.map.end()) slots[i] = it->second;
    else miss.push_back(i);
  }
  if (miss.empty()) return JY_OK;
  const u64 m = miss.size();
  std::vector<u64> mo(m + 1, 0);
  for (u64 j = 0; j < m; j++) {
    const u64 len = ko[miss[j] + 1] - ko[miss[j]];
    if (len > JY_LR_LEN_MASK) return eng->fail(JY_ERANGE, "key longer than 16 MiB");
    mo[j + 1] = mo[j] + len;
  }
  std::vector<uint8_t> mb(mo[m]);
  for (u64 j = 0; j < m; j++) std::memcpy(mb.data() + mo[j], kb + ko[miss[j]], mo[j + 1] - mo[j]);
  const void* db;
  const void* dofs;
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, mb.data(), mb.size(), JY_HOST, &db));
  JY_TRY(jy_stage(eng, 1, mo.data(), (m + 1) * 8, JY_HOST, &dofs));
  JY_TRY(stage_end(eng));
  void* ds;
  JY_TRY(jy_scratch(eng, 2, m * 4, &ds));
  u64 created = 0;
  JY_TRY(jy_keydir_run(eng, type, m, static_cast<const uint8_t*>(db), static_cast<const u64*>(dofs),
                       static_cast<u32*>(ds), create, &created));
  std::vector<u32> ms(m);
  JY_HIP(eng, hipMemcpyAsync(ms.data(), ds, m * 4, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  JY_TRY(keys_created(eng, type, created));
  const bool fill = m <= kCacheFill;
  for (u64 j = 0; j < m; j++) {
    slots[miss[j]] = ms[j];
    if (fill && ms[j] != JY_NO_SLOT)
      ix.map.emplace(std::string(reinterpret_cast<const char*>(mb.data()) + mo[j], mo[j + 1] - mo[j]), ms[j]);
  }
  return JY_OK;
}

// device keys interned (create on miss), with the directory's hook: `after`
// runs once the probe is enqueued, before the host waits for its counts (the
// node's one-shard path enqueues its long values there)
}  // extern "C"
int32_t jy_keys_intern_dev(jy_engine* eng, int32_t type, u64 n, const uint8_t* kb, const u64* ko, u32* slots,
                           int32_t (*after)(void*), void* arg, u64* created_out) {
  JY_TRY(check_type(eng, type));
  JY_HIP(eng, hipSetDevice(eng->device));
  u64 created = 0;
  JY_TRY(jy_keydir_run(eng, type, n, kb, ko, slots, true, &created, after, arg));
  if (created_out) *created_out = created;
  return keys_created(eng, type, created);
}
extern "C" {

int32_t jy_keys_intern(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* kb, const uint64_t* ko,
                       uint32_t* slots) {
  return jy_keys_intern_mem(eng, type, n, kb, ko, slots, JY_HOST);
}

int32_t jy_keys_lookup(const jy_engine* eng, int32_t type, uint64_t n, const uint8_t* kb, const uint64_t* ko,
                       uint32_t* slots) {
  return jy_keys_lookup_mem(const_cast<jy_engine*>(eng), type, n, kb, ko, slots, JY_HOST);
}

int32_t jy_keys_intern_mem(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* kb, const uint64_t* ko,
                           uint32_t* slots, int32_t mem) {
  JY_TRY(check_type(eng, type));
  JY_HIP(eng, hipSetDevice(eng->device));
  if (mem == JY_HOST) return keys_host(eng, type, n, kb, ko, slots, true);
  if (mem != JY_DEVICE) return eng->fail(JY_EINVAL, "mem must be JY_HOST or JY_DEVICE");
  u64 created = 0;
  JY_TRY(jy_keydir_run(eng, type, n, kb, reinterpret_cast<const u64*>(ko), slots, true, &created));
  return keys_created(eng, type, created);
}

int32_t jy_keys_lookup_mem(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* kb, const uint64_t* ko,
                           uint32_t* slots, int32_t mem) {
  JY_TRY(check_type(eng, type));
  JY_HIP(eng, hipSetDevice(eng->device));
  if (mem == JY_HOST) return keys_host(eng, type, n, kb, ko, slots, false);
  if (mem != JY_DEVICE) return eng->fail(JY_EINVAL, "mem must be JY_HOST or JY_DEVICE");
  u64 created = 0;
  return jy_keydir_run(eng, type, n, kb, reinterpret_cast<const u64*>(ko), slots, false, &created);
}

uint64_t jy_keys_count(const jy_engine* eng, int32_t type) {
  return (type < 0 || type >= JY_NTYPES) ? 0 : eng->nkeys[type];
}

int32_t jy_keys_reserve(jy_engine* eng, int32_t type, uint64_t cap) {
  JY_TRY(check_type(eng, type));
  JY_HIP(eng, hipSetDevice(eng->device));
  JY_TRY(jy_keydir_reserve(eng, type, cap));
  return jy_ensure_slots(eng, type, cap);
}

// Owner shard: FNV-1a 64 over the key bytes, splitmix64 finaliser, mod S.
uint32_t jy_key_owner(const uint8_t* key, uint64_t len, uint32_t nshards) {
  u64 h = 0xCBF29CE484222325ull;
  for (u64 i = 0; i < len; i++) {
    h ^= key[i];
    h *= 0x100000001B3ull;
  }
  h ^= h >> 30;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 27;
  h *= 0x94D049BB133111EBull;
  h ^= h >> 31;
  return nshards ? (uint32_t)(h % nshards) : 0;
}

// ---- string values ----
int32_t jy_values_pack(jy_engine* eng, int32_t type, uint64_t n, const uint8_t* bytes, const uint64_t* offs,
                       uint64_t* pre, uint64_t* lr) {
  JY_TRY(check_type(eng, type));
  JY_HIP(eng, hipSetDevice(eng->device));
  Arena& a = eng->arena[type];
  // long values start on kArenaAlign granules (jy_arena_collect relies on it)
  const u64 base = round_up(a.len, kArenaAlign);
  u64 add = base - a.len;
  for (u64 i = 0; i < n; i++) {
    u64 len = offs[i + 1] - offs[i];
    if (len > JY_MAX_VALUE_LEN) return eng->fail(JY_ERANGE, "value longer than 16 MiB");
    if (len > 8) add += round_up(len, kArenaAlign);
  }
  if (a.len + add > a.cap) {
    u64 nc = std::max<u64>(std::max<u64>(a.cap * 2, a.len + add), 1 << 16);
    void* p = a.p;
    JY_TRY(jy_realloc(eng, &p, a.len, nc, false));
    a.p = static_cast<uint8_t*>(p);
    a.cap = nc;
  }
  if ((a.len + add) >> (64 - JY_LR_LEN_BITS)) return eng->fail(JY_ERANGE, "arena offset overflow");
  std::vector<uint8_t> tail(base - a.len, 0);
  tail.reserve(add);
  u64 at = base;
  for (u64 i = 0; i < n; i++) {
    const uint8_t* v = bytes + offs[i];
    u64 len = offs[i + 1] - offs[i];
    u64 p = 0;
    for (u64 j = 0; j < 8; j++) p = (p << 8) | (j < len ? v[j] : 0);
    pre[i] = p;
    if (len > 8) {
      lr[i] = (at << JY_LR_LEN_BITS) | len;
      tail.insert(tail.end(), v, v + len);
      tail.resize(tail.size() + (round_up(len, kArenaAlign) - len), 0);
      at += round_up(len, kArenaAlign);
    } else {
      lr[i] = len;
    }
  }
  if (add) {
    JY_TRY(stage_begin(eng));
    const void* d;
    // stage through pinned memory, then device-to-device into the arena
    JY_TRY(jy_stage(eng, 7, tail.data(), add, JY_HOST, &d));
    JY_HIP(eng, hipMemcpyAsync(a.p + a.len, d, add, hipMemcpyDeviceToDevice, eng->stream));
    JY_TRY(stage_end(eng));
  }
  a.len += add;
  return JY_OK;
}

int32_t jy_arena_read(jy_engine* eng, int32_t type, uint64_t off, uint64_t len, uint8_t* dst) {
  JY_TRY(check_type(eng, type));
  JY_HIP(eng, hipSetDevice(eng->device));
  if (off + len > eng->arena[type].len) return eng->fail(JY_ERANGE, "arena read out of range");
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  JY_HIP(eng, hipMemcpy(dst, eng->arena[type].p + off, len, hipMemcpyDeviceToHost));
  return JY_OK;
}

// ---- counters ----
static int32_t counter_cols_check(jy_engine* eng, int which, u64 n, const u16* col, int32_t mem) {
  // columns must name known replicas; grow the slab's column capacity
  u32 nrep = (u32)eng->rep_id.size();
  if (mem == JY_HOST) {
    for (u64 i = 0; i < n; i++)
      if (col[i] >= nrep) return eng->fail(JY_ERANGE, "column names no registered replica");
  }
  return jy_counter_grow(eng, which, nrep, 0);
}

static int32_t slots_check(jy_engine* eng, int32_t type, u64 n, const u32* slot, int32_t mem) {
  if (mem != JY_HOST) return JY_OK;
  u64 nk = eng->nkeys[type];
  for (u64 i = 0; i < n; i++)
    if (slot[i] >= nk) return eng->fail(JY_ERANGE, "slot was never interned");
  return JY_OK;
}

int32_t jy_gcount_converge(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint16_t* col,
                           const uint64_t* val, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  JY_TRY(slots_check(eng, JY_GCOUNT, n, slot, mem));
  JY_TRY(counter_cols_check(eng, 0, n, col, mem));
  const void *ds, *dc, *dv;
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slot, n * 4, mem, &ds));
  JY_TRY(jy_stage(eng, 1, col, n * 2, mem, &dc));
  JY_TRY(jy_stage(eng, 2, val, n * 8, mem, &dv));
  JY_TRY(stage_end(eng));
  return jy_counter_coo(eng, 0, 0, n, (const u32*)ds, (const u16*)dc, (const u64*)dv);
}

// one decoded peer batch with its key strings: device interning (_data_for,
// create on miss) feeding the COO merge directly -- the slots never cross to
// the host.  Everything is staged in one pinned region first (one run of
// DMAs), then the directory runs, then the cells merge.
int32_t jy_counter_converge_keys(jy_engine* eng, int32_t type, uint64_t nkeys, const uint8_t* kb, const uint64_t* ko,
                                 uint64_t ncells, const uint32_t* cell_key, const uint8_t* sign, const uint16_t* col,
                                 const uint64_t* val, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type != JY_GCOUNT && type != JY_PNCOUNT) return eng->fail(JY_EINVAL, "type must be JY_GCOUNT or JY_PNCOUNT");
  if (mem != JY_HOST && mem != JY_DEVICE) return eng->fail(JY_EINVAL, "mem must be JY_HOST or JY_DEVICE");
  if (!cell_key && ncells != nkeys) return eng->fail(JY_EINVAL, "without cell_key, cell i is key i: ncells == nkeys");
  if (type == JY_GCOUNT && sign) return eng->fail(JY_EINVAL, "GCOUNT cells have no sign");
  if (nkeys == 0) return JY_OK;
  if (ncells == 0) {
    // keys with no cells are still created (_data_for, repo_gcount.pony:36-41)
    if (mem == JY_DEVICE) {
      void* ds;
      JY_TRY(jy_scratch(eng, 2, nkeys * 4, &ds));
      return jy_keys_intern_mem(eng, type, nkeys, kb, ko, static_cast<u32*>(ds), JY_DEVICE);
    }
    std::vector<u32> slots(nkeys);
    return jy_keys_intern_mem(eng, type, nkeys, kb, ko, slots.data(), JY_HOST);
  }
  const int which = type == JY_GCOUNT ? 0 : 1;
  if (mem == JY_HOST) {
    if (cell_key)
      for (u64 i = 0; i < ncells; i++)
        if (cell_key[i] >= nkeys) return eng->fail(JY_ERANGE, "cell_key names no key of the batch");
    if (sign)
      for (u64 i = 0; i < ncells; i++)
        if (sign[i] > 1) return eng->fail(JY_ERANGE, "sign must be 0 (P) or 1 (N)");
  }
  JY_TRY(counter_cols_check(eng, which, ncells, col, mem));
  const double t0 = jy_tracing() ? jy_now_us() : 0;
  // the keys first: the directory's probe starts once they are up, and the
  // cells are staged (host copies, their DMAs) while it runs
  const void *db, *dofs;
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, kb, mem == JY_HOST ? ko[nkeys] : 0, mem, &db));  // device: used in place
  JY_TRY(jy_stage(eng, 1, ko, (nkeys + 1) * 8, mem, &dofs));
  JY_TRY(stage_end(eng));
  struct Cells {
    jy_engine* eng;
    u64 n;
    const void *key, *sign, *col, *val;
    int32_t mem;
    const void *dk = nullptr, *dsg = nullptr, *dc = nullptr, *dv = nullptr;
  } C{eng, ncells, cell_key, sign, col, val, mem};
  auto stage_cells = [](void* p) -> int32_t {
    Cells& c = *static_cast<Cells*>(p);
    JY_TRY(stage_begin(c.eng));
    if (c.key) JY_TRY(jy_stage(c.eng, 3, c.key, c.n * 4, c.mem, &c.dk));
    if (c.sign) JY_TRY(jy_stage(c.eng, 4, c.sign, c.n, c.mem, &c.dsg));
    JY_TRY(jy_stage(c.eng, 5, c.col, c.n * 2, c.mem, &c.dc));
    JY_TRY(jy_stage(c.eng, 6, c.val, c.n * 8, c.mem, &c.dv));
    return stage_end(c.eng);
  };
  void* ds;
  JY_TRY(jy_scratch(eng, 2, nkeys * 4, &ds));
  u64 created = 0;
  const double t1 = jy_tracing() ? jy_now_us() : 0;
  JY_TRY(jy_keydir_run(eng, type, nkeys, static_cast<const uint8_t*>(db), static_cast<const u64*>(dofs),
                       static_cast<u32*>(ds), true, &created, stage_cells, &C));
  const void *dk = C.dk, *dsg = C.dsg, *dc = C.dc, *dv = C.dv;
  const double t2 = jy_tracing() ? jy_now_us() : 0;
  JY_TRY(keys_created(eng, type, created));  // grows the slabs before the merge is enqueued
  JY_TRACE("converge_keys: staging %.1f us, directory %.1f us, %llu created", t1 - t0, t2 - t1,
           (unsigned long long)created);
  JY_TRACE("converge_keys: %llu keys, %llu cells: %.1f us after the host checks", (unsigned long long)nkeys,
           (unsigned long long)ncells, jy_now_us() - t0);
  return jy_counter_coo_keyed(eng, which, ncells, nkeys, static_cast<const u32*>(ds), static_cast<const u32*>(dk),
                              static_cast<const uint8_t*>(dsg), static_cast<const u16*>(dc),
                              static_cast<const u64*>(dv));
}

int32_t jy_gcount_converge_block(jy_engine* eng, uint32_t ncols, const uint16_t* cols, uint32_t slot0,
                                 uint32_t nslots, const uint64_t* vals, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (ncols == 0 || nslots == 0) return JY_OK;
  if ((u64)slot0 + nslots > eng->nkeys[JY_GCOUNT]) return eng->fail(JY_ERANGE, "slot run was never interned");
  JY_TRY(counter_cols_check(eng, 0, ncols, cols, JY_HOST));
  const void* dv;
  const u16* dc;
  JY_TRY(cols_to_device(eng, ncols, cols, &dc));
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 2, vals, (u64)ncols * nslots * 8, mem, &dv));
  JY_TRY(stage_end(eng));
  return jy_counter_block(eng, 0, ncols, dc, slot0, nslots, (const u64*)dv, nullptr);
}

static int32_t counter_get(jy_engine* eng, int which, int32_t type, uint64_t n, const uint32_t* slots,
                           uint64_t* out, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  const void* ds;
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slots, n * 4, mem, &ds));
  JY_TRY(stage_end(eng));
  u64* dout = out;
  if (mem == JY_HOST) {
    void* p;
    JY_TRY(jy_scratch(eng, 3, n * 8, &p));
    dout = static_cast<u64*>(p);
  }
  JY_TRY(jy_counter_sum(eng, which, n, (const u32*)ds, dout));
  if (mem == JY_HOST) {
    JY_TRY(jy_readback(eng, out, dout, n * 8));
  }
  (void)type;
  return JY_OK;
}

int32_t jy_gcount_get(jy_engine* eng, uint64_t n, const uint32_t* slots, uint64_t* out, int32_t mem) {
  return counter_get(eng, 0, JY_GCOUNT, n, slots, out, mem);
}

int32_t jy_pncount_converge(jy_engine* eng, uint64_t np, const uint32_t* pslot, const uint16_t* pcol,
                            const uint64_t* pval, uint64_t nn, const uint32_t* nslot, const uint16_t* ncol,
                            const uint64_t* nval, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  JY_TRY(slots_check(eng, JY_PNCOUNT, np, pslot, mem));
  JY_TRY(slots_check(eng, JY_PNCOUNT, nn, nslot, mem));
  JY_TRY(counter_cols_check(eng, 1, np, pcol, mem));
  JY_TRY(counter_cols_check(eng, 1, nn, ncol, mem));
  if (np) {
    const void *ds, *dc, *dv;
    JY_TRY(stage_begin(eng));
    JY_TRY(jy_stage(eng, 0, pslot, np * 4, mem, &ds));
    JY_TRY(jy_stage(eng, 1, pcol, np * 2, mem, &dc));
    JY_TRY(jy_stage(eng, 2, pval, np * 8, mem, &dv));
    JY_TRY(stage_end(eng));
    JY_TRY(jy_counter_coo(eng, 1, 0, np, (const u32*)ds, (const u16*)dc, (const u64*)dv));
  }
  if (nn) {
    const void *ds, *dc, *dv;
    JY_TRY(stage_begin(eng));
    JY_TRY(jy_stage(eng, 4, nslot, nn * 4, mem, &ds));
    JY_TRY(jy_stage(eng, 5, ncol, nn * 2, mem, &dc));
    JY_TRY(jy_stage(eng, 6, nval, nn * 8, mem, &dv));
    JY_TRY(stage_end(eng));
    JY_TRY(jy_counter_coo(eng, 1, 1, nn, (const u32*)ds, (const u16*)dc, (const u64*)dv));
  }
  return JY_OK;
}

int32_t jy_pncount_converge_block(jy_engine* eng, uint32_t ncols, const uint16_t* cols, uint32_t slot0,
                                  uint32_t nslots, const uint64_t* vp, const uint64_t* vn, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (ncols == 0 || nslots == 0) return JY_OK;
  if ((u64)slot0 + nslots > eng->nkeys[JY_PNCOUNT]) return eng->fail(JY_ERANGE, "slot run was never interned");
  JY_TRY(counter_cols_check(eng, 1, ncols, cols, JY_HOST));
  const void *dp, *dn;
  const u16* dc;
  JY_TRY(cols_to_device(eng, ncols, cols, &dc));
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 2, vp, (u64)ncols * nslots * 8, mem, &dp));
  JY_TRY(jy_stage(eng, 6, vn, (u64)ncols * nslots * 8, mem, &dn));
  JY_TRY(stage_end(eng));
  return jy_counter_block(eng, 1, ncols, dc, slot0, nslots, (const u64*)dp, (const u64*)dn);
}

int32_t jy_pncount_get(jy_engine* eng, uint64_t n, const uint32_t* slots, int64_t* out, int32_t mem) {
  return counter_get(eng, 1, JY_PNCOUNT, n, slots, reinterpret_cast<uint64_t*>(out), mem);
}

int32_t jy_counter_export(jy_engine* eng, int32_t type, uint32_t ncols, uint32_t slot0, uint32_t nslots,
                          uint64_t* out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type != JY_GCOUNT && type != JY_PNCOUNT) return eng->fail(JY_ETYPE, "not a counter type");
  int w = type == JY_GCOUNT ? 0 : 1;
  CounterState& c = eng->cnt[w];
  if (ncols > c.ccap || (u64)slot0 + nslots > c.kcap) return eng->fail(JY_ERANGE, "export out of range");
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  int nsigns = w + 1;
  for (int s = 0; s < nsigns; s++)
    for (u32 col = 0; col < ncols; col++) {
      const u64* src = c.slab + ((u64)s * c.ccap + col) * c.kcap + slot0;
      JY_HIP(eng, hipMemcpy(out + ((u64)s * ncols + col) * nslots, src, (u64)nslots * 8, hipMemcpyDeviceToHost));
    }
  return JY_OK;
}

// ---- counter write path + flush_deltas ----
int32_t jy_counter_write(jy_engine* eng, int32_t type, int32_t sign, uint32_t col, uint64_t n, const uint32_t* slot,
                         const uint64_t* val, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type != JY_GCOUNT && type != JY_PNCOUNT) return eng->fail(JY_ETYPE, "not a counter type");
  const int w = type == JY_GCOUNT ? 0 : 1;
  if (sign < 0 || sign > w) return eng->fail(JY_EINVAL, "sign must be 0 (INC) or, for PNCOUNT, 1 (DEC)");
  if (col >= eng->rep_id.size()) return eng->fail(JY_ERANGE, "column names no registered replica");
  if (n == 0) return JY_OK;
  JY_TRY(slots_check(eng, type, n, slot, mem));
  JY_TRY(jy_counter_grow(eng, w, (u32)eng->rep_id.size(), eng->nkeys[type]));
  const void *ds, *dv;
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slot, n * 4, mem, &ds));
  JY_TRY(jy_stage(eng, 2, val, n * 8, mem, &dv));
  JY_TRY(stage_end(eng));
  return jy_cnt_write(eng, w, sign, (u16)col, n, (const u32*)ds, (const u64*)dv);
}

int32_t jy_counter_deltas_size(jy_engine* eng, int32_t type, uint64_t* n_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type != JY_GCOUNT && type != JY_PNCOUNT) return eng->fail(JY_ETYPE, "not a counter type");
  return jy_cnt_pending(eng, type == JY_GCOUNT ? 0 : 1, n_out);
}

int32_t jy_counter_flush(jy_engine* eng, int32_t type, uint64_t cap, uint32_t* slot_out, uint64_t* vals_out,
                         uint32_t* mask_out, uint64_t* n_out, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (type != JY_GCOUNT && type != JY_PNCOUNT) return eng->fail(JY_ETYPE, "not a counter type");
  const int w = type == JY_GCOUNT ? 0 : 1;
  const u64 nsigns = w + 1;
  u32 *ds = slot_out, *dm = mask_out;
  u64* dv = vals_out;
  u64 pending = 0;
  JY_TRY(jy_cnt_pending(eng, w, &pending));
  if (pending > cap) {
    *n_out = pending;
    return eng->fail(JY_ERANGE, "flush output capacity is smaller than the pending delta count");
  }
  if (mem == JY_HOST && pending) {  // device temporaries sized to the pending count, copied back
    void *a, *b, *c;
    JY_TRY(jy_scratch(eng, 8, pending * 4, &a));
    JY_TRY(jy_scratch(eng, 9, pending * 8 * nsigns, &b));
    JY_TRY(jy_scratch(eng, 10, pending * 4, &c));
    ds = static_cast<u32*>(a);
    dv = static_cast<u64*>(b);
    dm = static_cast<u32*>(c);
  }
  u64 cnt = 0;
  const u64 dcap = mem == JY_HOST ? pending : cap;
  JY_TRY(jy_cnt_flush(eng, w, eng->nkeys[type], dcap, ds, dv, dm, &cnt));
  *n_out = cnt;
  if (mem == JY_HOST && cnt) {
    JY_HIP(eng, hipMemcpyAsync(slot_out, ds, cnt * 4, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(mask_out, dm, cnt * 4, hipMemcpyDeviceToHost, eng->stream));
    for (u64 g = 0; g < nsigns; g++)
      JY_HIP(eng, hipMemcpyAsync(vals_out + g * cap, dv + g * dcap, cnt * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
  }
  return JY_OK;
}

// ---- TREG ----
// A key repeated inside one call (host or device memory) is exact: the
// device folds the repeats in after the wide merge (k_treg.hip), and LWW
// is a join, so SET batches and converges need no host-side rounds.
static int32_t treg_handles_check(jy_engine* eng, u64 n, const u64* lr) {
  const u64 alen = eng->arena[JY_TREG].len;
  for (u64 i = 0; i < n; i++)
    if ((lr[i] & JY_LR_LEN_MASK) > 8 && (lr[i] >> JY_LR_LEN_BITS) + (lr[i] & JY_LR_LEN_MASK) > alen)
      return eng->fail(JY_ERANGE, "value handle outside the arena");
  return JY_OK;
}

static int32_t treg_stage(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint64_t* ts, const uint64_t* pre,
                          const uint64_t* lr, int32_t mem, const void** ds, const void** dt, const void** dp,
                          const void** dl) {
  JY_TRY(slots_check(eng, JY_TREG, n, slot, mem));
  if (mem == JY_HOST) JY_TRY(treg_handles_check(eng, n, lr));
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slot, n * 4, mem, ds));
  JY_TRY(jy_stage(eng, 1, ts, n * 8, mem, dt));
  JY_TRY(jy_stage(eng, 2, pre, n * 8, mem, dp));
  JY_TRY(jy_stage(eng, 3, lr, n * 8, mem, dl));
  return stage_end(eng);
}

int32_t jy_treg_converge(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint64_t* ts, const uint64_t* pre,
                         const uint64_t* lr, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  if (n >= 0xFFFFFFFFull) return eng->fail(JY_ERANGE, "more than 2^32 - 1 entries in one call");
  const void *ds, *dt, *dp, *dl;
  JY_TRY(treg_stage(eng, n, slot, ts, pre, lr, mem, &ds, &dt, &dp, &dl));
  return jy_treg_merge(eng, n, (const u32*)ds, (const u64*)dt, (const u64*)dp, (const u64*)dl);
}

// a block batch: entry i is the delta of slot slot0 + i (no slot stream)
int32_t jy_treg_converge_block(jy_engine* eng, uint32_t slot0, uint64_t n, const uint64_t* ts, const uint64_t* pre,
                               const uint64_t* lr, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  if ((u64)slot0 + n > eng->nkeys[JY_TREG]) return eng->fail(JY_ERANGE, "slot run was never interned");
  if (mem == JY_HOST) JY_TRY(treg_handles_check(eng, n, lr));
  const void *dt, *dp, *dl;
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 1, ts, n * 8, mem, &dt));
  JY_TRY(jy_stage(eng, 2, pre, n * 8, mem, &dp));
  JY_TRY(jy_stage(eng, 3, lr, n * 8, mem, &dl));
  JY_TRY(stage_end(eng));
  return jy_treg_merge_block(eng, slot0, n, (const u64*)dt, (const u64*)dp, (const u64*)dl);
}

// local SET batch (RepoTREG.set repo_treg.pony:65-68): the state merge and
// the pending delta in one pass (k_treg.hip set_one)
int32_t jy_treg_set(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint64_t* ts, const uint64_t* pre,
                    const uint64_t* lr, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  if (n >= 0xFFFFFFFFull) return eng->fail(JY_ERANGE, "more than 2^32 - 1 entries in one call");
  const void *ds, *dt, *dp, *dl;
  JY_TRY(treg_stage(eng, n, slot, ts, pre, lr, mem, &ds, &dt, &dp, &dl));
  return jy_treg_set_batch(eng, n, (const u32*)ds, (const u64*)dt, (const u64*)dp, (const u64*)dl);
}

int32_t jy_treg_deltas_size(jy_engine* eng, uint64_t* n_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  return jy_treg_pending(eng, n_out);
}

int32_t jy_treg_flush(jy_engine* eng, uint64_t cap, uint32_t* slot_out, uint64_t* ts_out, uint64_t* pre_out,
                      uint64_t* lr_out, uint64_t* n_out, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  u64 pending = 0;
  JY_TRY(jy_treg_pending(eng, &pending));
  if (pending > cap) {
    *n_out = pending;
    return eng->fail(JY_ERANGE, "flush output capacity is smaller than the pending delta count");
  }
  u32* ds = slot_out;
  u64 *dt = ts_out, *dp = pre_out, *dl = lr_out;
  if (mem == JY_HOST && pending) {
    void *a, *b, *c, *d;
    JY_TRY(jy_scratch(eng, 8, pending * 4, &a));
    JY_TRY(jy_scratch(eng, 9, pending * 8, &b));
    JY_TRY(jy_scratch(eng, 10, pending * 8, &c));
    JY_TRY(jy_scratch(eng, 11, pending * 8, &d));
    ds = static_cast<u32*>(a);
    dt = static_cast<u64*>(b);
    dp = static_cast<u64*>(c);
    dl = static_cast<u64*>(d);
  }
  u64 cnt = 0;
  JY_TRY(jy_treg_flush_dev(eng, eng->nkeys[JY_TREG], mem == JY_HOST ? pending : cap, ds, dt, dp, dl, &cnt));
  *n_out = cnt;
  if (mem == JY_HOST && cnt) {
    JY_HIP(eng, hipMemcpyAsync(slot_out, ds, cnt * 4, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(ts_out, dt, cnt * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(pre_out, dp, cnt * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(lr_out, dl, cnt * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipStreamSynchronize(eng->stream));
  }
  return JY_OK;
}

int32_t jy_treg_read(jy_engine* eng, uint64_t n, const uint32_t* slots, uint64_t* ts, uint64_t* pre,
                     uint64_t* lr) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  JY_TRY(slots_check(eng, JY_TREG, n, slots, JY_HOST));
  const void* ds;
  JY_TRY(stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slots, n * 4, JY_HOST, &ds));
  JY_TRY(stage_end(eng));
  void* o;
  JY_TRY(jy_scratch(eng, 1, n * 24, &o));
  u64* d = static_cast<u64*>(o);
  JY_TRY(jy_treg_gather(eng, n, (const u32*)ds, d, d + n, d + 2 * n));
  JY_HIP(eng, hipMemcpyAsync(ts, d, n * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(pre, d + n, n * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(lr, d + 2 * n, n * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  // every launch before this read has finished: an overflow of the
  // duplicate list fails the read (the outputs are written, but may miss an
  // update that was dropped)
  return jy_treg_overflow_check(eng);
}

}  // extern "C"

int32_t jy_slots_check(jy_engine* eng, int32_t type, u64 n, const u32* slot, int32_t mem) {
  return slots_check(eng, type, n, slot, mem);
}
