// abi_logs.hip -- C ABI of the variable-length types: TLOG and UJSON.
//
// Boundary: RepoTLOG.converge (jylis/repo_tlog.pony:66-67) and reads
// (get/size/cutoff :69-96); RepoUJSON.converge (repo_ujson.pony:65-66) and
// get (:68-72).  Host-pointer calls validate the CSR shape and split keys
// that repeat inside one call into rounds (one delta per key per merge,
// as the sender's `_deltas` Map guarantees).

#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "jy_internal.hpp"

namespace {

bool csr_ok(const u64* offs, u64 n, u64 total) {
  if (offs[0] != 0 || offs[n] != total) return false;
  for (u64 i = 0; i < n; i++)
    if (offs[i] > offs[i + 1]) return false;
  return true;
}

// occurrence index of each slot inside the call; returns the number of rounds
// (a hash set sized to the call, not to the interned keys: the host mirror
// makes many one-key calls)
u32 rounds_of(u64 n, const u32* slot, std::vector<u32>& occ) {
  {
    std::unordered_set<u32> mark;
    mark.reserve(n * 2);
    bool dup = false;
    for (u64 i = 0; i < n && !dup; i++) dup = !mark.insert(slot[i]).second;
    if (!dup) return 1;
  }
  std::unordered_map<u32, u32> seen;
  occ.resize(n);
  u32 rounds = 1;
  for (u64 i = 0; i < n; i++) {
    occ[i] = seen[slot[i]]++;
    rounds = std::max(rounds, occ[i] + 1);
  }
  return rounds;
}

// gather the CSR segments of rows `idx` of (offs, cols...) into fresh arrays
struct CsrPick {
  std::vector<u64> offs;
  std::vector<std::vector<u64>> cols;
};
CsrPick pick(const std::vector<u64>& idx, const u64* offs, std::initializer_list<const u64*> cols) {
  CsrPick p;
  p.offs.push_back(0);
  p.cols.resize(cols.size());
  for (u64 i : idx) {
    size_t c = 0;
    for (const u64* col : cols) {
      p.cols[c].insert(p.cols[c].end(), col + offs[i], col + offs[i + 1]);
      c++;
    }
    p.offs.push_back(p.offs.back() + (offs[i + 1] - offs[i]));
  }
  return p;
}

}  // namespace

extern "C" {

int32_t jy_tlog_converge(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint64_t* cutoff,
                         const uint64_t* offs, uint64_t nent, const uint64_t* ts, const uint64_t* pre,
                         const uint64_t* lr, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  JY_TRY(jy_slots_check(eng, JY_TLOG, n, slot, mem));
  if (mem == JY_HOST) {
    if (!csr_ok(offs, n, nent)) return eng->fail(JY_EINVAL, "entry offsets are not a CSR of nent entries");
    const u64 alen = eng->arena[JY_TLOG].len;
    for (u64 j = 0; j < nent; j++)
      if ((lr[j] & JY_LR_LEN_MASK) > 8 && (lr[j] >> JY_LR_LEN_BITS) + (lr[j] & JY_LR_LEN_MASK) > alen)
        return eng->fail(JY_ERANGE, "value handle outside the arena");
    std::vector<u32> occ;
    const u32 rounds = rounds_of(n, slot, occ);
    if (rounds > 1) {
      for (u32 r = 0; r < rounds; r++) {
        std::vector<u64> idx;
        for (u64 i = 0; i < n; i++)
          if (occ[i] == r) idx.push_back(i);
        std::vector<u32> s;
        std::vector<u64> c;
        for (u64 i : idx) {
          s.push_back(slot[i]);
          c.push_back(cutoff[i]);
        }
        CsrPick p = pick(idx, offs, {ts, pre, lr});
        JY_TRY(jy_tlog_converge(eng, s.size(), s.data(), c.data(), p.offs.data(), p.offs.back(), p.cols[0].data(),
                                p.cols[1].data(), p.cols[2].data(), JY_HOST));
      }
      return JY_OK;
    }
  }
  const void *ds, *dc, *doff, *dt, *dp, *dl;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slot, n * 4, mem, &ds));
  JY_TRY(jy_stage(eng, 1, cutoff, n * 8, mem, &dc));
  JY_TRY(jy_stage(eng, 2, offs, (n + 1) * 8, mem, &doff));
  JY_TRY(jy_stage(eng, 3, ts, nent * 8, mem, &dt));
  JY_TRY(jy_stage(eng, 4, pre, nent * 8, mem, &dp));
  JY_TRY(jy_stage(eng, 5, lr, nent * 8, mem, &dl));
  JY_TRY(jy_stage_end(eng));
  return jy_tlog_merge(eng, n, (const u32*)ds, (const u64*)dc, (const u64*)doff, nent, (const u64*)dt,
                       (const u64*)dp, (const u64*)dl);
}

int32_t jy_tlog_write(jy_engine* eng, uint64_t n, const uint8_t* op, const uint32_t* slot, const uint64_t* ts,
                      const uint64_t* arg, const uint64_t* pre, const uint64_t* lr, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  if (n >= 0xFFFFFFFFull) return eng->fail(JY_ERANGE, "more than 2^32 - 1 commands in one call");
  JY_TRY(jy_slots_check(eng, JY_TLOG, n, slot, mem));
  if (mem == JY_HOST) {
    const u64 alen = eng->arena[JY_TLOG].len;
    for (u64 i = 0; i < n; i++) {
      if (op[i] > JY_TLOG_CLR) return eng->fail(JY_EINVAL, "unknown TLOG write op");
      if (op[i] == JY_TLOG_INS && (!ts || !pre || !lr)) return eng->fail(JY_EINVAL, "INS needs ts, pre and lr");
      if ((op[i] == JY_TLOG_TRIMAT && !ts) || (op[i] == JY_TLOG_TRIM && !arg))
        return eng->fail(JY_EINVAL, "TRIMAT needs ts, TRIM needs arg");
      if (op[i] == JY_TLOG_INS && (lr[i] & JY_LR_LEN_MASK) > 8 &&
          (lr[i] >> JY_LR_LEN_BITS) + (lr[i] & JY_LR_LEN_MASK) > alen)
        return eng->fail(JY_ERANGE, "value handle outside the arena");
    }
    std::vector<u32> occ;
    const u32 rounds = rounds_of(n, slot, occ);
    // full columns (zeros where a command does not use one)
    std::vector<u64> cts(n, 0), carg(n, 0), cpre(n, 0), clr(n, 0);
    for (u64 i = 0; i < n; i++) {
      if (ts) cts[i] = ts[i];
      if (arg) carg[i] = arg[i];
      if (pre) cpre[i] = pre[i];
      if (lr) clr[i] = lr[i];
    }
    for (u32 r = 0; r < rounds; r++) {
      std::vector<uint8_t> o;
      std::vector<u32> s;
      std::vector<u64> a, b, c, d;
      for (u64 i = 0; i < n; i++)
        if (rounds == 1 || occ[i] == r) {
          o.push_back(op[i]);
          s.push_back(slot[i]);
          a.push_back(cts[i]);
          b.push_back(carg[i]);
          c.push_back(cpre[i]);
          d.push_back(clr[i]);
        }
      const u64 m = s.size();
      const void *dop, *ds, *dt, *da, *dp, *dl;
      JY_TRY(jy_stage_begin(eng));
      JY_TRY(jy_stage(eng, 0, o.data(), m, JY_HOST, &dop));
      JY_TRY(jy_stage(eng, 1, s.data(), m * 4, JY_HOST, &ds));
      JY_TRY(jy_stage(eng, 2, a.data(), m * 8, JY_HOST, &dt));
      JY_TRY(jy_stage(eng, 3, b.data(), m * 8, JY_HOST, &da));
      JY_TRY(jy_stage(eng, 4, c.data(), m * 8, JY_HOST, &dp));
      JY_TRY(jy_stage(eng, 5, d.data(), m * 8, JY_HOST, &dl));
      JY_TRY(jy_stage_end(eng));
      JY_TRY(jy_tlog_write_batch(eng, m, (const uint8_t*)dop, (const u32*)ds, (const u64*)dt, (const u64*)da,
                                 (const u64*)dp, (const u64*)dl));
    }
    return JY_OK;
  }
  if (!op || !ts || !arg || !pre || !lr) return eng->fail(JY_EINVAL, "a device batch passes every column");
  return jy_tlog_write_batch(eng, n, op, slot, ts, arg, pre, lr);
}

int32_t jy_tlog_deltas_size(jy_engine* eng, uint64_t* n_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  return jy_tlog_pending(eng, n_out);
}

int32_t jy_tlog_flush(jy_engine* eng, uint64_t cap_keys, uint64_t cap_ent, uint32_t* slot_out, uint64_t* cutoff_out,
                      uint64_t* offs_out, uint64_t* ts_out, uint64_t* pre_out, uint64_t* lr_out, uint64_t* nkeys_out,
                      uint64_t* nent_out, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  u64 k = 0, m = 0;
  // sizes first (nothing written or cleared)
  JY_TRY(jy_tlog_flush_dev(eng, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &k, &m));
  *nkeys_out = k;
  *nent_out = m;
  if (k == 0 || cap_keys < k || cap_ent < m) return JY_OK;
  u32* ds = slot_out;
  u64 *dc = cutoff_out, *doff = offs_out, *dt = ts_out, *dp = pre_out, *dl = lr_out;
  if (mem == JY_HOST) {
    void* p;
    JY_TRY(jy_scratch(eng, 0, k * 4 + 64, &p));
    ds = static_cast<u32*>(p);
    JY_TRY(jy_scratch(eng, 1, k * 8 + 64, &p));
    dc = static_cast<u64*>(p);
    JY_TRY(jy_scratch(eng, 2, (k + 1) * 8 + 64, &p));
    doff = static_cast<u64*>(p);
    JY_TRY(jy_scratch(eng, 3, m * 8 + 64, &p));
    dt = static_cast<u64*>(p);
    JY_TRY(jy_scratch(eng, 4, m * 8 + 64, &p));
    dp = static_cast<u64*>(p);
    JY_TRY(jy_scratch(eng, 5, m * 8 + 64, &p));
    dl = static_cast<u64*>(p);
  }
  JY_TRY(jy_tlog_flush_dev(eng, k, m, ds, dc, doff, dt, dp, dl, &k, &m));
  if (mem == JY_HOST) {
    JY_HIP(eng, hipMemcpyAsync(slot_out, ds, k * 4, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(cutoff_out, dc, k * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(offs_out, doff, (k + 1) * 8, hipMemcpyDeviceToHost, eng->stream));
    if (m) {
      JY_HIP(eng, hipMemcpyAsync(ts_out, dt, m * 8, hipMemcpyDeviceToHost, eng->stream));
      JY_HIP(eng, hipMemcpyAsync(pre_out, dp, m * 8, hipMemcpyDeviceToHost, eng->stream));
      JY_HIP(eng, hipMemcpyAsync(lr_out, dl, m * 8, hipMemcpyDeviceToHost, eng->stream));
    }
  }
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

int32_t jy_tlog_read_sizes(jy_engine* eng, uint64_t n, const uint32_t* slots, uint64_t* len, uint64_t* cut) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  JY_TRY(jy_slots_check(eng, JY_TLOG, n, slots, JY_HOST));
  const void* ds;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slots, n * 4, JY_HOST, &ds));
  JY_TRY(jy_stage_end(eng));
  void* o;
  JY_TRY(jy_scratch(eng, 11, n * 16, &o));
  u64* d = static_cast<u64*>(o);
  JY_TRY(jy_tlog_sizes(eng, n, (const u32*)ds, d, d + n));
  JY_HIP(eng, hipMemcpyAsync(len, d, n * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(cut, d + n, n * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

int32_t jy_tlog_read(jy_engine* eng, uint64_t n, const uint32_t* slots, const uint64_t* out_offs, uint64_t* ts,
                     uint64_t* pre, uint64_t* lr) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  JY_TRY(jy_slots_check(eng, JY_TLOG, n, slots, JY_HOST));
  const u64 m = out_offs[n];
  const void *ds, *doo;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slots, n * 4, JY_HOST, &ds));
  JY_TRY(jy_stage(eng, 1, out_offs, (n + 1) * 8, JY_HOST, &doo));
  JY_TRY(jy_stage_end(eng));
  void* o;
  JY_TRY(jy_scratch(eng, 11, std::max<u64>(m, 1) * 24, &o));
  u64* d = static_cast<u64*>(o);
  JY_TRY(jy_tlog_gather(eng, n, (const u32*)ds, (const u64*)doo, d, d + m, d + 2 * m));
  if (m) {
    JY_HIP(eng, hipMemcpyAsync(ts, d, m * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(pre, d + m, m * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(lr, d + 2 * m, m * 8, hipMemcpyDeviceToHost, eng->stream));
  }
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

int32_t jy_ujson_converge(jy_engine* eng, uint64_t n, const uint32_t* slot, const uint64_t* eoffs, uint64_t nel,
                          const uint64_t* dots, const uint64_t* elems, const uint64_t* voffs, uint64_t nvv,
                          const uint64_t* vv, const uint64_t* coffs, uint64_t ncloud, const uint64_t* cloud,
                          int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  JY_TRY(jy_slots_check(eng, JY_UJSON, n, slot, mem));
  if (mem == JY_HOST) {
    if (!csr_ok(eoffs, n, nel) || !csr_ok(voffs, n, nvv) || !csr_ok(coffs, n, ncloud))
      return eng->fail(JY_EINVAL, "element / vv / cloud offsets are not CSRs of their totals");
    std::vector<u32> occ;
    const u32 rounds = rounds_of(n, slot, occ);
    if (rounds > 1) {
      for (u32 r = 0; r < rounds; r++) {
        std::vector<u64> idx;
        for (u64 i = 0; i < n; i++)
          if (occ[i] == r) idx.push_back(i);
        std::vector<u32> s;
        for (u64 i : idx) s.push_back(slot[i]);
        CsrPick e = pick(idx, eoffs, {dots, elems});
        CsrPick v = pick(idx, voffs, {vv});
        CsrPick c = pick(idx, coffs, {cloud});
        JY_TRY(jy_ujson_converge(eng, s.size(), s.data(), e.offs.data(), e.offs.back(), e.cols[0].data(),
                                 e.cols[1].data(), v.offs.data(), v.offs.back(), v.cols[0].data(), c.offs.data(),
                                 c.offs.back(), c.cols[0].data(), JY_HOST));
      }
      return JY_OK;
    }
  }
  const void *ds, *de, *dd, *del, *dv, *dvv, *dc, *dcl;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slot, n * 4, mem, &ds));
  JY_TRY(jy_stage(eng, 1, eoffs, (n + 1) * 8, mem, &de));
  JY_TRY(jy_stage(eng, 2, dots, nel * 8, mem, &dd));
  JY_TRY(jy_stage(eng, 3, elems, nel * 8, mem, &del));
  JY_TRY(jy_stage(eng, 4, voffs, (n + 1) * 8, mem, &dv));
  JY_TRY(jy_stage(eng, 5, vv, nvv * 8, mem, &dvv));
  JY_TRY(jy_stage(eng, 6, coffs, (n + 1) * 8, mem, &dc));
  JY_TRY(jy_stage(eng, 7, cloud, ncloud * 8, mem, &dcl));
  JY_TRY(jy_stage_end(eng));
  return jy_ujson_merge(eng, n, (const u32*)ds, (const u64*)de, nel, (const u64*)dd, (const u64*)del,
                        (const u64*)dv, nvv, (const u64*)dvv, (const u64*)dc, ncloud, (const u64*)dcl);
}

int32_t jy_ujson_write(jy_engine* eng, uint64_t n, const uint8_t* op, const uint32_t* slot, const uint64_t* elem,
                       uint32_t col, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  if (n >= 0xFFFFFFFFull) return eng->fail(JY_ERANGE, "more than 2^32 - 1 commands in one call");
  JY_TRY(jy_slots_check(eng, JY_UJSON, n, slot, mem));
  if (mem != JY_HOST) return jy_ujson_write_batch(eng, n, op, slot, elem, col);
  for (u64 i = 0; i < n; i++)
    if (op[i] > JY_UJSON_CLR) return eng->fail(JY_EINVAL, "unknown UJSON write op");
  std::vector<u32> occ;
  const u32 rounds = rounds_of(n, slot, occ);
  for (u32 r = 0; r < rounds; r++) {
    std::vector<uint8_t> o;
    std::vector<u32> s;
    std::vector<u64> e;
    for (u64 i = 0; i < n; i++)
      if (rounds == 1 || occ[i] == r) {
        o.push_back(op[i]);
        s.push_back(slot[i]);
        e.push_back(elem ? elem[i] : 0);
      }
    const u64 m = s.size();
    const void *dop, *ds, *de;
    JY_TRY(jy_stage_begin(eng));
    JY_TRY(jy_stage(eng, 0, o.data(), m, JY_HOST, &dop));
    JY_TRY(jy_stage(eng, 1, s.data(), m * 4, JY_HOST, &ds));
    JY_TRY(jy_stage(eng, 2, e.data(), m * 8, JY_HOST, &de));
    JY_TRY(jy_stage_end(eng));
    JY_TRY(jy_ujson_write_batch(eng, m, (const uint8_t*)dop, (const u32*)ds, (const u64*)de, col));
  }
  return JY_OK;
}

int32_t jy_ujson_deltas_size(jy_engine* eng, uint64_t* n_out) {
  JY_HIP(eng, hipSetDevice(eng->device));
  return jy_ujson_pending(eng, n_out);
}

int32_t jy_ujson_flush(jy_engine* eng, uint64_t cap_docs, uint64_t cap_el, uint64_t cap_cl, uint32_t* slot_out,
                       uint64_t* eoff_out, uint64_t* dots_out, uint64_t* elems_out, uint64_t* vv_out,
                       uint64_t* coff_out, uint64_t* cloud_out, uint64_t* ndocs_out, uint64_t* nel_out,
                       uint64_t* ncl_out, int32_t mem) {
  JY_HIP(eng, hipSetDevice(eng->device));
  u64 k = 0, me = 0, mc = 0;
  JY_TRY(jy_ujson_flush_dev(eng, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &k, &me,
                            &mc));
  *ndocs_out = k;
  *nel_out = me;
  *ncl_out = mc;
  if (k == 0 || cap_docs < k || cap_el < me || cap_cl < mc) return JY_OK;
  const u64 R = eng->ujson.R;
  u32* ds = slot_out;
  u64 *deo = eoff_out, *dd = dots_out, *de = elems_out, *dv = vv_out, *dco = coff_out, *dc = cloud_out;
  if (mem == JY_HOST) {
    void* p;
    JY_TRY(jy_scratch(eng, 0, k * 4 + 64, &p));
    ds = static_cast<u32*>(p);
    JY_TRY(jy_scratch(eng, 1, (k + 1) * 8 * 2 + 64, &p));
    deo = static_cast<u64*>(p);
    dco = deo + (k + 1);
    JY_TRY(jy_scratch(eng, 2, (2 * me + mc + k * R) * 8 + 64, &p));
    dd = static_cast<u64*>(p);
    de = dd + me;
    dc = de + me;
    dv = dc + mc;
  }
  JY_TRY(jy_ujson_flush_dev(eng, k, me, mc, ds, deo, dd, de, dv, dco, dc, &k, &me, &mc));
  if (mem == JY_HOST) {
    JY_HIP(eng, hipMemcpyAsync(slot_out, ds, k * 4, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(eoff_out, deo, (k + 1) * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(coff_out, dco, (k + 1) * 8, hipMemcpyDeviceToHost, eng->stream));
    if (me) {
      JY_HIP(eng, hipMemcpyAsync(dots_out, dd, me * 8, hipMemcpyDeviceToHost, eng->stream));
      JY_HIP(eng, hipMemcpyAsync(elems_out, de, me * 8, hipMemcpyDeviceToHost, eng->stream));
    }
    if (mc) JY_HIP(eng, hipMemcpyAsync(cloud_out, dc, mc * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(vv_out, dv, k * R * 8, hipMemcpyDeviceToHost, eng->stream));
  }
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

int32_t jy_ujson_read_sizes(jy_engine* eng, uint64_t n, const uint32_t* slots, uint64_t* ne, uint64_t* nc) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  JY_TRY(jy_slots_check(eng, JY_UJSON, n, slots, JY_HOST));
  const void* ds;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slots, n * 4, JY_HOST, &ds));
  JY_TRY(jy_stage_end(eng));
  void* o;
  JY_TRY(jy_scratch(eng, 11, n * 16, &o));
  u64* d = static_cast<u64*>(o);
  JY_TRY(jy_ujson_sizes(eng, n, (const u32*)ds, d, d + n));
  JY_HIP(eng, hipMemcpyAsync(ne, d, n * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(nc, d + n, n * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

int32_t jy_ujson_read(jy_engine* eng, uint64_t n, const uint32_t* slots, const uint64_t* eoffs, uint64_t* dots,
                      uint64_t* elems, uint64_t* vv, const uint64_t* coffs, uint64_t* cloud) {
  JY_HIP(eng, hipSetDevice(eng->device));
  if (n == 0) return JY_OK;
  JY_TRY(jy_slots_check(eng, JY_UJSON, n, slots, JY_HOST));
  const u64 me = eoffs[n], mc = coffs[n], R = eng->ujson.R;
  const void *ds, *de, *dc;
  JY_TRY(jy_stage_begin(eng));
  JY_TRY(jy_stage(eng, 0, slots, n * 4, JY_HOST, &ds));
  JY_TRY(jy_stage(eng, 1, eoffs, (n + 1) * 8, JY_HOST, &de));
  JY_TRY(jy_stage(eng, 2, coffs, (n + 1) * 8, JY_HOST, &dc));
  JY_TRY(jy_stage_end(eng));
  void* o;
  const u64 words = 2 * me + mc + n * R;
  JY_TRY(jy_scratch(eng, 11, std::max<u64>(words, 1) * 8, &o));
  u64* d = static_cast<u64*>(o);
  u64 *odots = d, *oelems = d + me, *ocloud = d + 2 * me, *ovv = d + 2 * me + mc;
  JY_TRY(jy_ujson_gather(eng, n, (const u32*)ds, (const u64*)de, (const u64*)dc, me, mc, odots, oelems, ovv, ocloud));
  if (me) {
    JY_HIP(eng, hipMemcpyAsync(dots, odots, me * 8, hipMemcpyDeviceToHost, eng->stream));
    JY_HIP(eng, hipMemcpyAsync(elems, oelems, me * 8, hipMemcpyDeviceToHost, eng->stream));
  }
  if (mc) JY_HIP(eng, hipMemcpyAsync(cloud, ocloud, mc * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipMemcpyAsync(vv, ovv, n * R * 8, hipMemcpyDeviceToHost, eng->stream));
  JY_HIP(eng, hipStreamSynchronize(eng->stream));
  return JY_OK;
}

}  // extern "C"
