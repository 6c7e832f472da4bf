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
  JY_TRY(jy_ujson_gather(eng, n, (const u32*)ds, (const u64*)de, (const u64*)dc, odots, oelems, ovv, ocloud));
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
