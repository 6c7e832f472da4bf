// k_tlog.hip -- TLOG segmented merge (placeholder until the merge lands).
#include <algorithm>

#include "jy_internal.hpp"

int32_t jy_tlog_grow(jy_engine* eng, u64 need) {
  TlogState& t = eng->tlog;
  if (need <= t.kcap && t.cutoff) return JY_OK;
  u64 nk = std::max<u64>(need, t.kcap ? t.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  void* c = t.cutoff;
  JY_TRY(jy_realloc(eng, &c, t.kcap * 8, nk * 8, true));
  t.cutoff = static_cast<u64*>(c);
  t.kcap = nk;
  return JY_OK;
}

int32_t jy_tlog_merge(jy_engine* eng, u64, const u32*, const u64*, const u64*, u64, const u64*, const u64*,
                      const u64*) {
  return eng->fail(JY_EINVAL, "TLOG merge not built yet");
}

extern "C" {
int32_t jy_tlog_converge(jy_engine* eng, uint64_t, const uint32_t*, const uint64_t*, const uint64_t*, uint64_t,
                         const uint64_t*, const uint64_t*, const uint64_t*, int32_t) {
  return eng->fail(JY_EINVAL, "TLOG merge not built yet");
}
int32_t jy_tlog_read_sizes(jy_engine* eng, uint64_t, const uint32_t*, uint64_t*, uint64_t*) {
  return eng->fail(JY_EINVAL, "TLOG read not built yet");
}
int32_t jy_tlog_read(jy_engine* eng, uint64_t, const uint32_t*, const uint64_t*, uint64_t*, uint64_t*, uint64_t*) {
  return eng->fail(JY_EINVAL, "TLOG read not built yet");
}
}
