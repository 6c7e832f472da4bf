// k_ujson.hip -- UJSON dot-kernel join (placeholder until the merge lands).
#include <algorithm>

#include "jy_internal.hpp"

int32_t jy_ujson_grow(jy_engine* eng, u64 need) {
  UjsonState& u = eng->ujson;
  if (need <= u.kcap && u.vv) return JY_OK;
  if (u.R == 0) u.R = eng->cfg.ujson_columns;
  u64 nk = std::max<u64>(need, u.kcap ? u.kcap * 2 : need);
  nk = std::max<u64>((nk + 63) & ~63ull, 64);
  void* v = u.vv;
  JY_TRY(jy_realloc(eng, &v, u.kcap * u.R * 8, nk * u.R * 8, true));
  u.vv = static_cast<u64*>(v);
  u.kcap = nk;
  return JY_OK;
}

int32_t jy_ujson_merge(jy_engine* eng, u64, const u32*, const u64*, u64, const u64*, const u64*, const u64*, u64,
                       const u64*, const u64*, u64, const u64*) {
  return eng->fail(JY_EINVAL, "UJSON merge not built yet");
}

extern "C" {
int32_t jy_ujson_converge(jy_engine* eng, uint64_t, const uint32_t*, const uint64_t*, uint64_t, const uint64_t*,
                          const uint64_t*, const uint64_t*, uint64_t, const uint64_t*, const uint64_t*, uint64_t,
                          const uint64_t*, int32_t) {
  return eng->fail(JY_EINVAL, "UJSON merge not built yet");
}
int32_t jy_ujson_read_sizes(jy_engine* eng, uint64_t, const uint32_t*, uint64_t*, uint64_t*) {
  return eng->fail(JY_EINVAL, "UJSON read not built yet");
}
int32_t jy_ujson_read(jy_engine* eng, uint64_t, const uint32_t*, const uint64_t*, uint64_t*, uint64_t*, uint64_t*,
                      const uint64_t*, uint64_t*) {
  return eng->fail(JY_EINVAL, "UJSON read not built yet");
}
}
