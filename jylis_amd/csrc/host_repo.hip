// host_repo.hip -- host mirror of the reference's Database / RepoManagerCore /
// Repo* layer over the GPU engine (include/jylis_host.h).
//
// The reference host is compiled Pony (no ponyc in this image), so its
// operator interface is restated in C++ above the C ABI:
//   RepoManagerCore.apply / flush_deltas / converge_deltas / clean_shutdown
//                                               jylis/repo_manager.pony:36-108
//   RepoGCOUNT / RepoPNCOUNT / RepoTREG / RepoTLOG  jylis/repo_*.pony
//   Database routing + help                     jylis/database.pony:25-51
//   HelpRespond / HelpRepo                      jylis/help.pony:4-44
// State lives on the GPU; converge of a peer batch is ONE engine call per
// type (the drop-in change of repo_manager.pony:92-93).  Local writes build a
// one-entry delta, converge it into the engine, and record it in the host's
// pending-delta map exactly like `_delta_for(key)` (flushed on demand).
// UJSON commands need the UJSON parse/render layer;
// UJSON converges through the engine ABI directly.

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/jylis_gpu.h"
#include "../../include/jylis_host.h"

namespace {

typedef uint64_t u64;
typedef int64_t i64;
typedef uint32_t u32;
typedef uint16_t u16;

struct BadCommand {};  // the `?` partial-function error of RepoXXX.apply
struct EngineError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---- RESP writer (jemc/pony-resp Respond) -----------------------------------
struct Respond {
  std::string out;
  void ok() { out += "+OK\r\n"; }
  void err(const std::string& m) { out += "-" + m + "\r\n"; }
  void u64v(u64 v) { out += ":" + std::to_string(v) + "\r\n"; }
  void i64v(i64 v) { out += ":" + std::to_string(v) + "\r\n"; }
  void str(const std::string& s) { out += "$" + std::to_string(s.size()) + "\r\n" + s + "\r\n"; }
  void null() { out += "$-1\r\n"; }
  void array_start(u64 n) { out += "*" + std::to_string(n) + "\r\n"; }
};

struct Cmd {  // Iterator[String] over the words after the data type
  const std::vector<std::string>& w;
  size_t i;
  std::string next() {
    if (i >= w.size()) throw BadCommand();
    return w[i++];
  }
  bool has() const { return i < w.size(); }
};

// Pony String.u64()? / i64()? / usize()?: decimal integer, whole string
u64 parse_u64(const std::string& s) {
  if (s.empty() || s.size() > 20) throw BadCommand();
  u64 v = 0;
  for (char c : s) {
    if (c < '0' || c > '9') throw BadCommand();
    u64 d = (u64)(c - '0');
    if (v > (~0ull - d) / 10) throw BadCommand();
    v = v * 10 + d;
  }
  return v;
}
i64 parse_i64(const std::string& s) {
  if (s.empty()) throw BadCommand();
  bool neg = s[0] == '-';
  u64 m = parse_u64(neg || s[0] == '+' ? s.substr(1) : s);
  if (neg ? m > (1ull << 63) : m > (u64)INT64_MAX) throw BadCommand();
  return neg ? (i64)(0 - m) : (i64)m;
}

// Pony String order (unsigned bytewise, then shorter first)
int str_cmp(const std::string& a, const std::string& b) {
  const size_t n = std::min(a.size(), b.size());
  const int c = n ? std::memcmp(a.data(), b.data(), n) : 0;
  if (c) return c < 0 ? -1 : 1;
  return a.size() == b.size() ? 0 : (a.size() < b.size() ? -1 : 1);
}

// ---- delta objects (host-side pony-crdt deltas) --------------------------------
struct TLEntry {
  std::string v;
  u64 ts;
};
bool tl_before(const TLEntry& a, const TLEntry& b) {
  return a.ts != b.ts ? a.ts > b.ts : str_cmp(a.v, b.v) > 0;
}
struct TLDelta {  // a TLog: canonical entries + cutoff
  u64 cutoff = 0;
  std::vector<TLEntry> e;
  bool write(const std::string& v, u64 ts) {
    if (ts < cutoff) return false;
    TLEntry x{v, ts};
    auto it = std::lower_bound(e.begin(), e.end(), x, tl_before);
    if (it != e.end() && it->ts == ts && it->v == v) return false;
    e.insert(it, x);
    return true;
  }
  void raise(u64 c) {
    if (c <= cutoff) return;
    cutoff = c;
    while (!e.empty() && e.back().ts < c) e.pop_back();
  }
};
struct TRDelta {
  std::string v;
  u64 ts = 0;
};

struct Batch {  // (type name, Array[(String, Any box)]) of msg.pony:20-24
  std::string type;
  std::vector<std::string> keys;
  std::vector<std::vector<std::pair<u64, u64>>> g;  // GCOUNT; PNCOUNT: P
  std::vector<std::vector<std::pair<u64, u64>>> n;  // PNCOUNT: N
  std::vector<TRDelta> tr;
  std::vector<TLDelta> tl;
};

// ---- engine helpers ----------------------------------------------------------
struct Eng {
  jy_engine* e = nullptr;
  void ck(int32_t rc) {
    if (rc != JY_OK) throw EngineError(jy_last_error(e));
  }
  u32 intern(int type, const std::string& k) {
    u64 offs[2] = {0, k.size()};
    u32 s;
    ck(jy_keys_intern(e, type, 1, reinterpret_cast<const uint8_t*>(k.data()), offs, &s));
    return s;
  }
  bool lookup(int type, const std::string& k, u32& s) {
    u64 offs[2] = {0, k.size()};
    ck(jy_keys_lookup(e, type, 1, reinterpret_cast<const uint8_t*>(k.data()), offs, &s));
    return s != JY_NO_SLOT;
  }
  std::vector<u32> intern_all(int type, const std::vector<std::string>& keys) {
    std::vector<uint8_t> kb;
    std::vector<u64> ko{0};
    for (const auto& k : keys) {
      kb.insert(kb.end(), k.begin(), k.end());
      ko.push_back(kb.size());
    }
    std::vector<u32> s(keys.size());
    if (!keys.empty()) ck(jy_keys_intern(e, type, keys.size(), kb.data(), ko.data(), s.data()));
    return s;
  }
  u16 col(u64 id) {
    u32 c;
    ck(jy_replica_col(e, id, &c));
    return (u16)c;
  }
  // one counter cell (sign 0 = P / GCOUNT, 1 = N) of a slot, as the engine holds it
  u64 cell(int type, u32 slot, u16 c, int sign) {
    const u32 ncols = (u32)c + 1;
    std::vector<u64> out((type == JY_PNCOUNT ? 2 : 1) * ncols);
    ck(jy_counter_export(e, type, ncols, slot, 1, out.data()));
    return out[(u64)sign * ncols + c];
  }
  void pack(int type, const std::vector<std::string>& vals, std::vector<u64>& pre, std::vector<u64>& lr) {
    std::vector<uint8_t> vb;
    std::vector<u64> vo{0};
    for (const auto& v : vals) {
      vb.insert(vb.end(), v.begin(), v.end());
      vo.push_back(vb.size());
    }
    pre.resize(vals.size());
    lr.resize(vals.size());
    if (!vals.empty()) ck(jy_values_pack(e, type, vals.size(), vb.data(), vo.data(), pre.data(), lr.data()));
  }
  std::string value(int type, u64 pre, u64 lr) {
    const u64 n = lr & ((1ull << 24) - 1);
    std::string s(n, '\0');
    if (n <= 8) {
      for (u64 j = 0; j < n; j++) s[j] = (char)((pre >> (56 - 8 * j)) & 0xFF);
    } else {
      ck(jy_arena_read(e, type, lr >> 24, n, reinterpret_cast<uint8_t*>(&s[0])));
    }
    return s;
  }
  // one TLOG read: cutoff + entries of a slot
  TLDelta tlog(u32 s) {
    u64 len, cut;
    ck(jy_tlog_read_sizes(e, 1, &s, &len, &cut));
    TLDelta d;
    d.cutoff = cut;
    std::vector<u64> ts(len + 1), pre(len + 1), lr(len + 1);
    u64 offs[2] = {0, len};
    ck(jy_tlog_read(e, 1, &s, offs, ts.data(), pre.data(), lr.data()));
    for (u64 j = 0; j < len; j++) d.e.push_back(TLEntry{value(JY_TLOG, pre[j], lr[j]), ts[j]});
    return d;
  }
};

// ---- repos -------------------------------------------------------------------
struct Repo {
  Eng* eng;
  u64 identity;
  virtual ~Repo() = default;
  virtual const char* datatype() const = 0;
  virtual std::vector<std::pair<std::string, std::string>> commands() const = 0;
  virtual bool apply(Respond& r, Cmd& c) = 0;  // returns "changed"
  virtual size_t deltas_size() const = 0;
  virtual Batch flush_deltas() = 0;
  virtual void converge_batch(const Batch& b) = 0;
  // HelpRepo.apply (help.pony:17-44)
  std::string help(Cmd& c) const {
    auto cmds = commands();
    if (c.has()) {
      const std::string op = c.next();
      for (auto& kv : cmds)
        if (kv.first == op)
          return std::string("This operation expects the arguments in the following form:\n") + datatype() + " " + op +
                 " " + kv.second;
    }
    std::string buf = "The following are valid operations for this data type:";
    for (auto& kv : cmds) buf += std::string("\n") + datatype() + " " + kv.first + " " + kv.second;
    return buf;
  }
};

// Counters keep THIS replica's own entry on the host, with the reference's
// rules: INC assigns own + v (wrapping, GCounter.increment) and a converged
// echo of our id max-merges into it.  The engine max-merges every column,
// own included, so after a wrapping INC its own cell can exceed the
// reference's; GET therefore reads the engine sum and swaps in the host's own
// entry: sum - engine_cell(own) + own (all mod 2^64).  Every other column --
// the converge path -- is exactly the engine's.
struct OwnCol {
  std::unordered_map<std::string, u64> own;
  u64 get(const std::string& k) const {
    auto it = own.find(k);
    return it == own.end() ? 0 : it->second;
  }
  void echo(const std::string& k, u64 v) {  // converge of our id: max-merge
    u64& t = own[k];
    if (v > t) t = v;
  }
};

// GCOUNT (repo_gcount.pony)
struct RepoGCOUNT : Repo {
  OwnCol mine;
  std::map<std::string, u64> deltas;  // _deltas: key -> our total at the last INC
  const char* datatype() const override { return "GCOUNT"; }
  std::vector<std::pair<std::string, std::string>> commands() const override {
    return {{"GET", "key"}, {"INC", "key value"}};
  }
  bool apply(Respond& r, Cmd& c) override {
    const std::string op = c.next();
    if (op == "GET") {  // repo_gcount.pony:53-55
      const std::string k = c.next();
      u32 s;
      u64 v = 0;
      if (eng->lookup(JY_GCOUNT, k, s)) {
        eng->ck(jy_gcount_get(eng->e, 1, &s, &v, JY_HOST));
        v = v - eng->cell(JY_GCOUNT, s, eng->col(identity), 0) + mine.get(k);
      }
      r.u64v(v);
      return false;
    }
    if (op == "INC") {  // repo_gcount.pony:57-60
      const std::string k = c.next();
      const u64 v = parse_u64(c.next());
      const u32 s = eng->intern(JY_GCOUNT, k);
      const u16 col = eng->col(identity);
      u64& t = mine.own[k];
      t += v;
      deltas[k] = t;
      eng->ck(jy_gcount_converge(eng->e, 1, &s, &col, &t, JY_HOST));
      r.ok();
      return true;
    }
    throw BadCommand();
  }
  size_t deltas_size() const override { return deltas.size(); }
  Batch flush_deltas() override {
    Batch b;
    b.type = "GCOUNT";
    for (auto& kv : deltas) {
      b.keys.push_back(kv.first);
      b.g.push_back({{identity, kv.second}});
    }
    deltas.clear();
    return b;
  }
  void converge_batch(const Batch& b) override {
    auto slots = eng->intern_all(JY_GCOUNT, b.keys);
    std::vector<u32> cs;
    std::vector<u16> cc;
    std::vector<u64> cv;
    for (size_t i = 0; i < b.keys.size(); i++)
      for (auto& e : b.g[i]) {
        if (e.first == identity) mine.echo(b.keys[i], e.second);
        cs.push_back(slots[i]);
        cc.push_back(eng->col(e.first));
        cv.push_back(e.second);
      }
    if (!cs.empty()) eng->ck(jy_gcount_converge(eng->e, cs.size(), cs.data(), cc.data(), cv.data(), JY_HOST));
  }
};

// PNCOUNT (repo_pncount.pony): INC/DEC parse i64 and bit-cast to u64 (:36,60,65)
struct RepoPNCOUNT : Repo {
  OwnCol mp, mn;
  std::map<std::string, std::pair<bool, bool>> touched;  // which of P / N a delta carries
  std::map<std::string, std::pair<u64, u64>> dval;       // their values at the last INC / DEC
  const char* datatype() const override { return "PNCOUNT"; }
  std::vector<std::pair<std::string, std::string>> commands() const override {
    return {{"GET", "key"}, {"INC", "key value"}, {"DEC", "key value"}};
  }
  bool apply(Respond& r, Cmd& c) override {
    const std::string op = c.next();
    if (op == "GET") {  // repo_pncount.pony:55-57
      const std::string k = c.next();
      u32 s;
      i64 v = 0;
      if (eng->lookup(JY_PNCOUNT, k, s)) {
        eng->ck(jy_pncount_get(eng->e, 1, &s, &v, JY_HOST));
        const u16 col = eng->col(identity);
        u64 u = (u64)v;
        u = u - eng->cell(JY_PNCOUNT, s, col, 0) + mp.get(k);
        u = u + eng->cell(JY_PNCOUNT, s, col, 1) - mn.get(k);
        v = (i64)u;
      }
      r.i64v(v);
      return false;
    }
    if (op == "INC" || op == "DEC") {  // repo_pncount.pony:59-67
      const std::string k = c.next();
      const u64 v = (u64)parse_i64(c.next());
      const bool inc = op == "INC";
      const u32 s = eng->intern(JY_PNCOUNT, k);
      const u16 col = eng->col(identity);
      u64& t = (inc ? mp : mn).own[k];
      t += v;
      auto& tt = touched[k];
      auto& dv = dval[k];
      (inc ? tt.first : tt.second) = true;
      (inc ? dv.first : dv.second) = t;
      if (inc) eng->ck(jy_pncount_converge(eng->e, 1, &s, &col, &t, 0, nullptr, nullptr, nullptr, JY_HOST));
      else eng->ck(jy_pncount_converge(eng->e, 0, nullptr, nullptr, nullptr, 1, &s, &col, &t, JY_HOST));
      r.ok();
      return true;
    }
    throw BadCommand();
  }
  size_t deltas_size() const override { return touched.size(); }
  Batch flush_deltas() override {
    Batch b;
    b.type = "PNCOUNT";
    for (auto& kv : touched) {
      b.keys.push_back(kv.first);
      b.g.push_back({});
      b.n.push_back({});
      const auto& dv = dval[kv.first];
      if (kv.second.first) b.g.back().push_back({identity, dv.first});
      if (kv.second.second) b.n.back().push_back({identity, dv.second});
    }
    touched.clear();
    dval.clear();
    return b;
  }
  void converge_batch(const Batch& b) override {
    auto slots = eng->intern_all(JY_PNCOUNT, b.keys);
    std::vector<u32> ps, ns;
    std::vector<u16> pc, nc;
    std::vector<u64> pv, nv;
    for (size_t i = 0; i < b.keys.size(); i++) {
      for (auto& e : b.g[i]) {
        if (e.first == identity) mp.echo(b.keys[i], e.second);
        ps.push_back(slots[i]);
        pc.push_back(eng->col(e.first));
        pv.push_back(e.second);
      }
      for (auto& e : b.n[i]) {
        if (e.first == identity) mn.echo(b.keys[i], e.second);
        ns.push_back(slots[i]);
        nc.push_back(eng->col(e.first));
        nv.push_back(e.second);
      }
    }
    eng->ck(jy_pncount_converge(eng->e, ps.size(), ps.data(), pc.data(), pv.data(), ns.size(), ns.data(), nc.data(),
                                nv.data(), JY_HOST));
  }
};

// TREG (repo_treg.pony)
struct RepoTREG : Repo {
  std::map<std::string, TRDelta> deltas;
  const char* datatype() const override { return "TREG"; }
  std::vector<std::pair<std::string, std::string>> commands() const override {
    return {{"GET", "key"}, {"SET", "key value timestamp"}};
  }
  std::pair<std::string, u64> read(u32 s) {
    u64 ts, pre, lr;
    eng->ck(jy_treg_read(eng->e, 1, &s, &ts, &pre, &lr));
    return {eng->value(JY_TREG, pre, lr), ts};
  }
  void put(const std::vector<u32>& slots, const std::vector<std::string>& vals, const std::vector<u64>& ts) {
    std::vector<u64> pre, lr;
    eng->pack(JY_TREG, vals, pre, lr);
    if (!slots.empty())
      eng->ck(jy_treg_converge(eng->e, slots.size(), slots.data(), ts.data(), pre.data(), lr.data(), JY_HOST));
  }
  bool apply(Respond& r, Cmd& c) override {
    const std::string op = c.next();
    if (op == "GET") {  // repo_treg.pony:54-63
      const std::string k = c.next();
      u32 s;
      if (!eng->lookup(JY_TREG, k, s)) {
        r.null();
        return false;
      }
      auto cur = read(s);
      r.array_start(2);
      r.str(cur.first);
      r.u64v(cur.second);
      return false;
    }
    if (op == "SET") {  // repo_treg.pony:65-68
      const std::string k = c.next(), v = c.next();
      const u64 ts = parse_u64(c.next());
      const u32 s = eng->intern(JY_TREG, k);  // _data_for(key)
      auto cur = read(s);
      TRDelta& d = deltas[k];                  // _delta_for(key)
      if (ts > cur.second || (ts == cur.second && str_cmp(v, cur.first) > 0)) {
        put({s}, {v}, {ts});
        if (ts > d.ts || (ts == d.ts && str_cmp(v, d.v) > 0)) d = TRDelta{v, ts};
      }
      r.ok();
      return true;
    }
    throw BadCommand();
  }
  size_t deltas_size() const override { return deltas.size(); }
  Batch flush_deltas() override {
    Batch b;
    b.type = "TREG";
    for (auto& kv : deltas) {
      b.keys.push_back(kv.first);
      b.tr.push_back(kv.second);
    }
    deltas.clear();
    return b;
  }
  void converge_batch(const Batch& b) override {
    auto slots = eng->intern_all(JY_TREG, b.keys);
    std::vector<std::string> vals;
    std::vector<u64> ts;
    for (auto& d : b.tr) {
      vals.push_back(d.v);
      ts.push_back(d.ts);
    }
    put(slots, vals, ts);
  }
};

// TLOG (repo_tlog.pony)
struct RepoTLOG : Repo {
  std::map<std::string, TLDelta> deltas;
  const char* datatype() const override { return "TLOG"; }
  std::vector<std::pair<std::string, std::string>> commands() const override {
    return {{"GET", "key [count]"}, {"INS", "key value timestamp"}, {"SIZE", "key"}, {"CUTOFF", "key"},
            {"TRIMAT", "key timestamp"}, {"TRIM", "key count"}, {"CLR", "key"}};
  }
  void put(u32 s, const TLDelta& d) {
    std::vector<std::string> vals;
    std::vector<u64> ts, pre, lr;
    for (auto& e : d.e) {
      vals.push_back(e.v);
      ts.push_back(e.ts);
    }
    eng->pack(JY_TLOG, vals, pre, lr);
    u64 offs[2] = {0, d.e.size()};
    eng->ck(jy_tlog_converge(eng->e, 1, &s, &d.cutoff, offs, d.e.size(), ts.data(), pre.data(), lr.data(),
                             JY_HOST));
  }
  void raise(const std::string& k, u32 s, u64 c) {  // raise_cutoff(c, _delta_for(key))
    TLDelta d;
    d.cutoff = c;
    put(s, d);
    deltas[k].raise(c);
  }
  bool apply(Respond& r, Cmd& c) override {
    const std::string op = c.next();
    if (op == "GET") {  // repo_tlog.pony:69-83; count defaults to USize max (:49-50)
      const std::string k = c.next();
      u64 count = ~0ull;
      if (c.has()) {
        try {
          count = parse_u64(c.next());
        } catch (BadCommand&) {
          count = ~0ull;
        }
      }
      u32 s;
      if (!eng->lookup(JY_TLOG, k, s)) {
        r.array_start(0);
        return false;
      }
      TLDelta cur = eng->tlog(s);
      const u64 total = std::min<u64>(cur.e.size(), count);
      r.array_start(total);
      for (u64 j = 0; j < total; j++) {
        r.array_start(2);
        r.str(cur.e[j].v);
        r.u64v(cur.e[j].ts);
      }
      return false;
    }
    if (op == "SIZE" || op == "CUTOFF") {  // :90-96
      const std::string k = c.next();
      u32 s;
      u64 v = 0;
      if (eng->lookup(JY_TLOG, k, s)) {
        TLDelta cur = eng->tlog(s);
        v = op == "SIZE" ? cur.e.size() : cur.cutoff;
      }
      r.u64v(v);
      return false;
    }
    if (op == "INS") {  // :85-88
      const std::string k = c.next(), v = c.next();
      const u64 ts = parse_u64(c.next());
      const u32 s = eng->intern(JY_TLOG, k);
      TLDelta& d = deltas[k];
      TLDelta cur = eng->tlog(s);
      if (cur.write(v, ts)) {
        TLDelta one;
        one.e.push_back(TLEntry{v, ts});
        put(s, one);
        d.write(v, ts);
      }
      r.ok();
      return true;
    }
    if (op == "TRIMAT") {  // :98-101
      const std::string k = c.next();
      const u64 ts = parse_u64(c.next());
      const u32 s = eng->intern(JY_TLOG, k);
      deltas[k];
      if (ts > eng->tlog(s).cutoff) raise(k, s, ts);
      r.ok();
      return true;
    }
    if (op == "TRIM" || op == "CLR") {  // :103-111
      const std::string k = c.next();
      u64 n = 0;
      if (op == "TRIM") n = parse_u64(c.next());
      const u32 s = eng->intern(JY_TLOG, k);
      deltas[k];
      TLDelta cur = eng->tlog(s);
      if (n == 0) {
        if (!cur.e.empty() && cur.e.front().ts + 1 > cur.cutoff) raise(k, s, cur.e.front().ts + 1);
      } else if (n - 1 < cur.e.size() && cur.e[n - 1].ts > cur.cutoff) {
        raise(k, s, cur.e[n - 1].ts);
      }
      r.ok();
      return true;
    }
    throw BadCommand();
  }
  size_t deltas_size() const override { return deltas.size(); }
  Batch flush_deltas() override {
    Batch b;
    b.type = "TLOG";
    for (auto& kv : deltas) {
      b.keys.push_back(kv.first);
      b.tl.push_back(kv.second);
    }
    deltas.clear();
    return b;
  }
  void converge_batch(const Batch& b) override {
    auto slots = eng->intern_all(JY_TLOG, b.keys);
    std::vector<u64> cut, offs{0}, ts, pre, lr;
    std::vector<std::string> vals;
    for (auto& d : b.tl) {
      cut.push_back(d.cutoff);
      for (auto& e : d.e) {
        vals.push_back(e.v);
        ts.push_back(e.ts);
      }
      offs.push_back(ts.size());
    }
    eng->pack(JY_TLOG, vals, pre, lr);
    if (!slots.empty())
      eng->ck(jy_tlog_converge(eng->e, slots.size(), slots.data(), cut.data(), offs.data(), ts.size(), ts.data(),
                               pre.data(), lr.data(), JY_HOST));
  }
};

// ---- batch blob (engine-neutral stand-in for MsgPushDeltas bytes) --------------
struct Writer {
  std::vector<uint8_t> b;
  void u32v(u32 v) { b.insert(b.end(), reinterpret_cast<uint8_t*>(&v), reinterpret_cast<uint8_t*>(&v) + 4); }
  void u64v(u64 v) { b.insert(b.end(), reinterpret_cast<uint8_t*>(&v), reinterpret_cast<uint8_t*>(&v) + 8); }
  void str(const std::string& s) {
    u32v((u32)s.size());
    b.insert(b.end(), s.begin(), s.end());
  }
};
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  void need(size_t n) {
    if ((size_t)(end - p) < n) throw BadCommand();
  }
  u32 u32v() {
    need(4);
    u32 v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  u64 u64v() {
    need(8);
    u64 v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  std::string str() {
    const u32 n = u32v();
    need(n);
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
};

void write_batch(Writer& w, const Batch& b) {
  w.str(b.type);
  w.u64v(b.keys.size());
  for (size_t i = 0; i < b.keys.size(); i++) {
    w.str(b.keys[i]);
    if (b.type == "GCOUNT" || b.type == "PNCOUNT") {
      w.u32v((u32)b.g[i].size());
      for (auto& e : b.g[i]) {
        w.u64v(e.first);
        w.u64v(e.second);
      }
      if (b.type == "PNCOUNT") {
        w.u32v((u32)b.n[i].size());
        for (auto& e : b.n[i]) {
          w.u64v(e.first);
          w.u64v(e.second);
        }
      }
    } else if (b.type == "TREG") {
      w.u64v(b.tr[i].ts);
      w.str(b.tr[i].v);
    } else if (b.type == "TLOG") {
      w.u64v(b.tl[i].cutoff);
      w.u32v((u32)b.tl[i].e.size());
      for (auto& e : b.tl[i].e) {
        w.u64v(e.ts);
        w.str(e.v);
      }
    }
  }
}

Batch read_batch(Reader& r) {
  Batch b;
  b.type = r.str();
  const u64 n = r.u64v();
  for (u64 i = 0; i < n; i++) {
    b.keys.push_back(r.str());
    if (b.type == "GCOUNT" || b.type == "PNCOUNT") {
      b.g.emplace_back();
      for (u32 m = r.u32v(); m; m--) {
        const u64 id = r.u64v();
        b.g.back().push_back({id, r.u64v()});
      }
      if (b.type == "PNCOUNT") {
        b.n.emplace_back();
        for (u32 m = r.u32v(); m; m--) {
          const u64 id = r.u64v();
          b.n.back().push_back({id, r.u64v()});
        }
      }
    } else if (b.type == "TREG") {
      TRDelta d;
      d.ts = r.u64v();
      d.v = r.str();
      b.tr.push_back(d);
    } else if (b.type == "TLOG") {
      TLDelta d;
      d.cutoff = r.u64v();
      for (u32 m = r.u32v(); m; m--) {
        const u64 ts = r.u64v();
        d.write(r.str(), ts);  // a decoded TLog is canonical by construction
      }
      b.tl.push_back(d);
    } else {
      throw BadCommand();
    }
  }
  return b;
}

const char* kDatabaseHelp =
    "The first word of each command must be a data type.\n"
    "The following are valid data types (case sensitive):\n"
    "  TREG    - Timestamped Register (Latest Write Wins)\n"
    "  TLOG    - Timestamped Log (Retain Latest Entries)\n"
    "  GCOUNT  - Grow-Only Counter\n"
    "  PNCOUNT - Positive/Negative Counter\n"
    "  UJSON   - Unordered JSON (Nested Observed-Remove Maps and Sets)\n"
    "  SYSTEM  - (miscellaneous system-level operations)";

void help_respond(Respond& r, const std::string& help) {  // help.pony:4-7
  std::string h = help;
  while (!h.empty() && (h.back() == '\n' || h.back() == ' ')) h.pop_back();
  r.err("BADCOMMAND (could not parse command)\n" + h);
}

}  // namespace

struct jyh_db {
  Eng eng;
  std::map<std::string, std::unique_ptr<Repo>> repos;  // database.pony:18-22
  bool shutdown = false;
  std::string err;
};

extern "C" {

int32_t jyh_db_create(int32_t device, uint64_t identity, jyh_db** out) {
  *out = nullptr;
  jy_config cfg;
  jy_config_default(&cfg);
  cfg.device = device;
  jy_engine* e = nullptr;
  const int32_t rc = jy_engine_create(&cfg, &e);
  if (rc != JY_OK) return rc;
  jyh_db* db = new jyh_db();
  db->eng.e = e;
  auto add = [&](Repo* r) {
    r->eng = &db->eng;
    r->identity = identity;
    db->repos[r->datatype()] = std::unique_ptr<Repo>(r);
  };
  add(new RepoTREG());
  add(new RepoTLOG());
  add(new RepoGCOUNT());
  add(new RepoPNCOUNT());
  *out = db;
  return JY_OK;
}

void jyh_db_destroy(jyh_db* db) {
  if (!db) return;
  jy_engine_destroy(db->eng.e);
  delete db;
}

const char* jyh_db_error(const jyh_db* db) { return db ? db->err.c_str() : "null"; }

int32_t jyh_db_apply(jyh_db* db, uint32_t argc, const char* const* argv, const uint64_t* lens, uint8_t* out,
                     uint64_t cap, uint64_t* out_len) {
  std::vector<std::string> w;
  for (u32 i = 0; i < argc; i++) w.emplace_back(argv[i], lens[i]);
  Respond r;
  try {
    auto it = w.empty() ? db->repos.end() : db->repos.find(w[0]);
    if (it == db->repos.end()) {
      help_respond(r, kDatabaseHelp);  // database.pony:25-40
    } else if (db->shutdown) {         // repo_manager.pony:50-54
      r.err("SHUTDOWN (server is shutting down, rejecting all requests)");
    } else {
      Cmd c{w, 1};
      try {
        it->second->apply(r, c);  // repo_manager.pony:56-61
      } catch (BadCommand&) {
        Respond rr;
        Cmd h{w, 1};
        help_respond(rr, it->second->help(h));  // repo_manager.pony:62-65
        r = rr;
      }
    }
  } catch (EngineError& e) {
    db->err = e.what();
    return JY_EHIP;
  }
  *out_len = r.out.size();
  if (r.out.size() > cap) return JY_ERANGE;
  std::memcpy(out, r.out.data(), r.out.size());
  return JY_OK;
}

int32_t jyh_db_flush(jyh_db* db, uint8_t** out, uint64_t* len) {
  Writer w;
  std::vector<Batch> bs;
  for (auto& kv : db->repos)
    if (kv.second->deltas_size() > 0) bs.push_back(kv.second->flush_deltas());  // repo_manager.pony:86-90
  w.u32v((u32)bs.size());
  for (auto& b : bs) write_batch(w, b);
  *len = w.b.size();
  *out = static_cast<uint8_t*>(std::malloc(w.b.size() ? w.b.size() : 1));
  std::memcpy(*out, w.b.data(), w.b.size());
  return JY_OK;
}

int32_t jyh_db_converge(jyh_db* db, const uint8_t* blob, uint64_t len) {
  try {
    Reader r{blob, blob + len};
    for (u32 n = r.u32v(); n; n--) {
      Batch b = read_batch(r);
      auto it = db->repos.find(b.type);  // database.pony:50-51 routes on the type name
      if (it != db->repos.end()) it->second->converge_batch(b);
    }
  } catch (BadCommand&) {
    db->err = "malformed delta blob";
    return JY_EINVAL;
  } catch (EngineError& e) {
    db->err = e.what();
    return JY_EHIP;
  }
  return JY_OK;
}

int32_t jyh_db_shutdown(jyh_db* db) {
  db->shutdown = true;
  return JY_OK;
}

void jyh_free(void* p) { std::free(p); }

}  // extern "C"
