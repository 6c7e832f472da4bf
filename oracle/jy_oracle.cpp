// jy_oracle.cpp -- CPU restatement of the Jylis converge path.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library, and only as the checker
// (or the timed CPU baseline).  The product path (jylis_amd/) never links it.
//
// What it restates
//   * RepoManagerCore.converge_deltas      jylis/repo_manager.pony:92-93
//     (serial per-key loop over Array[(String, Any box)])
//   * Repo{GCOUNT,PNCOUNT,TREG,TLOG,UJSON}.converge / _data_for / _delta_for /
//     flush_deltas and the write commands that produce deltas
//     (jylis/repo_gcount.pony, repo_pncount.pony, repo_treg.pony,
//      repo_tlog.pony, repo_ujson.pony)
//   * The merge arithmetic of the external library jemc/pony-crdt
//     (bundle.json:3-6, UNPINNED: no tag/commit, not vendored, no network).
//     Its published semantics are restated from the normative docs
//     docs/_docs/types/{gcount,pncount,treg,tlog,ujson}.md.
//
// Data structures deliberately mirror the reference's shape (hash map from
// String key to a CRDT object holding per-replica hash maps), because this
// file doubles as the CPU baseline of the bench (kind "port").
//
// Parity pinning (see DESIGN.md "Oracle"):
//   GCOUNT   pinned by the reference's only converge test,
//            jylis/test/test_cluster.pony:122-129 (INC 2,3,4 on 3 nodes -> 9)
//            and the gcount.md:30-41 example.
//   PNCOUNT  pinned by pncount.md:36-47 (10 - 15 = -5); merge internals
//            follow pncount.md:49-55.
//   TREG     pinned by treg.md:36-54; tie-break treg.md:58-63.
//   TLOG     pinned by tlog.md:70-114; merge tlog.md:116-133.
//   UJSON    dot-kernel join restated from ujson.md:172-182; the doc example
//            (ujson.md:107-132) pins only the observable element set.
//   Anything pony-crdt does beyond those documents is "parity unpinned".

#include <algorithm>
#include <deque>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <array>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

typedef uint64_t u64;
typedef int64_t i64;

namespace {

// ---------------------------------------------------------------------------
// Pony String ordering: unsigned bytewise, then the shorter string is less
// (Pony stdlib String.lt / String.compare; used by TReg/TLog tie-breaks).
int pony_str_cmp(const std::string& a, const std::string& b) {
  size_t n = a.size() < b.size() ? a.size() : b.size();
  int c = n ? std::memcmp(a.data(), b.data(), n) : 0;
  if (c != 0) return c < 0 ? -1 : 1;
  if (a.size() == b.size()) return 0;
  return a.size() < b.size() ? -1 : 1;
}

// ---------------------------------------------------------------------------
// GCounter -- gcount.md:43-47: map replica id -> u64; merge = per-id max.
// Write path: repo_gcount.pony:57-60 (delta records the post-increment total
// under the data counter's id).
struct GCounter {
  std::unordered_map<u64, u64> data;

  bool converge(const GCounter& that) {
    bool changed = false;
    for (const auto& kv : that.data) {
      auto it = data.find(kv.first);
      if (it == data.end()) {
        data.emplace(kv.first, kv.second);
        changed = true;
      } else if (kv.second > it->second) {
        it->second = kv.second;
        changed = true;
      }
    }
    return changed;
  }
  u64 value() const {  // wrapping sum (Pony U64 '+')
    u64 s = 0;
    for (const auto& kv : data) s += kv.second;
    return s;
  }
  void increment(u64 id, u64 v, GCounter& delta) {
    u64& cur = data[id];
    cur += v;
    delta.data[id] = cur;
  }
};

// PNCounter -- pncount.md:49-55: two GCounters merged separately;
// value = P - N (wrapping), read as i64 (repo_pncount.pony:56).
struct PNCounter {
  GCounter p, n;
  bool converge(const PNCounter& that) {
    bool a = p.converge(that.p);
    bool b = n.converge(that.n);
    return a || b;
  }
  u64 value() const { return p.value() - n.value(); }
};

// TRegString -- treg.md:58-63: (value, ts) replaced iff ts' > ts, or
// ts' == ts and value' > value (Pony String order).  Initial ("", 0)
// (repo_treg.pony:37-42 creates TRegString with no arguments).
struct TReg {
  std::string value;
  u64 ts = 0;
  bool update(const std::string& v, u64 t) {
    if (t > ts || (t == ts && pony_str_cmp(v, value) > 0)) {
      value = v;
      ts = t;
      return true;
    }
    return false;
  }
  bool converge(const TReg& that) { return update(that.value, that.ts); }
};

// TLog[String] -- tlog.md:116-133.  Entries kept sorted: later timestamp
// first, equal timestamps by greater value first; (ts, value) duplicates
// collapse; a grow-only cutoff removes entries with ts < cutoff.
struct TLogEntry {
  std::string value;
  u64 ts;
};
// true iff a sorts strictly before b (tlog.md:124-127)
inline bool tlog_before(const TLogEntry& a, const TLogEntry& b) {
  if (a.ts != b.ts) return a.ts > b.ts;
  return pony_str_cmp(a.value, b.value) > 0;
}

struct TLog {
  std::vector<TLogEntry> values;
  u64 cutoff = 0;

  // INS: ignored below the cutoff or when a duplicate (tlog.md:30-34)
  bool write(const std::string& v, u64 ts) {
    if (ts < cutoff) return false;
    TLogEntry e{v, ts};
    auto it = std::lower_bound(values.begin(), values.end(), e, tlog_before);
    if (it != values.end() && it->ts == ts && it->value == v) return false;
    values.insert(it, std::move(e));
    return true;
  }
  // TRIMAT: raise only (tlog.md:46-50, 129-133: strict '<' removes)
  bool raise_cutoff(u64 c) {
    if (c <= cutoff) return false;
    cutoff = c;
    while (!values.empty() && values.back().ts < c) values.pop_back();
    return true;
  }
  // CLR: cutoff = newest ts + 1 (U64 wrap as Pony); no-op if empty (tlog.md:60-64)
  bool clear() {
    if (values.empty()) return false;
    return raise_cutoff(values.front().ts + 1);
  }
  // TRIM n: cutoff = ts of entry n-1; n == 0 is CLR (tlog.md:52-58).  An
  // index past the end raises nothing (the Pony `try ... end` swallows the
  // out-of-bounds error) -- parity unpinned, documented in DESIGN.md.
  bool trim(size_t n) {
    if (n == 0) return clear();
    if (n - 1 >= values.size()) return false;
    return raise_cutoff(values[n - 1].ts);
  }
  bool converge(const TLog& that) {
    bool changed = raise_cutoff(that.cutoff);
    for (const auto& e : that.values) changed = write(e.value, e.ts) || changed;
    return changed;
  }
};

// ---------------------------------------------------------------------------
// UJSON -- ujson.md:172-182.  An observed-remove set of (path, value)
// elements, each tagged with a dot (replica id, seq), inside a causal
// context (version vector + dot cloud, compacted).  Elements are opaque
// u64 handles here: merge never inspects them (ujson.md:180-182).
struct Dot {
  u64 id, seq;
  bool operator==(const Dot& o) const { return id == o.id && seq == o.seq; }
  bool operator<(const Dot& o) const { return id != o.id ? id < o.id : seq < o.seq; }
};
struct DotHash {
  size_t operator()(const Dot& d) const {
    u64 x = d.id * 0x9E3779B97F4A7C15ull ^ (d.seq + 0x632BE59BD9B4E019ull);
    x ^= x >> 31;
    return (size_t)(x * 0xBF58476D1CE4E5B9ull);
  }
};

struct CausalContext {
  std::unordered_map<u64, u64> complete;  // id -> every seq <= n observed
  std::unordered_set<Dot, DotHash> cloud;  // observed dots beyond `complete`

  bool contains(const Dot& d) const {
    auto it = complete.find(d.id);
    if (it != complete.end() && d.seq <= it->second) return true;
    return cloud.count(d) != 0;
  }
  void compact() {
    bool progress = true;
    while (progress) {
      progress = false;
      for (auto it = cloud.begin(); it != cloud.end();) {
        u64 c = 0;
        auto ct = complete.find(it->id);
        if (ct != complete.end()) c = ct->second;
        if (it->seq <= c) {
          it = cloud.erase(it);
        } else if (it->seq == c + 1) {
          complete[it->id] = it->seq;
          it = cloud.erase(it);
          progress = true;
        } else {
          ++it;
        }
      }
    }
  }
  void insert(const Dot& d) {
    cloud.insert(d);
    compact();
  }
  Dot next_dot(u64 id) {
    u64& c = complete[id];
    // every dot the local replica issued is contiguous: compacted context
    c += 1;
    return Dot{id, c};
  }
  void converge(const CausalContext& that) {
    for (const auto& kv : that.complete) {
      u64& c = complete[kv.first];
      if (kv.second > c) c = kv.second;
    }
    for (const auto& d : that.cloud) cloud.insert(d);
    compact();
  }
};

struct UJSON {
  std::unordered_map<Dot, u64, DotHash> map;  // dot -> element handle
  CausalContext ctx;

  // Dot-kernel join (delta-state OR-set, ujson.md:176-182):
  //   keep local (d,e) unless that.ctx saw d and that.map lacks d;
  //   add that's (d,e) whose d the local context has not seen;
  //   context := union, compacted.
  bool converge(const UJSON& that) {
    bool changed = false;
    for (const auto& kv : that.map) {
      if (!ctx.contains(kv.first)) {
        map[kv.first] = kv.second;
        changed = true;
      }
    }
    for (auto it = map.begin(); it != map.end();) {
      if (that.ctx.contains(it->first) && that.map.count(it->first) == 0) {
        it = map.erase(it);
        changed = true;
      } else {
        ++it;
      }
    }
    ctx.converge(that.ctx);
    return changed;
  }
  // write path on opaque elements (INS / RM / CLR of a whole doc)
  void insert(u64 id, u64 elem, UJSON& delta) {
    Dot d = ctx.next_dot(id);
    map[d] = elem;
    delta.map[d] = elem;
    delta.ctx.insert(d);
  }
  void remove(u64 elem, UJSON& delta) {
    for (auto it = map.begin(); it != map.end();) {
      if (it->second == elem) {
        delta.ctx.insert(it->first);
        it = map.erase(it);
      } else {
        ++it;
      }
    }
  }
  void clear(UJSON& delta) {
    for (const auto& kv : map) delta.ctx.insert(kv.first);
    map.clear();
  }
};

enum { T_GCOUNT = 0, T_PNCOUNT = 1, T_TREG = 2, T_TLOG = 3, T_UJSON = 4 };

// ---------------------------------------------------------------------------
// A flat table of named arrays: the exchange format with the Python tests.
struct Field {
  std::string name;
  std::vector<uint8_t> bytes;
  size_t elem = 8;
};
struct Table {
  std::deque<Field> fields;  // deque: add() keeps earlier references valid
  Field& add(const std::string& n, size_t elem) {
    fields.push_back(Field{n, {}, elem});
    return fields.back();
  }
  const Field* get(const char* n) const {
    for (const auto& f : fields)
      if (f.name == n) return &f;
    return nullptr;
  }
};
template <class T>
void push(Field& f, T v) {
  size_t o = f.bytes.size();
  f.bytes.resize(o + sizeof(T));
  std::memcpy(f.bytes.data() + o, &v, sizeof(T));
}
void push_bytes(Field& f, const std::string& s) { f.bytes.insert(f.bytes.end(), s.begin(), s.end()); }
template <class T>
const T* arr(const Table& t, const char* n, size_t* count) {
  const Field* f = t.get(n);
  if (!f) {
    *count = 0;
    return nullptr;
  }
  *count = f->bytes.size() / sizeof(T);
  return reinterpret_cast<const T*>(f->bytes.data());
}

// ---------------------------------------------------------------------------
// Batch = Array[(String, Any box)] of one CRDT type (repo_manager.pony:92-93)
struct Batch {
  int type = -1;
  std::vector<std::string> keys;
  std::vector<GCounter> gc;
  std::vector<PNCounter> pn;
  std::vector<TReg> tr;
  std::vector<TLog> tl;
  std::vector<UJSON> uj;
  size_t size() const { return keys.size(); }
};

// Repo -- one per type, as RepoGCOUNT & co. (repo_*.pony): `_data` and
// `_deltas` maps from key to CRDT; converge goes through `_data_for`.
struct Repo {
  int type;
  u64 identity;
  std::unordered_map<std::string, GCounter> gc, gc_d;
  std::unordered_map<std::string, PNCounter> pn, pn_d;
  std::unordered_map<std::string, TReg> tr, tr_d;
  std::unordered_map<std::string, TLog> tl, tl_d;
  std::unordered_map<std::string, UJSON> uj, uj_d;
};

// RepoManagerCore.converge_deltas (repo_manager.pony:92-93) composed with
// Repo*.converge (repo_gcount.pony:50-51 etc.): `_data_for(key)` creates the
// key on a miss, then the CRDT converge.  A batch of another type is the
// swallowed `delta' as T box` failure: nothing happens.
void converge_batch(Repo& r, const Batch& b) {
  if (b.type != r.type) return;
  const size_t n = b.size();
  switch (r.type) {
    case T_GCOUNT:
      for (size_t i = 0; i < n; i++) r.gc[b.keys[i]].converge(b.gc[i]);
      break;
    case T_PNCOUNT:
      for (size_t i = 0; i < n; i++) r.pn[b.keys[i]].converge(b.pn[i]);
      break;
    case T_TREG:
      for (size_t i = 0; i < n; i++) r.tr[b.keys[i]].converge(b.tr[i]);
      break;
    case T_TLOG:
      for (size_t i = 0; i < n; i++) r.tl[b.keys[i]].converge(b.tl[i]);
      break;
    case T_UJSON:
      for (size_t i = 0; i < n; i++) r.uj[b.keys[i]].converge(b.uj[i]);
      break;
  }
}

template <class M>
std::vector<std::string> sorted_keys(const M& m) {
  std::vector<std::string> ks;
  ks.reserve(m.size());
  for (const auto& kv : m) ks.push_back(kv.first);
  std::sort(ks.begin(), ks.end());
  return ks;
}

// ---- export (state dump / flushed delta batch) to a Table -----------------
void export_keys(Table& t, const std::vector<std::string>& keys) {
  Field& kb = t.add("key_bytes", 1);
  Field& ko = t.add("key_offs", 8);
  u64 off = 0;
  push<u64>(ko, 0);
  for (const auto& k : keys) {
    push_bytes(kb, k);
    off += k.size();
    push<u64>(ko, off);
  }
}

void export_gcounter(Table& t, const char* pre, const std::vector<const GCounter*>& v) {
  std::string p(pre);
  Field& offs = t.add(p + "offs", 8);
  Field& ids = t.add(p + "ids", 8);
  Field& vals = t.add(p + "vals", 8);
  u64 off = 0;
  push<u64>(offs, 0);
  for (const GCounter* g : v) {
    std::vector<std::pair<u64, u64>> e(g->data.begin(), g->data.end());
    std::sort(e.begin(), e.end());
    for (auto& kv : e) {
      push<u64>(ids, kv.first);
      push<u64>(vals, kv.second);
    }
    off += e.size();
    push<u64>(offs, off);
  }
}

void export_treg(Table& t, const std::vector<const TReg*>& v) {
  Field& ts = t.add("ts", 8);
  Field& vb = t.add("val_bytes", 1);
  Field& vo = t.add("val_offs", 8);
  u64 off = 0;
  push<u64>(vo, 0);
  for (const TReg* r : v) {
    push<u64>(ts, r->ts);
    push_bytes(vb, r->value);
    off += r->value.size();
    push<u64>(vo, off);
  }
}

void export_tlog(Table& t, const std::vector<const TLog*>& v) {
  Field& co = t.add("cutoff", 8);
  Field& eo = t.add("ent_offs", 8);
  Field& ts = t.add("ts", 8);
  Field& vb = t.add("val_bytes", 1);
  Field& vo = t.add("val_offs", 8);
  u64 ne = 0, nb = 0;
  push<u64>(eo, 0);
  push<u64>(vo, 0);
  for (const TLog* l : v) {
    push<u64>(co, l->cutoff);
    for (const auto& e : l->values) {
      push<u64>(ts, e.ts);
      push_bytes(vb, e.value);
      nb += e.value.size();
      push<u64>(vo, nb);
    }
    ne += l->values.size();
    push<u64>(eo, ne);
  }
}

void export_ujson(Table& t, const std::vector<const UJSON*>& v) {
  Field& eo = t.add("el_offs", 8);
  Field& di = t.add("dot_ids", 8);
  Field& ds = t.add("dot_seqs", 8);
  Field& el = t.add("elems", 8);
  Field& vo = t.add("vv_offs", 8);
  Field& vi = t.add("vv_ids", 8);
  Field& vs = t.add("vv_seqs", 8);
  Field& co = t.add("cloud_offs", 8);
  Field& ci = t.add("cloud_ids", 8);
  Field& cs = t.add("cloud_seqs", 8);
  u64 ne = 0, nv = 0, nc = 0;
  push<u64>(eo, 0);
  push<u64>(vo, 0);
  push<u64>(co, 0);
  for (const UJSON* u : v) {
    std::vector<std::pair<Dot, u64>> e(u->map.begin(), u->map.end());
    std::sort(e.begin(), e.end(), [](const std::pair<Dot, u64>& a, const std::pair<Dot, u64>& b) { return a.first < b.first; });
    for (auto& kv : e) {
      push<u64>(di, kv.first.id);
      push<u64>(ds, kv.first.seq);
      push<u64>(el, kv.second);
    }
    ne += e.size();
    push<u64>(eo, ne);
    std::vector<std::pair<u64, u64>> vv;
    for (const auto& kv : u->ctx.complete)
      if (kv.second != 0) vv.push_back(kv);
    std::sort(vv.begin(), vv.end());
    for (auto& kv : vv) {
      push<u64>(vi, kv.first);
      push<u64>(vs, kv.second);
    }
    nv += vv.size();
    push<u64>(vo, nv);
    std::vector<Dot> cl(u->ctx.cloud.begin(), u->ctx.cloud.end());
    std::sort(cl.begin(), cl.end());
    for (auto& d : cl) {
      push<u64>(ci, d.id);
      push<u64>(cs, d.seq);
    }
    nc += cl.size();
    push<u64>(co, nc);
  }
}

template <class M, class T>
std::vector<const T*> ptrs_in_order(const M& m, const std::vector<std::string>& keys) {
  std::vector<const T*> v;
  v.reserve(keys.size());
  for (const auto& k : keys) v.push_back(&m.at(k));
  return v;
}

Table* export_state(const Repo& r) {
  Table* t = new Table();
  std::vector<std::string> keys;
  switch (r.type) {
    case T_GCOUNT: {
      keys = sorted_keys(r.gc);
      export_keys(*t, keys);
      export_gcounter(*t, "", ptrs_in_order<decltype(r.gc), GCounter>(r.gc, keys));
      break;
    }
    case T_PNCOUNT: {
      keys = sorted_keys(r.pn);
      export_keys(*t, keys);
      std::vector<const GCounter*> p, n;
      for (const auto& k : keys) {
        p.push_back(&r.pn.at(k).p);
        n.push_back(&r.pn.at(k).n);
      }
      export_gcounter(*t, "p_", p);
      export_gcounter(*t, "n_", n);
      break;
    }
    case T_TREG:
      keys = sorted_keys(r.tr);
      export_keys(*t, keys);
      export_treg(*t, ptrs_in_order<decltype(r.tr), TReg>(r.tr, keys));
      break;
    case T_TLOG:
      keys = sorted_keys(r.tl);
      export_keys(*t, keys);
      export_tlog(*t, ptrs_in_order<decltype(r.tl), TLog>(r.tl, keys));
      break;
    case T_UJSON:
      keys = sorted_keys(r.uj);
      export_keys(*t, keys);
      export_ujson(*t, ptrs_in_order<decltype(r.uj), UJSON>(r.uj, keys));
      break;
  }
  return t;
}

Table* export_batch(const Batch& b) {
  Table* t = new Table();
  export_keys(*t, b.keys);
  std::vector<size_t> idx(b.size());
  for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
  switch (b.type) {
    case T_GCOUNT: {
      std::vector<const GCounter*> v;
      for (auto i : idx) v.push_back(&b.gc[i]);
      export_gcounter(*t, "", v);
      break;
    }
    case T_PNCOUNT: {
      std::vector<const GCounter*> p, n;
      for (auto i : idx) {
        p.push_back(&b.pn[i].p);
        n.push_back(&b.pn[i].n);
      }
      export_gcounter(*t, "p_", p);
      export_gcounter(*t, "n_", n);
      break;
    }
    case T_TREG: {
      std::vector<const TReg*> v;
      for (auto i : idx) v.push_back(&b.tr[i]);
      export_treg(*t, v);
      break;
    }
    case T_TLOG: {
      std::vector<const TLog*> v;
      for (auto i : idx) v.push_back(&b.tl[i]);
      export_tlog(*t, v);
      break;
    }
    case T_UJSON: {
      std::vector<const UJSON*> v;
      for (auto i : idx) v.push_back(&b.uj[i]);
      export_ujson(*t, v);
      break;
    }
  }
  return t;
}

// ---- import a Table as a delta batch (the decoded MsgPushDeltas payload) ---
void import_gcounters(const Table& t, const char* pre, size_t nkeys, std::vector<GCounter*>& out) {
  std::string p(pre);
  size_t no, ni, nv;
  const u64* offs = arr<u64>(t, (p + "offs").c_str(), &no);
  const u64* ids = arr<u64>(t, (p + "ids").c_str(), &ni);
  const u64* vals = arr<u64>(t, (p + "vals").c_str(), &nv);
  if (!offs || no != nkeys + 1) return;
  for (size_t k = 0; k < nkeys; k++)
    for (u64 j = offs[k]; j < offs[k + 1] && j < ni && j < nv; j++) {
      // a delta holds at most one value per replica id (Map[ID, U64]); a
      // repeated id keeps the larger, as the map write would after max-merge
      u64& cur = out[k]->data[ids[j]];
      if (vals[j] > cur) cur = vals[j];
    }
}

Batch* import_batch(int type, const Table& t) {
  Batch* b = new Batch();
  b->type = type;
  size_t nkb, nko;
  const uint8_t* kb = arr<uint8_t>(t, "key_bytes", &nkb);
  const u64* ko = arr<u64>(t, "key_offs", &nko);
  if (!ko || nko == 0) return b;
  size_t n = nko - 1;
  b->keys.resize(n);
  for (size_t i = 0; i < n; i++) b->keys[i].assign(reinterpret_cast<const char*>(kb) + ko[i], ko[i + 1] - ko[i]);
  switch (type) {
    case T_GCOUNT: {
      b->gc.resize(n);
      std::vector<GCounter*> v;
      for (auto& g : b->gc) v.push_back(&g);
      import_gcounters(t, "", n, v);
      break;
    }
    case T_PNCOUNT: {
      b->pn.resize(n);
      std::vector<GCounter*> p, q;
      for (auto& g : b->pn) {
        p.push_back(&g.p);
        q.push_back(&g.n);
      }
      import_gcounters(t, "p_", n, p);
      import_gcounters(t, "n_", n, q);
      break;
    }
    case T_TREG: {
      b->tr.resize(n);
      size_t nts, nvb, nvo;
      const u64* ts = arr<u64>(t, "ts", &nts);
      const uint8_t* vb = arr<uint8_t>(t, "val_bytes", &nvb);
      const u64* vo = arr<u64>(t, "val_offs", &nvo);
      for (size_t i = 0; i < n; i++) {
        b->tr[i].ts = ts[i];
        b->tr[i].value.assign(reinterpret_cast<const char*>(vb) + vo[i], vo[i + 1] - vo[i]);
      }
      break;
    }
    case T_TLOG: {
      b->tl.resize(n);
      size_t x;
      const u64* co = arr<u64>(t, "cutoff", &x);
      const u64* eo = arr<u64>(t, "ent_offs", &x);
      const u64* ts = arr<u64>(t, "ts", &x);
      const uint8_t* vb = arr<uint8_t>(t, "val_bytes", &x);
      const u64* vo = arr<u64>(t, "val_offs", &x);
      for (size_t i = 0; i < n; i++) {
        TLog& l = b->tl[i];
        // a decoded TLog is canonical by construction: rebuild it through
        // its own write path so the invariant holds whatever the table says
        l.cutoff = co[i];
        for (u64 j = eo[i]; j < eo[i + 1]; j++)
          l.write(std::string(reinterpret_cast<const char*>(vb) + vo[j], vo[j + 1] - vo[j]), ts[j]);
      }
      break;
    }
    case T_UJSON: {
      b->uj.resize(n);
      size_t x;
      const u64* eo = arr<u64>(t, "el_offs", &x);
      const u64* di = arr<u64>(t, "dot_ids", &x);
      const u64* ds = arr<u64>(t, "dot_seqs", &x);
      const u64* el = arr<u64>(t, "elems", &x);
      const u64* vo = arr<u64>(t, "vv_offs", &x);
      const u64* vi = arr<u64>(t, "vv_ids", &x);
      const u64* vs = arr<u64>(t, "vv_seqs", &x);
      const u64* co = arr<u64>(t, "cloud_offs", &x);
      const u64* ci = arr<u64>(t, "cloud_ids", &x);
      const u64* cs = arr<u64>(t, "cloud_seqs", &x);
      for (size_t i = 0; i < n; i++) {
        UJSON& u = b->uj[i];
        for (u64 j = vo[i]; j < vo[i + 1]; j++) {
          u64& c = u.ctx.complete[vi[j]];
          if (vs[j] > c) c = vs[j];
        }
        for (u64 j = co[i]; j < co[i + 1]; j++) u.ctx.cloud.insert(Dot{ci[j], cs[j]});
        u.ctx.compact();
        for (u64 j = eo[i]; j < eo[i + 1]; j++) u.map[Dot{di[j], ds[j]}] = el[j];
      }
      break;
    }
  }
  return b;
}

// flush_deltas (repo_gcount.pony:18-23 & co.): emit every pending delta, clear
template <class M, class V>
void flush_map(M& m, Batch* b, std::vector<V>& out) {
  for (const auto& k : sorted_keys(m)) {
    b->keys.push_back(k);
    out.push_back(m.at(k));
  }
  m.clear();
}

}  // namespace

// ===========================================================================
// C ABI (ctypes from tests/ and bench.py's cpu_baseline leg only)
extern "C" {

void* or_table_new() { return new Table(); }
void or_table_free(void* t) { delete static_cast<Table*>(t); }
void or_table_set(void* tp, const char* name, const void* data, u64 nbytes, u64 elem) {
  Table* t = static_cast<Table*>(tp);
  for (auto& f : t->fields)
    if (f.name == name) {
      f.bytes.assign((const uint8_t*)data, (const uint8_t*)data + nbytes);
      f.elem = elem;
      return;
    }
  Field& f = t->add(name, elem);
  f.bytes.assign((const uint8_t*)data, (const uint8_t*)data + nbytes);
}
u64 or_table_nfields(void* t) { return static_cast<Table*>(t)->fields.size(); }
const char* or_table_field_name(void* t, u64 i) { return static_cast<Table*>(t)->fields[i].name.c_str(); }
const void* or_table_field_data(void* t, u64 i) { return static_cast<Table*>(t)->fields[i].bytes.data(); }
u64 or_table_field_nbytes(void* t, u64 i) { return static_cast<Table*>(t)->fields[i].bytes.size(); }
u64 or_table_field_elem(void* t, u64 i) { return static_cast<Table*>(t)->fields[i].elem; }

void* or_repo_new(int32_t type, u64 identity) {
  Repo* r = new Repo();
  r->type = type;
  r->identity = identity;
  return r;
}
void or_repo_free(void* r) { delete static_cast<Repo*>(r); }
u64 or_repo_nkeys(void* rp) {
  Repo* r = static_cast<Repo*>(rp);
  switch (r->type) {
    case T_GCOUNT: return r->gc.size();
    case T_PNCOUNT: return r->pn.size();
    case T_TREG: return r->tr.size();
    case T_TLOG: return r->tl.size();
    case T_UJSON: return r->uj.size();
  }
  return 0;
}

void* or_batch_import(int32_t type, void* table) { return import_batch(type, *static_cast<Table*>(table)); }
void or_batch_free(void* b) { delete static_cast<Batch*>(b); }
u64 or_batch_size(void* b) { return static_cast<Batch*>(b)->size(); }
void* or_batch_export(void* b) { return export_batch(*static_cast<Batch*>(b)); }

// the hot loop: RepoManagerCore.converge_deltas (repo_manager.pony:92-93)
void or_converge(void* r, void* b) { converge_batch(*static_cast<Repo*>(r), *static_cast<Batch*>(b)); }

void* or_state_export(void* r) { return export_state(*static_cast<Repo*>(r)); }

// flush_deltas: returns a Batch (possibly empty); the repo's deltas clear
void* or_flush(void* rp) {
  Repo* r = static_cast<Repo*>(rp);
  Batch* b = new Batch();
  b->type = r->type;
  switch (r->type) {
    case T_GCOUNT: flush_map(r->gc_d, b, b->gc); break;
    case T_PNCOUNT: flush_map(r->pn_d, b, b->pn); break;
    case T_TREG: flush_map(r->tr_d, b, b->tr); break;
    case T_TLOG: flush_map(r->tl_d, b, b->tl); break;
    case T_UJSON: flush_map(r->uj_d, b, b->uj); break;
  }
  return b;
}
u64 or_deltas_size(void* rp) {
  Repo* r = static_cast<Repo*>(rp);
  switch (r->type) {
    case T_GCOUNT: return r->gc_d.size();
    case T_PNCOUNT: return r->pn_d.size();
    case T_TREG: return r->tr_d.size();
    case T_TLOG: return r->tl_d.size();
    case T_UJSON: return r->uj_d.size();
  }
  return 0;
}

// ---- reads (repo_*.pony `get` & co.) ----
static std::string K(const char* k, u64 n) { return std::string(k, n); }

u64 or_gcount_get(void* rp, const char* k, u64 n) {  // repo_gcount.pony:53-55
  Repo* r = static_cast<Repo*>(rp);
  auto it = r->gc.find(K(k, n));
  return it == r->gc.end() ? 0 : it->second.value();
}
i64 or_pncount_get(void* rp, const char* k, u64 n) {  // repo_pncount.pony:55-57
  Repo* r = static_cast<Repo*>(rp);
  auto it = r->pn.find(K(k, n));
  return it == r->pn.end() ? 0 : (i64)it->second.value();
}
// returns 1 and fills ts / value if the key exists, 0 for nil (repo_treg.pony:54-63)
int32_t or_treg_get(void* rp, const char* k, u64 n, u64* ts, char* buf, u64 cap, u64* vlen) {
  Repo* r = static_cast<Repo*>(rp);
  auto it = r->tr.find(K(k, n));
  if (it == r->tr.end()) return 0;
  *ts = it->second.ts;
  *vlen = it->second.value.size();
  std::memcpy(buf, it->second.value.data(), std::min<u64>(cap, *vlen));
  return 1;
}
u64 or_tlog_size(void* rp, const char* k, u64 n) {  // repo_tlog.pony:90-92
  Repo* r = static_cast<Repo*>(rp);
  auto it = r->tl.find(K(k, n));
  return it == r->tl.end() ? 0 : it->second.values.size();
}
u64 or_tlog_cutoff(void* rp, const char* k, u64 n) {  // repo_tlog.pony:94-96
  Repo* r = static_cast<Repo*>(rp);
  auto it = r->tl.find(K(k, n));
  return it == r->tl.end() ? 0 : it->second.cutoff;
}

// ---- writes (delta producers) ----
void or_gcount_inc(void* rp, const char* k, u64 n, u64 v) {  // repo_gcount.pony:57-60
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n);
  r->gc[key].increment(r->identity, v, r->gc_d[key]);
}
void or_pncount_inc(void* rp, const char* k, u64 n, i64 v) {  // repo_pncount.pony:59-62
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n);
  r->pn[key].p.increment(r->identity, (u64)v, r->pn_d[key].p);
}
void or_pncount_dec(void* rp, const char* k, u64 n, i64 v) {  // repo_pncount.pony:64-67
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n);
  r->pn[key].n.increment(r->identity, (u64)v, r->pn_d[key].n);
}
void or_treg_set(void* rp, const char* k, u64 n, const char* v, u64 vn, u64 ts) {  // repo_treg.pony:65-68
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n), val(v, vn);
  if (r->tr[key].update(val, ts)) r->tr_d[key].update(val, ts);
  else r->tr_d[key];  // _delta_for(key) is evaluated by the call either way
}
void or_tlog_ins(void* rp, const char* k, u64 n, const char* v, u64 vn, u64 ts) {  // repo_tlog.pony:85-88
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n), val(v, vn);
  TLog& d = r->tl_d[key];
  if (r->tl[key].write(val, ts)) d.write(val, ts);
}
void or_tlog_trimat(void* rp, const char* k, u64 n, u64 ts) {  // repo_tlog.pony:98-101
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n);
  TLog& d = r->tl_d[key];
  TLog& l = r->tl[key];
  if (l.raise_cutoff(ts)) d.raise_cutoff(ts);
}
void or_tlog_trim(void* rp, const char* k, u64 n, u64 count) {  // repo_tlog.pony:103-106
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n);
  TLog& d = r->tl_d[key];
  TLog& l = r->tl[key];
  if (l.trim(count)) d.raise_cutoff(l.cutoff);
}
void or_tlog_clr(void* rp, const char* k, u64 n) {  // repo_tlog.pony:108-111
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n);
  TLog& d = r->tl_d[key];
  TLog& l = r->tl[key];
  if (l.clear()) d.raise_cutoff(l.cutoff);
}
void or_ujson_ins(void* rp, const char* k, u64 n, u64 elem) {  // repo_ujson.pony:90-99
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n);
  r->uj[key].insert(r->identity, elem, r->uj_d[key]);
}
void or_ujson_rm(void* rp, const char* k, u64 n, u64 elem) {  // repo_ujson.pony:101-110 (no key creation)
  Repo* r = static_cast<Repo*>(rp);
  auto it = r->uj.find(K(k, n));
  if (it != r->uj.end()) it->second.remove(elem, r->uj_d[it->first]);
}
void or_ujson_clr(void* rp, const char* k, u64 n) {  // repo_ujson.pony:85-88 (no key creation)
  Repo* r = static_cast<Repo*>(rp);
  auto it = r->uj.find(K(k, n));
  if (it != r->uj.end()) it->second.clear(r->uj_d[it->first]);
}
// _data_for(key) + _delta_for(key) with no change: SET of an empty node
// (repo_ujson.pony:80-81), a path-scoped CLR that matches nothing (:86)
void or_ujson_touch(void* rp, const char* k, u64 n) {
  Repo* r = static_cast<Repo*>(rp);
  std::string key = K(k, n);
  r->uj[key];
  r->uj_d[key];
}

// ---- canonical state digests (the full-size pins of tests/golden) ----------
// A digest is a wrapping sum over keys of per-key digests, so it does not
// depend on key or slot order; inside a key a TLOG is a LIST (entry rank in
// the canonical newest-first order is part of an entry's hash) and UJSON
// elements, version-vector entries and cloud dots are SETS (summed).  Three
// entry points compute the same digest: from the oracle's own maps
// (or_digest_repo), from an oracle-format table (or_digest_table) and from
// the engine's read-back arrays (or_digest_tlog_handles / _ujson_packed);
// tests/test_digest.py checks they agree.  out4 = {digest, keys, entries or
// elements, bytes or cloud dots}.
}  // extern "C"

namespace {
inline u64 dmix(u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
inline u64 dcomb(u64 a, u64 b) { return dmix(a ^ dmix(b)); }
inline u64 dbytes(const uint8_t* p, u64 n) {
  u64 h = 0xCBF29CE484222325ull;
  for (u64 i = 0; i < n; i++) {
    h ^= p[i];
    h *= 0x100000001B3ull;
  }
  return dcomb(h, n);
}
enum : u64 { kTagLog = 0x7100, kTagEnt = 0x7200, kTagDoc = 0x7300, kTagEl = 0x7400, kTagVV = 0x7500, kTagCl = 0x7600,
             kTagReg = 0x7700, kTagCnt = 0x7800, kTagCell = 0x7900 };
inline u64 d_reg(u64 kh, u64 ts, u64 vh) { return dcomb(kh, dcomb(kTagReg, dcomb(ts, vh))); }
inline u64 d_log(u64 kh, u64 cutoff) { return dcomb(kh, dcomb(kTagLog, cutoff)); }
inline u64 d_ent(u64 kh, u64 rank, u64 ts, u64 vh) { return dcomb(kh, dcomb(kTagEnt ^ (rank << 16), dcomb(ts, vh))); }
inline u64 d_doc(u64 kh) { return dcomb(kh, kTagDoc); }
inline u64 d_el(u64 kh, u64 id, u64 seq, u64 elem) { return dcomb(kh, dcomb(kTagEl, dcomb(id, dcomb(seq, elem)))); }
inline u64 d_vv(u64 kh, u64 id, u64 n) { return dcomb(kh, dcomb(kTagVV, dcomb(id, n))); }
inline u64 d_cl(u64 kh, u64 id, u64 seq) { return dcomb(kh, dcomb(kTagCl, dcomb(id, seq))); }
inline u64 dstr(const std::string& s) { return dbytes(reinterpret_cast<const uint8_t*>(s.data()), s.size()); }
// counters: a key, and each (sign, replica id, value) entry with a value
// other than 0 -- a 0 entry and an absent one read alike (max and sum), and
// the engine's dense columns cannot tell them apart
inline u64 d_cnt(u64 kh) { return dcomb(kh, kTagCnt); }
inline u64 d_cell(u64 kh, u64 sign, u64 id, u64 v) { return dcomb(kh, dcomb(kTagCell ^ (sign << 16), dcomb(id, v))); }
}  // namespace

extern "C" {

int32_t or_digest_repo(void* rp, u64* out4) {
  const Repo& r = *static_cast<Repo*>(rp);
  u64 d = 0, nk = 0, ni = 0, nb = 0;
  if (r.type == T_GCOUNT || r.type == T_PNCOUNT) {  // nb: the wrapping sum of every entry
    auto cells = [&](u64 kh, u64 sign, const GCounter& g) {
      for (const auto& kv : g.data)
        if (kv.second) {
          d += d_cell(kh, sign, kv.first, kv.second);
          nb += kv.second;
          ni++;
        }
    };
    if (r.type == T_GCOUNT)
      for (const auto& kv : r.gc) {
        const u64 kh = dstr(kv.first);
        d += d_cnt(kh);
        cells(kh, 0, kv.second);
        nk++;
      }
    else
      for (const auto& kv : r.pn) {
        const u64 kh = dstr(kv.first);
        d += d_cnt(kh);
        cells(kh, 0, kv.second.p);
        cells(kh, 1, kv.second.n);
        nk++;
      }
  } else if (r.type == T_TREG) {  // one (ts, value) register per key
    for (const auto& kv : r.tr) {
      d += d_reg(dstr(kv.first), kv.second.ts, dstr(kv.second.value));
      nb += kv.second.value.size();
      nk++;
    }
    ni = nk;
  } else if (r.type == T_TLOG) {
    for (const auto& kv : r.tl) {
      const u64 kh = dstr(kv.first);
      d += d_log(kh, kv.second.cutoff);
      u64 rank = 0;
      for (const auto& e : kv.second.values) {
        d += d_ent(kh, rank++, e.ts, dstr(e.value));
        nb += e.value.size();
      }
      ni += kv.second.values.size();
      nk++;
    }
  } else if (r.type == T_UJSON) {
    for (const auto& kv : r.uj) {
      const u64 kh = dstr(kv.first);
      d += d_doc(kh);
      for (const auto& e : kv.second.map) d += d_el(kh, e.first.id, e.first.seq, e.second);
      for (const auto& c : kv.second.ctx.complete)
        if (c.second) d += d_vv(kh, c.first, c.second);
      for (const auto& c : kv.second.ctx.cloud) d += d_cl(kh, c.id, c.seq);
      ni += kv.second.map.size();
      nb += kv.second.ctx.cloud.size();
      nk++;
    }
  } else {
    return -1;
  }
  out4[0] = d;
  out4[1] = nk;
  out4[2] = ni;
  out4[3] = nb;
  return 0;
}

// the engine's dense counter read-back: n keys (kb / ko), vals[(sign * ncols
// + col) * pitch + i] with column col holding replica ids[col]; the same
// digest as or_digest_repo of a GCOUNT (nsigns 1) / PNCOUNT (2) repo holding
// those keys.  Key ranges digest on up to `threads` threads (a full-size
// config-2 state is 2^31 cells).
int32_t or_digest_counter_dense(u64 n, const uint8_t* kb, const u64* ko, uint32_t nsigns, uint32_t ncols, const u64* ids,
                                const u64* vals, u64 pitch, uint32_t threads, u64* out4) {
  if (nsigns < 1 || nsigns > 2) return -1;
  const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(threads, 64));
  std::vector<std::array<u64, 4>> part(T, std::array<u64, 4>{0, 0, 0, 0});
  auto work = [&](uint32_t t) {
    const u64 a = n * t / T, b = n * (t + 1) / T;
    u64 d = 0, ni = 0, nb = 0;
    for (u64 i = a; i < b; i++) {
      const u64 kh = dbytes(kb + ko[i], ko[i + 1] - ko[i]);
      d += d_cnt(kh);
      for (uint32_t sg = 0; sg < nsigns; sg++)
        for (uint32_t c = 0; c < ncols; c++) {
          const u64 v = vals[((u64)sg * ncols + c) * pitch + i];
          if (v) {
            d += d_cell(kh, sg, ids[c], v);
            nb += v;
            ni++;
          }
        }
    }
    part[t] = {d, b - a, ni, nb};
  };
  std::vector<std::thread> th;
  for (uint32_t t = 1; t < T; t++) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  u64 o[4] = {0, 0, 0, 0};
  for (const auto& p : part)
    for (int q = 0; q < 4; q++) o[q] += p[q];
  std::memcpy(out4, o, sizeof(o));
  return 0;
}

int32_t or_digest_table(int32_t type, void* tp, u64* out4) {
  const Table& t = *static_cast<Table*>(tp);
  size_t nkb, nko;
  const uint8_t* kb = arr<uint8_t>(t, "key_bytes", &nkb);
  const u64* ko = arr<u64>(t, "key_offs", &nko);
  if (!ko || nko == 0) return -1;
  const u64 n = nko - 1;
  u64 d = 0, ni = 0, nb = 0;
  if (type == T_TREG) {
    size_t a, e, f;
    const u64* ts = arr<u64>(t, "ts", &a);
    const uint8_t* vb = arr<uint8_t>(t, "val_bytes", &e);
    const u64* vo = arr<u64>(t, "val_offs", &f);
    for (u64 i = 0; i < n; i++)
      d += d_reg(dbytes(kb + ko[i], ko[i + 1] - ko[i]), ts[i], dbytes(vb + vo[i], vo[i + 1] - vo[i]));
    ni = n;
    nb = vo[n];
  } else if (type == T_TLOG) {
    size_t a, b, c, e, f;
    const u64* cut = arr<u64>(t, "cutoff", &a);
    const u64* eo = arr<u64>(t, "ent_offs", &b);
    const u64* ts = arr<u64>(t, "ts", &c);
    const uint8_t* vb = arr<uint8_t>(t, "val_bytes", &e);
    const u64* vo = arr<u64>(t, "val_offs", &f);
    for (u64 i = 0; i < n; i++) {
      const u64 kh = dbytes(kb + ko[i], ko[i + 1] - ko[i]);
      d += d_log(kh, cut[i]);
      for (u64 j = eo[i]; j < eo[i + 1]; j++) d += d_ent(kh, j - eo[i], ts[j], dbytes(vb + vo[j], vo[j + 1] - vo[j]));
    }
    ni = eo[n];
    nb = vo[ni];
  } else if (type == T_UJSON) {
    size_t z;
    const u64 *eo = arr<u64>(t, "el_offs", &z), *di = arr<u64>(t, "dot_ids", &z), *dq = arr<u64>(t, "dot_seqs", &z),
              *el = arr<u64>(t, "elems", &z), *vo = arr<u64>(t, "vv_offs", &z), *vi = arr<u64>(t, "vv_ids", &z),
              *vs = arr<u64>(t, "vv_seqs", &z), *co = arr<u64>(t, "cloud_offs", &z),
              *ci = arr<u64>(t, "cloud_ids", &z), *cq = arr<u64>(t, "cloud_seqs", &z);
    for (u64 i = 0; i < n; i++) {
      const u64 kh = dbytes(kb + ko[i], ko[i + 1] - ko[i]);
      d += d_doc(kh);
      for (u64 j = eo[i]; j < eo[i + 1]; j++) d += d_el(kh, di[j], dq[j], el[j]);
      for (u64 j = vo[i]; j < vo[i + 1]; j++)
        if (vs[j]) d += d_vv(kh, vi[j], vs[j]);
      for (u64 j = co[i]; j < co[i + 1]; j++) d += d_cl(kh, ci[j], cq[j]);
    }
    ni = eo[n];
    nb = co[n];
  } else {
    return -1;
  }
  out4[0] = d;
  out4[1] = n;
  out4[2] = ni;
  out4[3] = nb;
  return 0;
}

// the engine's TREG read-back: per key (ts, pre, lr) value handles (pre =
// first 8 bytes big-endian; lr = arena offset << 24 | length)
int32_t or_digest_treg_handles(u64 n, const uint8_t* kb, const u64* ko, const u64* ts, const u64* pre, const u64* lr,
                               const uint8_t* arena, u64 alen, u64* out4) {
  u64 d = 0, nb = 0;
  for (u64 i = 0; i < n; i++) {
    const u64 len = lr[i] & ((1ull << 24) - 1), off = lr[i] >> 24;
    u64 vh;
    if (len <= 8) {
      uint8_t b[8];
      for (int q = 0; q < 8; q++) b[q] = (uint8_t)(pre[i] >> (56 - 8 * q));
      vh = dbytes(b, len);
    } else {
      if (off + len > alen) return -2;
      vh = dbytes(arena + off, len);
    }
    d += d_reg(dbytes(kb + ko[i], ko[i + 1] - ko[i]), ts[i], vh);
    nb += len;
  }
  out4[0] = d;
  out4[1] = n;
  out4[2] = n;
  out4[3] = nb;
  return 0;
}

// the engine's TLOG read-back: entries newest first per key (offs), values as
// handles (pre = first 8 bytes big-endian; lr = arena offset << 24 | length)
int32_t or_digest_tlog_handles(u64 n, const uint8_t* kb, const u64* ko, const u64* cut, const u64* eo, const u64* ts,
                               const u64* pre, const u64* lr, const uint8_t* arena, u64 alen, u64* out4) {
  u64 d = 0, nb = 0;
  std::vector<uint8_t> buf;
  for (u64 i = 0; i < n; i++) {
    const u64 kh = dbytes(kb + ko[i], ko[i + 1] - ko[i]);
    d += d_log(kh, cut[i]);
    for (u64 j = eo[i]; j < eo[i + 1]; j++) {
      const u64 len = lr[j] & ((1ull << 24) - 1), off = lr[j] >> 24;
      u64 vh;
      if (len <= 8) {
        uint8_t b[8];
        for (int q = 0; q < 8; q++) b[q] = (uint8_t)(pre[j] >> (56 - 8 * q));
        vh = dbytes(b, len);
      } else {
        if (off + len > alen) return -2;
        vh = dbytes(arena + off, len);
      }
      d += d_ent(kh, j - eo[i], ts[j], vh);
      nb += len;
    }
  }
  out4[0] = d;
  out4[1] = n;
  out4[2] = eo[n];
  out4[3] = nb;
  return 0;
}

// the engine's UJSON read-back: dots packed (column << 48 | seq), vv dense
// [n][R] by column, col_ids[column] = the replica identity
int32_t or_digest_ujson_packed(u64 n, const uint8_t* kb, const u64* ko, const u64* eo, const u64* dots,
                               const u64* elems, const u64* vv, u64 R, const u64* co, const u64* cloud,
                               const u64* col_ids, u64 ncols, u64* out4) {
  const u64 mask = (1ull << 48) - 1;
  u64 d = 0;
  for (u64 i = 0; i < n; i++) {
    const u64 kh = dbytes(kb + ko[i], ko[i + 1] - ko[i]);
    d += d_doc(kh);
    for (u64 j = eo[i]; j < eo[i + 1]; j++) {
      const u64 c = dots[j] >> 48;
      if (c >= ncols) return -2;
      d += d_el(kh, col_ids[c], dots[j] & mask, elems[j]);
    }
    for (u64 c = 0; c < R; c++) {
      const u64 v = vv[i * R + c];
      if (!v) continue;
      if (c >= ncols) return -2;
      d += d_vv(kh, col_ids[c], v);
    }
    for (u64 j = co[i]; j < co[i + 1]; j++) {
      const u64 c = cloud[j] >> 48;
      if (c >= ncols) return -2;
      d += d_cl(kh, col_ids[c], cloud[j] & mask);
    }
  }
  out4[0] = d;
  out4[1] = n;
  out4[2] = eo[n];
  out4[3] = co[n];
  return 0;
}

}  // extern "C"
