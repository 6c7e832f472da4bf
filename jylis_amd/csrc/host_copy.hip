// host_copy.hip -- parallel host copies for the pinned staging ring.
//
// A host batch (a decoded peer batch handed over as plain host pointers:
// key strings, slots, columns, values) reaches HBM through the engine's
// pinned ring: a host copy into pinned memory, then a DMA.  One thread
// copies ~10-20 GB/s, below the PCIe link, so for large batches the copy,
// not the link, was the e2e ingest bound (round-2/3 e2e line: 1.2 ms of a
// 2.2 ms step).  Here the copy is cut into chunks that a small pool of
// worker threads (and the calling thread) take in order; the caller issues
// each chunk's DMA as soon as the chunks before it are done, so the link
// starts while later chunks are still being copied.
//
// Host-only code.  One pool per process, shared by every engine (a caller
// holds it for the duration of one copy); JY_COPY_THREADS sets the number
// of workers (default 6; 0 = copy on the calling thread only).

#include <atomic>
#include <immintrin.h>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "jy_internal.hpp"

namespace {

constexpr u64 kChunk = 1ull << 20;       // bytes per chunk
constexpr u64 kParallelMin = 2ull << 20;  // smaller copies stay on the calling thread

class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool* p = new CopyPool();  // never destroyed: workers sleep until exit
    return *p;
  }

  int workers() const { return (int)th_.size(); }

  // copy [src, src + bytes) to dst; issue(off, len) is called on the calling
  // thread, in order, for each run of chunks copied since the last call
  template <class F>
  int32_t run(uint8_t* dst, const uint8_t* src, u64 bytes, F&& issue) {
    std::lock_guard<std::mutex> use(use_mu_);
    const u64 nch = (bytes + kChunk - 1) / kChunk;
    if (done_.size() < nch) done_ = std::vector<std::atomic<u32>>(nch);
    u64 g;
    {
      std::lock_guard<std::mutex> lk(mu_);
      g = ++gen_;
      job_ = Job{dst, src, bytes, nch};
      // the chunk counter carries the job's generation: a worker still
      // holding an older job can never claim one of this job's chunks
      next_.store(g << kGenShift, std::memory_order_release);
    }
    cv_.notify_all();
    const Job j = job_;
    const u32 tag = (u32)g;
    u64 issued = 0;
    int32_t rc = JY_OK;
    for (;;) {
      u64 c;
      if (claim(g, nch, c)) copy_chunk(j, c, tag);
      else if (issued < nch) std::this_thread::yield();
      // every copied chunk from `issued` on goes out in ONE DMA: the link
      // idles ~10 us between two DMAs (1-MB DMAs: 24.7 us each, one every
      // ~35 us, ~30 GB/s), so the chunks the pool has finished meanwhile ride
      // together
      u64 k = issued;
      while (k < nch && done_[k].load(std::memory_order_acquire) == tag) k++;
      if (k > issued) {
        const u64 off = issued * kChunk, end = std::min<u64>(k * kChunk, bytes);
        if (rc == JY_OK) rc = issue(off, end - off);
        issued = k;
      }
      if (issued == nch) break;
    }
    return rc;
  }

 private:
  CopyPool() {
    int n = 6;
    if (const char* e = std::getenv("JY_COPY_THREADS")) n = std::max(0, std::atoi(e));
    const unsigned hw = std::thread::hardware_concurrency();
    if (hw && (unsigned)n > hw - 1) n = (int)(hw > 1 ? hw - 1 : 0);
    for (int i = 0; i < n; i++) th_.emplace_back([this] { loop(); });
    for (auto& t : th_) t.detach();
  }

  struct Job {
    uint8_t* dst;
    const uint8_t* src;
    u64 bytes, nch;
  };
  static constexpr int kGenShift = 40;

  // take the next chunk of job generation g (false: none left, or another job)
  bool claim(u64 g, u64 nch, u64& c) {
    u64 v = next_.load(std::memory_order_acquire);
    for (;;) {
      if ((v >> kGenShift) != g || (v & ((1ull << kGenShift) - 1)) >= nch) return false;
      if (next_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) {
        c = v & ((1ull << kGenShift) - 1);
        return true;
      }
    }
  }

  void copy_chunk(const Job& j, u64 c, u32 tag) {
    const u64 off = c * kChunk;
    std::memcpy(j.dst + off, j.src + off, std::min<u64>(kChunk, j.bytes - off));
    // memcpy may use weakly ordered (non-temporal / fast-string) stores,
    // which a release store does not order: fence them, so that the DMA the
    // calling thread enqueues once it sees `done` reads the copied bytes
    _mm_sfence();
    done_[c].store(tag, std::memory_order_release);
  }

  void loop() {
    u64 seen = 0;
    for (;;) {
      Job j;
      u64 g;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = g = gen_;
        j = job_;
      }
      u64 c;
      while (claim(g, j.nch, c)) copy_chunk(j, c, (u32)g);
    }
  }

  std::vector<std::thread> th_;
  std::mutex use_mu_, mu_;
  std::condition_variable cv_;
  u64 gen_ = 0;
  Job job_{};
  std::atomic<u64> next_{0};
  std::vector<std::atomic<u32>> done_;
};

}  // namespace

// host -> pinned -> device in chunks: the copied chunks' DMA is enqueued on
// the engine stream as soon as they (and every chunk before them) are copied
int32_t jy_copy_h2d_staged(jy_engine* eng, void* dev, uint8_t* pinned, const void* src, u64 bytes) {
  const uint8_t* s = static_cast<const uint8_t*>(src);
  uint8_t* d = static_cast<uint8_t*>(dev);
  CopyPool& pool = CopyPool::get();
  const double t0 = jy_tracing() ? jy_now_us() : 0;
  if (bytes < kParallelMin || pool.workers() == 0) {
    std::memcpy(pinned, s, bytes);
    JY_HIP(eng, hipMemcpyAsync(d, pinned, bytes, hipMemcpyHostToDevice, eng->stream));
    return JY_OK;
  }
  const int32_t rc = pool.run(pinned, s, bytes, [&](u64 off, u64 len) -> int32_t {
    JY_HIP(eng, hipMemcpyAsync(d + off, pinned + off, len, hipMemcpyHostToDevice, eng->stream));
    return JY_OK;
  });
  JY_TRACE("h2d staged %llu B in %.1f us (%d workers)", (unsigned long long)bytes, jy_now_us() - t0, pool.workers());
  return rc;
}

// pinned -> host, parallel (a device result already landed in pinned memory)
void jy_copy_host(void* dst, const void* src, u64 bytes) {
  CopyPool& pool = CopyPool::get();
  if (bytes < kParallelMin || pool.workers() == 0) {
    std::memcpy(dst, src, bytes);
    return;
  }
  pool.run(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), bytes, [](u64, u64) { return JY_OK; });
}
