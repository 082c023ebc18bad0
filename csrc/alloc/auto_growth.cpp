// Native auto-growth best-fit device allocator with stream-safe reuse
// (reference: paddle/phi/core/memory/allocation/auto_growth_best_fit_allocator.cc,
//             stream_safe_cuda_allocator.cc, retry_allocator.cc).
//
// Plugged into PyTorch-ROCm through torch.cuda.memory.CUDAPluggableAllocator (pd_alloc_malloc /
// pd_alloc_free), so every framework tensor on the device is carved from it.  Design, sized for 288 GB HBM3E:
//   * chunks: hipMalloc'd regions of max(request, chunk_size) bytes (chunk_size from
//     FLAGS_auto_growth_chunk_size_in_mb; default 256 MiB so a 7B training step lives in ~1k chunks, not 100k
//     hipMallocs); never returned to the driver except by pd_alloc_empty_cache / the OOM retry path;
//   * blocks: each chunk is an address-ordered doubly-linked list of blocks; free blocks are indexed in a
//     size-ordered multimap (best fit = lower_bound), split on allocation when the remainder is >= 1 KiB and
//     coalesced with free neighbours of the same stream on release;
//   * stream safety: a block remembers the stream it was freed on.  Reuse on that stream is ordered by the
//     stream itself.  Once a second stream has been seen, every free also records a HIP event, and a block is
//     handed to a different stream only after its event completed (hipEventQuery) — no host sync, no
//     cross-stream hazard;
//   * record_stream (stream_safe_cuda_allocator.cc RecordStream): a live block can be marked as used by other
//     streams (torch's Tensor.record_stream reaches pd_alloc_record_stream through the pluggable allocator's
//     record-stream hook).  Freeing such a block records an event on every one of those streams and on the
//     freeing stream and parks the block on a deferred list; it re-enters the free index only once all of its
//     events completed (polled, never waited for, at the next allocation);
//   * limit: an optional byte cap (FLAGS_fraction_of_gpu_memory_to_use / FLAGS_gpu_memory_limit_mb); on a
//     failed growth the cache of fully-free chunks is released and the growth retried once;
//   * headroom (opt-in, FLAGS_native_allocator_headroom_mb): a growth never leaves less than `g_headroom` bytes of
//     the device free (hipMemGetInfo at every growth), for the runtime's own later allocations;
//   * out of memory: one device sync settles every fence, the free index is coalesced and scanned in full, then
//     fully-free chunks go back to the driver for a last growth (see do_alloc_impl).
// Thread-safe (one mutex per device).  C ABI for ctypes; no Python dependency, loads on CPU-only machines.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace pd {
namespace alloc {

constexpr size_t kAlign = 256;          // HBM transaction / LDS-DMA friendly alignment
constexpr size_t kMinSplit = 1024;      // do not leave slivers smaller than this
constexpr int kMaxDevices = 64;
constexpr int kMaxScan = 64;            // candidates examined for a cross-stream reusable block
constexpr size_t kTailGuard = size_t(2) << 20;  // unused slack mapped after every chunk

struct Chunk;

struct Block {
  char* ptr;
  size_t size;
  size_t req;            // bytes the caller asked for (guard / canary bookkeeping)
  bool free;
  hipStream_t stream;
  hipEvent_t event;      // recorded at free time when more than one stream is in use
  bool event_pending;
  Chunk* chunk;
  Block* prev;
  Block* next;
  std::multimap<size_t, Block*>::iterator pos;  // position in the free index (valid when free)
  std::vector<hipStream_t> uses;                 // other streams recorded on the live block (record_stream)
};

// a freed block still in use by recorded streams: re-indexed once every event completed
struct Deferred {
  Block* b;
  hipStream_t stream;             // freeing stream
  std::vector<hipEvent_t> events;
};

struct Chunk {
  char* base;
  size_t size;
  Block* head;
};

struct Stats {
  uint64_t allocated = 0, reserved = 0, peak_allocated = 0, peak_reserved = 0;
  uint64_t num_allocs = 0, num_frees = 0, num_chunks = 0, num_grow = 0, num_oom_retries = 0;
  uint64_t cross_stream_reuse = 0;
  uint64_t record_stream = 0, deferred_frees = 0;
};

struct Device {
  std::mutex mu;
  std::multimap<size_t, Block*> free_index;
  std::unordered_map<void*, Block*> live;
  std::vector<Chunk*> chunks;
  std::vector<hipEvent_t> event_pool;
  std::vector<Deferred> deferred;
  hipStream_t first_stream = nullptr;
  bool seen_stream = false;
  bool multi_stream = false;
  Stats st;
};

// Immortal: torch frees the last tensors (MemPools, module globals) during interpreter teardown, after static
// destructors would have run — the per-device state must outlive every free.
static Device* const g_dev = new Device[kMaxDevices];
static size_t g_chunk_bytes = size_t(256) << 20;
// debug: every block gets g_guard extra bytes past the request; with g_canary the slack is filled with a
// pattern at allocation and verified at free, so a kernel writing past its tensor is reported (pointer,
// size, first bad offset) instead of silently corrupting the neighbour
static size_t g_guard = 0;
static bool g_canary = false;
constexpr unsigned char kCanary = 0xA5;
struct Violation {
  uint64_t ptr, req, offset;
};
static std::vector<Violation>& g_violations = *new std::vector<Violation>();
static uint64_t g_limit_bytes = 0;   // 0 = unlimited
static uint64_t g_headroom = 0;   // device bytes a growth leaves free for the runtime (0 = off)
static std::mutex& g_cfg_mu = *new std::mutex();

static inline size_t round_up(size_t n, size_t a) { return (n + a - 1) / a * a; }

static void process_deferred(Device& d);

static hipEvent_t take_event(Device& d) {
  if (!d.event_pool.empty()) {
    hipEvent_t e = d.event_pool.back();
    d.event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

static void give_event(Device& d, hipEvent_t e) {
  if (e) d.event_pool.push_back(e);
}

static void index_free(Device& d, Block* b) {
  b->free = true;
  b->pos = d.free_index.emplace(b->size, b);
}

static void unindex_free(Device& d, Block* b) {
  d.free_index.erase(b->pos);
  b->free = false;
}

// a free block may be used by `stream` now
static bool usable_on(Device& d, Block* b, hipStream_t stream) {
  if (!d.multi_stream || b->stream == stream) return true;
  if (!b->event_pending) return true;
  if (hipEventQuery(b->event) == hipSuccess) {
    b->event_pending = false;
    give_event(d, b->event);
    b->event = nullptr;
    return true;
  }
  return false;
}

// the work that last used free block b has finished (or is ordered before anything that can reuse it)
static bool fence_done(Device& d, Block* b) {
  if (!d.multi_stream || !b->event_pending) return true;  // unfenced free blocks are settled (see usable_on)
  if (hipEventQuery(b->event) == hipSuccess) {
    b->event_pending = false;
    give_event(d, b->event);
    b->event = nullptr;
    return true;
  }
  return false;
}

static Block* carve(Device& d, Block* b, size_t size, hipStream_t stream) {
  unindex_free(d, b);
  if (b->stream != stream) d.st.cross_stream_reuse++;
  // usable_on() guaranteed: same stream (ordered) or the free-time event has completed
  hipEvent_t ev = b->event;
  bool pending = b->event_pending;
  b->event = nullptr;
  b->event_pending = false;
  if (b->size - size >= kMinSplit) {
    // the remainder stays "freed on b's stream" and keeps its fence for other streams
    Block* rest = new Block{b->ptr + size, b->size - size, 0, true, b->stream, ev, pending, b->chunk, b, b->next, {}, {}};
    ev = nullptr;
    if (b->next) b->next->prev = rest;
    b->next = rest;
    b->size = size;
    index_free(d, rest);
  }
  give_event(d, ev);
  b->stream = stream;
  return b;
}

static bool grow(Device& d, int dev, size_t size, hipStream_t stream) {
  size_t bytes = size > g_chunk_bytes ? round_up(size, size_t(2) << 20) : g_chunk_bytes;
  if (g_limit_bytes && d.st.reserved + bytes > g_limit_bytes) {
    if (d.st.reserved + size > g_limit_bytes) return false;
    bytes = round_up(size, kAlign);  // last chunk below the cap: exactly what is asked
  }
  int prev_dev = -1;
  hipGetDevice(&prev_dev);
  if (prev_dev != dev) hipSetDevice(dev);
  if (g_headroom) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && total_b > 0) {
      const size_t exact = round_up(size, kAlign);
      if ((uint64_t)free_b < (uint64_t)bytes + kTailGuard + g_headroom) {
        // a full chunk would eat into the runtime's headroom: take only what is asked, if even that fits
        if ((uint64_t)free_b < (uint64_t)exact + kTailGuard + g_headroom) {
          if (prev_dev != dev) hipSetDevice(prev_dev);
          return false;
        }
        bytes = exact;
      }
    }
  }
  void* p = nullptr;
  // every chunk carries kTailGuard mapped-but-never-handed-out bytes: a kernel whose vector / tile loads run
  // a little past the end of the last tensor of a chunk reads guard memory instead of faulting on unmapped VA
  // (the caching allocator's rounding gives the same slack; tight packing exposed it on the 7B step)
  hipError_t err = hipMalloc(&p, bytes + kTailGuard);
  if (prev_dev != dev) hipSetDevice(prev_dev);
  if (err != hipSuccess || !p) {
    (void)hipGetLastError();
    return false;
  }
  Chunk* c = new Chunk{static_cast<char*>(p), bytes, nullptr};
  Block* b = new Block{c->base, bytes, 0, true, stream, nullptr, false, c, nullptr, nullptr, {}, {}};
  c->head = b;
  d.chunks.push_back(c);
  index_free(d, b);
  d.st.reserved += bytes + kTailGuard;
  d.st.num_chunks++;
  d.st.num_grow++;
  if (d.st.reserved > d.st.peak_reserved) d.st.peak_reserved = d.st.reserved;
  return true;
}

// merge adjacent free blocks whose fences have completed (run before growing: pending fences block
// coalescing at free time, so fragmentation is settled lazily here); caller holds the lock
static void coalesce_settled(Device& d) {
  for (Chunk* c : d.chunks) {
    Block* b = c->head;
    while (b && b->next) {
      Block* n = b->next;
      if (b->free && n->free && fence_done(d, b) && fence_done(d, n)) {
        unindex_free(d, b);
        unindex_free(d, n);
        b->size += n->size;
        b->next = n->next;
        if (n->next) n->next->prev = b;
        delete n;
        index_free(d, b);
      } else {
        b = n;
      }
    }
  }
}

// return every chunk whose blocks are all free to the driver; caller holds the lock
static uint64_t release_free_chunks(Device& d, int dev) {
  uint64_t released = 0;
  if (!d.deferred.empty()) {  // settle deferred frees first (their streams' work is done after a device sync)
    int prev = -1;
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
    hipDeviceSynchronize();
    if (prev != dev) hipSetDevice(prev);
    process_deferred(d);
  }
  std::vector<Chunk*> keep;
  bool synced = false;
  for (Chunk* c : d.chunks) {
    bool all_free = true;
    for (Block* b = c->head; b; b = b->next) all_free = all_free && b->free;
    if (!all_free) {
      keep.push_back(c);
      continue;
    }
    if (!synced) {  // pending kernels may still read freed blocks
      int prev = -1;
      hipGetDevice(&prev);
      if (prev != dev) hipSetDevice(dev);
      hipDeviceSynchronize();
      if (prev != dev) hipSetDevice(prev);
      synced = true;
    }
    for (Block* b = c->head; b;) {
      Block* n = b->next;
      unindex_free(d, b);
      give_event(d, b->event);
      delete b;
      b = n;
    }
    hipFree(c->base);
    released += c->size + kTailGuard;
    d.st.reserved -= c->size + kTailGuard;
    d.st.num_chunks--;
    delete c;
  }
  d.chunks.swap(keep);
  return released;
}

static Block* find_fit(Device& d, size_t size, hipStream_t stream) {
  int scanned = 0;
  for (auto it = d.free_index.lower_bound(size); it != d.free_index.end() && scanned < kMaxScan; ++it, ++scanned) {
    if (usable_on(d, it->second, stream)) return it->second;
  }
  return nullptr;
}

// PD_ALLOC_TRACE=<file>: every allocation / free appended as one line ("A <ptr> <bytes> <stream>" /
// "F <ptr>") with an unbuffered write, so the file is complete up to the instant a GPU fault aborts the process:
// replaying it gives the live-block map at the fault (scripts/alloc_fault_map.py maps the faulting address to
// the block it falls in or lies next to).
static int trace_fd() {
  static int fd = [] {
    const char* p = std::getenv("PD_ALLOC_TRACE");
    return (p && *p) ? ::open(p, O_WRONLY | O_CREAT | O_APPEND | O_TRUNC, 0644) : -1;
  }();
  return fd;
}

static void trace(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
static void trace(const char* fmt, ...) {
  const int fd = trace_fd();
  if (fd < 0) return;
  char buf[128];
  va_list ap;
  va_start(ap, fmt);
  const int n = std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (n > 0) (void)!::write(fd, buf, (size_t)std::min(n, (int)sizeof(buf) - 1));
}

static void* do_alloc_impl(size_t size, int dev, hipStream_t stream);

static void* do_alloc(size_t size, int dev, hipStream_t stream) {
  void* p = do_alloc_impl(size, dev, stream);
  trace("A %p %zu %p\n", p, size, (void*)stream);
  return p;
}

static void* do_alloc_impl(size_t size, int dev, hipStream_t stream) {
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  Device& d = g_dev[dev];
  std::unique_lock<std::mutex> lk(d.mu);
  if (!d.seen_stream) {
    d.seen_stream = true;
    d.first_stream = stream;
  } else if (stream != d.first_stream && !d.multi_stream) {
    // blocks freed so far carry no fence: settle the device once before any cross-stream hand-off
    d.multi_stream = true;
    hipDeviceSynchronize();
  }
  if (!d.deferred.empty()) process_deferred(d);
  size_t need = round_up((size ? size : 1) + g_guard, kAlign);
  Block* b = find_fit(d, need, stream);
  if (!b) {
    coalesce_settled(d);
    b = find_fit(d, need, stream);
  }
  if (!b) {
    if (grow(d, dev, need, stream)) {
      b = find_fit(d, need, stream);
    } else {
      // out of device memory: first settle — one device sync retires every pending fence (deferred record_stream
      // frees re-enter the index, cross-stream blocks become usable), settled neighbours coalesce, and the whole
      // free index is scanned (not just the first kMaxScan candidates); only then are fully-free chunks returned
      // to the driver for one more growth.  If nothing fits the allocation fails (torch.OutOfMemoryError through
      // the torch hook — a null pointer handed to torch became a GPU memory-access fault).
      d.st.num_oom_retries++;
      // Under stream capture a device sync is illegal (it would invalidate the capture instead of failing the
      // allocation): settle only what the fences already show, never return chunks, and fail with OOM.  Outside
      // capture the sync runs with the allocator lock RELEASED, so other threads' allocations (and RCCL / p2p work
      // waiting on peers) are not blocked behind the drain; the free index is re-scanned after relocking.
      hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
      const bool capturing = hipStreamIsCapturing(stream, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
      if (!capturing) {
        lk.unlock();
        int prev = -1;
        hipGetDevice(&prev);
        if (prev != dev) hipSetDevice(dev);
        hipDeviceSynchronize();
        if (prev != dev) hipSetDevice(prev);
        lk.lock();
      }
      process_deferred(d);
      for (auto& kv : d.free_index) fence_done(d, kv.second);
      coalesce_settled(d);
      for (auto it = d.free_index.lower_bound(need); it != d.free_index.end(); ++it) {
        if (usable_on(d, it->second, stream)) {
          b = it->second;
          break;
        }
      }
      if (!b && !capturing) {
        // last resort: return the fully-free chunks to the driver and grow once more (the pool is fragmented:
        // free bytes exist but no block holds `need`)
        release_free_chunks(d, dev);
        if (grow(d, dev, need, stream)) b = find_fit(d, need, stream);
      }
      if (!b) {
        std::fprintf(stderr, "[pd_alloc] out of memory: %zu bytes on device %d (allocated %llu, reserved %llu)\n",
                     need, dev, (unsigned long long)d.st.allocated, (unsigned long long)d.st.reserved);
        return nullptr;   // the torch hook turns this into torch.OutOfMemoryError
      }
    }
    if (!b) return nullptr;
  }
  b = carve(d, b, need, stream);
  b->req = size;
  if (g_canary && b->size > size) hipMemsetAsync(b->ptr + size, kCanary, b->size - size, stream);
  d.live.emplace(b->ptr, b);
  d.st.allocated += b->size;
  d.st.num_allocs++;
  if (d.st.allocated > d.st.peak_allocated) d.st.peak_allocated = d.st.allocated;
  return b->ptr;
}

// b (no longer live) becomes a free block freed on `stream`; `settled`: every use of it has completed (a deferred
// free whose events all fired), so it needs no fence.  Coalesces with free neighbours; caller holds the lock.
static void finish_free(Device& d, Block* b, hipStream_t stream, bool settled) {
  b->stream = stream;
  b->uses.clear();
  if (d.multi_stream && !settled) {
    b->event = take_event(d);
    if (b->event && hipEventRecord(b->event, stream) == hipSuccess) {
      b->event_pending = true;
    } else {
      give_event(d, b->event);
      b->event = nullptr;
      hipStreamSynchronize(stream);  // could not fence: make the block safe the slow way
    }
  }
  // coalesce with free neighbours that are either from the same stream (b's newer fence covers their earlier
  // work) or already fenced complete (safe for anyone): the merged block carries b's stream and fence
  Block* p = b->prev;
  if (p && p->free && (p->stream == b->stream || fence_done(d, p)) && (!settled || fence_done(d, p))) {
    unindex_free(d, p);
    give_event(d, p->event);
    p->size += b->size;
    p->next = b->next;
    if (b->next) b->next->prev = p;
    p->event = b->event;
    p->event_pending = b->event_pending;
    delete b;
    b = p;
  }
  Block* n = b->next;
  if (n && n->free && (n->stream == b->stream || fence_done(d, n)) && (!settled || fence_done(d, n))) {
    unindex_free(d, n);
    give_event(d, n->event);
    b->size += n->size;
    b->next = n->next;
    if (n->next) n->next->prev = b;
    delete n;
  }
  if (b->prev == nullptr) b->chunk->head = b;
  index_free(d, b);
}

// re-index deferred frees whose recorded-stream events have all completed; caller holds the lock
static void process_deferred(Device& d) {
  size_t keep = 0;
  for (size_t i = 0; i < d.deferred.size(); ++i) {
    Deferred& f = d.deferred[i];
    bool done = true;
    for (hipEvent_t e : f.events) done = done && hipEventQuery(e) == hipSuccess;
    if (!done) {
      if (keep != i) d.deferred[keep] = std::move(f);
      ++keep;
      continue;
    }
    for (hipEvent_t e : f.events) give_event(d, e);
    finish_free(d, f.b, f.stream, /*settled=*/true);
  }
  d.deferred.resize(keep);
}

static void do_free(void* ptr, int dev, hipStream_t stream) {
  if (!ptr || dev < 0 || dev >= kMaxDevices) return;
  trace("F %p\n", ptr);
  Device& d = g_dev[dev];
  std::lock_guard<std::mutex> lk(d.mu);
  auto it = d.live.find(ptr);
  if (it == d.live.end()) {
    std::fprintf(stderr, "[pd_alloc] free of unknown pointer %p on device %d\n", ptr, dev);
    return;
  }
  Block* b = it->second;
  d.live.erase(it);
  if (g_canary && b->size > b->req) {
    size_t n = b->size - b->req;
    std::vector<unsigned char> host(n);
    hipStreamSynchronize(stream);
    if (hipMemcpy(host.data(), b->ptr + b->req, n, hipMemcpyDeviceToHost) == hipSuccess) {
      for (size_t i = 0; i < n; ++i) {
        if (host[i] != kCanary) {
          g_violations.push_back({reinterpret_cast<uint64_t>(b->ptr), b->req, i});
          std::fprintf(stderr, "[pd_alloc] write past the end of a %zu-byte block at %p: +%zu bytes\n", b->req,
                       (void*)b->ptr, i);
          break;
        }
      }
    }
  }
  d.st.allocated -= b->size;
  d.st.num_frees++;
  if (!b->uses.empty()) {
    // used by other streams: fence every one of them (and the freeing stream), re-index when all have passed
    Deferred f{b, stream, {}};
    bool ok = true;
    for (size_t i = 0; i <= b->uses.size() && ok; ++i) {
      hipStream_t s = i < b->uses.size() ? b->uses[i] : stream;
      hipEvent_t e = take_event(d);
      if (!e || hipEventRecord(e, s) != hipSuccess) {
        give_event(d, e);
        ok = false;
        break;
      }
      f.events.push_back(e);
    }
    if (ok) {
      d.st.deferred_frees++;
      d.deferred.push_back(std::move(f));
      return;
    }
    for (hipEvent_t e : f.events) give_event(d, e);  // could not fence: settle the slow way
    for (hipStream_t s : b->uses) hipStreamSynchronize(s);
    hipStreamSynchronize(stream);
    finish_free(d, b, stream, /*settled=*/true);
    return;
  }
  finish_free(d, b, stream, /*settled=*/false);
}

// Tensor.record_stream: the live block holding `ptr` is also used by `stream`
static void do_record_stream(void* ptr, hipStream_t stream) {
  for (int dev = 0; dev < kMaxDevices; ++dev) {
    Device& d = g_dev[dev];
    if (!d.seen_stream) continue;
    std::lock_guard<std::mutex> lk(d.mu);
    auto it = d.live.find(ptr);
    if (it == d.live.end()) continue;
    Block* b = it->second;
    if (stream == b->stream) return;
    for (hipStream_t s : b->uses)
      if (s == stream) return;
    b->uses.push_back(stream);
    d.st.record_stream++;
    if (!d.multi_stream) {  // blocks freed so far carry no fence: settle once (as for a second allocating stream)
      d.multi_stream = true;
      hipDeviceSynchronize();
    }
    return;
  }
}

}  // namespace alloc
}  // namespace pd

using namespace pd::alloc;

extern "C" {

// CUDAPluggableAllocator entry points
void* pd_alloc_malloc(size_t size, int device, hipStream_t stream) { return do_alloc(size, device, stream); }

void pd_alloc_free(void* ptr, size_t /*size*/, int device, hipStream_t stream) { do_free(ptr, device, stream); }

void pd_alloc_record_stream(void* ptr, hipStream_t stream) { do_record_stream(ptr, stream); }

void pd_alloc_debug(uint64_t guard_bytes, int canary) {
  std::lock_guard<std::mutex> lk(g_cfg_mu);
  g_guard = round_up(guard_bytes, kAlign);
  g_canary = canary != 0;
}

// violations recorded by the canary check: out[3*i .. 3*i+2] = (ptr, requested bytes, first bad offset)
uint64_t pd_alloc_violations(uint64_t* out, uint64_t max_n) {
  uint64_t n = 0;
  for (auto& v : g_violations) {
    if (n >= max_n) break;
    out[3 * n] = v.ptr;
    out[3 * n + 1] = v.req;
    out[3 * n + 2] = v.offset;
    ++n;
  }
  return g_violations.size();
}

void pd_alloc_configure(uint64_t chunk_bytes, uint64_t limit_bytes) {
  std::lock_guard<std::mutex> lk(g_cfg_mu);
  if (chunk_bytes) g_chunk_bytes = round_up(chunk_bytes, size_t(2) << 20);
  g_limit_bytes = limit_bytes;
}

// bytes of device memory every growth leaves free for the HIP runtime / RCCL / driver (0 disables the check)
void pd_alloc_set_headroom(uint64_t bytes) {
  std::lock_guard<std::mutex> lk(g_cfg_mu);
  g_headroom = bytes;
}

// out[0..12] = allocated, reserved, peak_allocated, peak_reserved, num_allocs, num_frees, num_chunks,
//              num_grow, num_oom_retries, cross_stream_reuse, record_stream, deferred_frees, deferred_pending
void pd_alloc_stats(int device, uint64_t* out) {
  if (device < 0 || device >= kMaxDevices) return;
  Device& d = g_dev[device];
  std::lock_guard<std::mutex> lk(d.mu);
  const Stats& s = d.st;
  uint64_t v[13] = {s.allocated, s.reserved, s.peak_allocated, s.peak_reserved, s.num_allocs,
                    s.num_frees, s.num_chunks, s.num_grow, s.num_oom_retries, s.cross_stream_reuse,
                    s.record_stream, s.deferred_frees, (uint64_t)d.deferred.size()};
  std::memcpy(out, v, sizeof(v));
}

void pd_alloc_reset_peak(int device) {
  if (device < 0 || device >= kMaxDevices) return;
  Device& d = g_dev[device];
  std::lock_guard<std::mutex> lk(d.mu);
  d.st.peak_allocated = d.st.allocated;
  d.st.peak_reserved = d.st.reserved;
}

uint64_t pd_alloc_empty_cache(int device) {
  if (device < 0 || device >= kMaxDevices) return 0;
  Device& d = g_dev[device];
  std::lock_guard<std::mutex> lk(d.mu);
  uint64_t r = release_free_chunks(d, device);
  for (hipEvent_t e : d.event_pool) hipEventDestroy(e);
  d.event_pool.clear();
  return r;
}

// largest free block and number of free blocks (fragmentation diagnostics)
void pd_alloc_fragmentation(int device, uint64_t* out) {
  if (device < 0 || device >= kMaxDevices) return;
  Device& d = g_dev[device];
  std::lock_guard<std::mutex> lk(d.mu);
  out[0] = d.free_index.empty() ? 0 : d.free_index.rbegin()->first;
  out[1] = d.free_index.size();
}

}  // extern "C"
