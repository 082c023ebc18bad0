// Installs the native allocator (auto_growth.cpp) as PyTorch-ROCm's device allocator WITH its record-stream hook
// and hipGraph private-pool support.
//
// torch.cuda.memory.CUDAPluggableAllocator only takes malloc/free, so Tensor.record_stream (used by the executor's
// stream analyzer, AsyncLoad, the stage-3 prefetch stream and the process groups for async collectives) was
// a no-op under it: a tensor still read on a side stream could be re-handed out on its allocating stream.  This
// shim builds the pluggable allocator in C++ and sets record_stream_fn -> pd_alloc_record_stream, the
// reference's StreamSafeCUDAAllocator::RecordStream (stream_safe_cuda_allocator.cc) equivalent.
//
// Graph capture (torch.cuda.graph / CUDAGraph: the serving decode step, the static executor's replay) asks the
// allocator for a private pool: begin_allocate_to_pool(device, pool, filter) routes every allocation whose
// stream passes `filter` (the capturing stream) to that pool until end_allocate_to_pool.  Pool blocks are
// dedicated hipMalloc allocations: memory freed inside the pool is reused only by the same pool (a replay
// rewrites exactly the addresses the capture recorded), no events are recorded or queried while a capture is
// underway (both would become graph nodes or invalidate the capture), and release_pool returns the pool's free
// blocks to the driver (blocks still referenced are freed when their tensor dies).
#include <hip/hip_runtime.h>
#include <torch/csrc/cuda/CUDAPluggableAllocator.h>

#include <algorithm>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

extern "C" {
void* pd_alloc_malloc(size_t size, int device, hipStream_t stream);
void pd_alloc_free(void* ptr, size_t size, int device, hipStream_t stream);
void pd_alloc_record_stream(void* ptr, hipStream_t stream);
void pd_alloc_fragmentation(int device, uint64_t* out);
void pd_alloc_stats(int device, uint64_t* out);
void pd_alloc_reset_peak(int device);
}

namespace {

using PoolId = std::pair<unsigned long long, unsigned long long>;

struct Router {
  std::mutex mu;
  struct Active {
    int device;
    PoolId pool;
    std::function<bool(hipStream_t)> filter;
  };
  std::vector<Active> active;                                   // pools currently capturing
  std::unordered_map<void*, std::pair<PoolId, size_t>> live;    // pool block -> (pool, bytes)
  std::map<PoolId, std::multimap<size_t, void*>> free_blocks;   // per pool: freed blocks by size
  std::map<PoolId, bool> released;

  void* malloc(size_t size, int device, hipStream_t stream) {
    {
      std::lock_guard<std::mutex> lk(mu);
      for (auto& a : active) {
        if (a.device != device || !a.filter(stream)) continue;
        auto& fl = free_blocks[a.pool];
        auto it = fl.lower_bound(size);
        if (it != fl.end() && it->first <= 2 * size + (1 << 20)) {   // best fit, bounded waste
          void* p = it->second;
          live[p] = {a.pool, it->first};
          fl.erase(it);
          return p;
        }
        const size_t bytes = (size + 511) & ~size_t(511);
        void* p = nullptr;
        int prev = 0;
        hipGetDevice(&prev);
        if (prev != device) hipSetDevice(device);
        // a malloc inside a global-mode capture invalidates it: relax this thread's capture mode around it
        // (the capture records new VA; replays do not allocate again)
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        hipThreadExchangeStreamCaptureMode(&mode);
        const hipError_t e = hipMalloc(&p, bytes ? bytes : 512);
        hipThreadExchangeStreamCaptureMode(&mode);
        if (prev != device) hipSetDevice(prev);
        if (e != hipSuccess) return nullptr;
        live[p] = {a.pool, bytes};
        return p;
      }
    }
    return pd_alloc_malloc(size, device, stream);
  }

  void free(void* ptr, size_t size, int device, hipStream_t stream) {
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = live.find(ptr);
      if (it != live.end()) {
        const PoolId pool = it->second.first;
        const size_t bytes = it->second.second;
        live.erase(it);
        if (released[pool]) hipFree(ptr);
        else free_blocks[pool].emplace(bytes, ptr);
        return;
      }
    }
    pd_alloc_free(ptr, size, device, stream);
  }

  void begin(int device, PoolId pool, std::function<bool(hipStream_t)> filter) {
    std::lock_guard<std::mutex> lk(mu);
    released[pool] = false;
    active.push_back({device, pool, std::move(filter)});
  }

  void end(int device, PoolId pool) {
    std::lock_guard<std::mutex> lk(mu);
    for (auto it = active.begin(); it != active.end(); ++it) {
      if (it->device == device && it->pool == pool) {
        active.erase(it);
        break;
      }
    }
  }

  void release(int device, PoolId pool) {
    std::lock_guard<std::mutex> lk(mu);
    auto fit = free_blocks.find(pool);
    if (fit != free_blocks.end()) {
      hipDeviceSynchronize();   // a replay still in flight may use the blocks
      for (auto& kv : fit->second) hipFree(kv.second);
      free_blocks.erase(fit);
    }
    released[pool] = true;      // blocks still live are freed by their own free()
  }
};

Router& router() {
  static Router* r = new Router();   // never destroyed: frees may arrive during interpreter teardown
  return *r;
}

PoolId key(const c10::hip::MempoolId_t& id) { return {(unsigned long long)id.first, (unsigned long long)id.second}; }

namespace P = torch::cuda::CUDAPluggableAllocator;

// The pluggable allocator base throws from cacheInfo / getDeviceStats.  ATen's MIOpen convolution sizes its
// workspace from cacheInfo (the largest block it could get): with the throwing base the workspace bound is 0 and
// MIOpen falls back to its naive direct kernels (ResNet50 ran `naive_conv_ab_nonpacked_*` at ~200 ms per call);
// torch.cuda.max_memory_allocated() raised.  Both answer from the native allocator here.
struct PdTorchAllocator : P::CUDAPluggableAllocator {
  using P::CUDAPluggableAllocator::CUDAPluggableAllocator;

  void cacheInfo(c10::DeviceIndex device, size_t* largestBlock) override {
    uint64_t st[13] = {};
    pd_alloc_stats(device, st);
    size_t free_b = 0, total_b = 0;
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != device) hipSetDevice(device);
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    if (prev != device) hipSetDevice(prev);
    // a workspace can come from the largest free block of the pool or from new device memory (the pool's free
    // BYTES are scattered over many blocks: quoting them promised workspaces no single block could hold)
    uint64_t frag[2] = {0, 0};
    pd_alloc_fragmentation(device, frag);
    *largestBlock = std::max((size_t)frag[0], free_b);
  }

  c10::CachingDeviceAllocator::DeviceStats getDeviceStats(c10::DeviceIndex device) override {
    uint64_t st[13] = {};
    pd_alloc_stats(device, st);
    c10::CachingDeviceAllocator::DeviceStats d;
    const size_t agg = static_cast<size_t>(c10::CachingDeviceAllocator::StatType::AGGREGATE);
    auto set = [&](c10::CachingDeviceAllocator::StatArray& a, uint64_t cur, uint64_t peak) {
      a[agg].current = (int64_t)cur;
      a[agg].peak = (int64_t)peak;
    };
    set(d.allocated_bytes, st[0], st[2]);
    set(d.active_bytes, st[0], st[2]);
    set(d.requested_bytes, st[0], st[2]);
    set(d.reserved_bytes, st[1], st[3]);
    d.allocation[agg].allocated = (int64_t)st[4];
    d.allocation[agg].freed = (int64_t)st[5];
    d.allocation[agg].current = (int64_t)(st[4] - st[5]);
    d.segment[agg].current = (int64_t)st[6];
    d.num_alloc_retries = (int64_t)st[8];
    return d;
  }

  void resetPeakStats(c10::DeviceIndex device) override { pd_alloc_reset_peak(device); }
  void resetAccumulatedStats(c10::DeviceIndex) override {}
};

}  // namespace

extern "C" {

// 0 on success, 1 if the created allocator is not a CUDAPluggableAllocator (no hooks possible)
int pd_alloc_install_torch() {
  auto pa = std::make_shared<PdTorchAllocator>(
      [](size_t size, int device, hipStream_t stream) {
        void* p = router().malloc(size, device, stream);
        // torch's pluggable allocator wraps whatever pointer comes back: a null one for a non-empty tensor made
        // the next kernel write to address 0 (an out-of-memory turned into a GPU memory-access fault).  Raise
        // torch's OutOfMemoryError instead, as its caching allocator does.
        TORCH_CHECK_WITH(OutOfMemoryError, p != nullptr || size == 0,
                         "native allocator: out of memory allocating ", size, " bytes on device ", device,
                         " (FLAGS_use_native_allocator=0 selects torch's caching allocator)");
        return p;
      },
      [](void* ptr, size_t size, int device, hipStream_t stream) { router().free(ptr, size, device, stream); });
  std::shared_ptr<c10::hip::HIPCachingAllocator::HIPAllocator> a = pa;
  pa->set_record_stream_fn([](void* ptr, hipStream_t stream) {
    {
      std::lock_guard<std::mutex> lk(router().mu);
      if (router().live.count(ptr)) return;   // pool blocks: ordered by the captured stream
    }
    pd_alloc_record_stream(ptr, stream);
  });
  pa->set_begin_allocate_to_pool(
      [](int device, c10::hip::MempoolId_t id, std::function<bool(hipStream_t)> filter) {
        router().begin(device, key(id), std::move(filter));
      });
  pa->set_end_allocate_to_pool_fn([](int device, c10::hip::MempoolId_t id) { router().end(device, key(id)); });
  pa->set_release_pool([](int device, c10::hip::MempoolId_t id) { router().release(device, key(id)); });
  P::changeCurrentAllocator(a);
  return 0;
}
}
