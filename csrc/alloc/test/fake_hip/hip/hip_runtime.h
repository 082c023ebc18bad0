// Host-only stand-in for the handful of HIP runtime calls csrc/alloc/auto_growth.cpp makes, used ONLY by the
// CPU stress test (csrc/alloc/test/alloc_stress.cpp) so the allocator's bookkeeping can run under ASan/TSan on
// a machine without a GPU.  "Device" memory is host memory; events complete after a few queries (async
// stand-in); device/stream synchronization completes every outstanding event.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <set>

typedef int hipError_t;
enum { hipSuccess = 0, hipErrorOutOfMemory = 2, hipErrorNotReady = 600 };
constexpr unsigned hipEventDisableTiming = 2;
typedef struct FakeStream* hipStream_t;
struct FakeEvent {
  std::atomic<int> remaining{0};
};
typedef FakeEvent* hipEvent_t;

namespace fakehip {
inline std::mutex& mu() { static std::mutex m; return m; }
inline std::set<FakeEvent*>& live() { static std::set<FakeEvent*> s; return s; }
inline std::atomic<size_t>& in_use() { static std::atomic<size_t> v{0}; return v; }
inline size_t cap() { return size_t(1) << 32; }
inline thread_local int cur_dev = 0;
}  // namespace fakehip

inline hipError_t hipMalloc(void** p, size_t n) {
  if (fakehip::in_use() + n > fakehip::cap()) { *p = nullptr; return hipErrorOutOfMemory; }
  *p = std::malloc(n);
  if (!*p) return hipErrorOutOfMemory;
  fakehip::in_use() += n;
  return hipSuccess;
}
inline hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }  // byte accounting is approximate
inline hipError_t hipMemGetInfo(size_t* free_b, size_t* total_b) {
  *total_b = fakehip::cap();
  *free_b = fakehip::cap() > fakehip::in_use() ? fakehip::cap() - fakehip::in_use() : 0;
  return hipSuccess;
}
inline hipError_t hipGetDevice(int* d) { *d = fakehip::cur_dev; return hipSuccess; }
inline hipError_t hipSetDevice(int d) { fakehip::cur_dev = d; return hipSuccess; }
inline hipError_t hipGetLastError() { return hipSuccess; }
enum { hipMemcpyDeviceToHost = 2 };
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { std::memset(p, v, n); return hipSuccess; }
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, int) { std::memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  *e = new FakeEvent();
  std::lock_guard<std::mutex> lk(fakehip::mu());
  fakehip::live().insert(*e);
  return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t e) {
  {
    std::lock_guard<std::mutex> lk(fakehip::mu());
    fakehip::live().erase(e);
  }
  delete e;
  return hipSuccess;
}
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t) { e->remaining = 3; return hipSuccess; }
inline hipError_t hipEventQuery(hipEvent_t e) {
  if (e->remaining.load() <= 0) return hipSuccess;
  e->remaining--;
  return hipErrorNotReady;
}
inline hipError_t hipEventSynchronize(hipEvent_t e) { e->remaining = 0; return hipSuccess; }
inline hipError_t hipDeviceSynchronize() {
  std::lock_guard<std::mutex> lk(fakehip::mu());
  for (auto* e : fakehip::live()) e->remaining = 0;
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipDeviceSynchronize(); }
enum hipStreamCaptureStatus { hipStreamCaptureStatusNone = 0, hipStreamCaptureStatusActive = 1 };
inline hipError_t hipStreamIsCapturing(hipStream_t, hipStreamCaptureStatus* s) {
  *s = hipStreamCaptureStatusNone;
  return hipSuccess;
}
