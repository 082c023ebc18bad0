// Host-only stand-in for the HIP runtime calls csrc/comm/rccl_core.h makes, used ONLY by the CPU stress test
// (csrc/comm/test/rccl_stress.cpp) so the process group's stream / event / task logic runs under TSan and ASan on
// a machine without a GPU.  Unlike a synchronous mock it keeps HIP's asynchrony: every stream is a worker thread
// draining a FIFO of closures, hipEventRecord enqueues a completion marker, hipStreamWaitEvent enqueues a wait on
// the event's record generation — so calc -> comm fences, end events and Task::synchronize really race the way
// they do on the device.  "Device" memory is host memory.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <set>
#include <thread>

typedef int hipError_t;
enum { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorNotReady = 600 };
constexpr unsigned hipEventDisableTiming = 2;
constexpr unsigned hipStreamNonBlocking = 1;

inline const char* hipGetErrorString(hipError_t e) {
  switch (e) {
    case hipSuccess: return "hipSuccess";
    case hipErrorNotReady: return "hipErrorNotReady";
    default: return "hipError(fake)";
  }
}

struct FakeEvent {
  std::atomic<int> refs{1};   // the handle + every queued closure that touches the event (HIP lets a pending
                              // event be destroyed; it is freed once its stream is done with it)
  std::mutex mu;
  std::condition_variable cv;
  uint64_t recorded = 0;   // generation of the latest hipEventRecord
  uint64_t done = 0;       // highest generation its stream has reached
};
typedef FakeEvent* hipEvent_t;
inline void fake_event_unref(FakeEvent* e) {
  if (--e->refs == 0) delete e;
}

struct FakeStream {
  std::thread::id owner = std::this_thread::get_id();   // the rank thread ("process") that created it
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  bool stop = false;
  size_t busy = 0;   // closures popped but not finished
  std::thread worker;
  FakeStream() : worker([this] { run(); }) {}
  ~FakeStream() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    worker.join();
  }
  void push(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu);
      q.push_back(std::move(f));
    }
    cv.notify_all();
  }
  void drain() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return q.empty() && busy == 0; });
  }

 private:
  void run() {
    std::unique_lock<std::mutex> lk(mu);
    while (true) {
      cv.wait(lk, [this] { return stop || !q.empty(); });
      if (q.empty()) return;   // stop requested and nothing left
      auto f = std::move(q.front());
      q.pop_front();
      ++busy;
      lk.unlock();
      f();
      lk.lock();
      --busy;
      cv.notify_all();
    }
  }
};
typedef FakeStream* hipStream_t;

namespace fakehip {
inline std::mutex& mu() {
  static std::mutex m;
  return m;
}
inline std::set<FakeStream*>& streams() {
  static std::set<FakeStream*> s;
  return s;
}
inline thread_local int cur_dev = 0;
}  // namespace fakehip

inline hipError_t hipSetDevice(int d) {
  fakehip::cur_dev = d;
  return hipSuccess;
}
inline hipError_t hipGetDevice(int* d) {
  *d = fakehip::cur_dev;
  return hipSuccess;
}
inline hipError_t hipDeviceGetStreamPriorityRange(int* lo, int* hi) {
  *lo = 0;
  *hi = -1;
  return hipSuccess;
}
inline hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned, int) {
  *s = new FakeStream();
  std::lock_guard<std::mutex> lk(fakehip::mu());
  fakehip::streams().insert(*s);
  return hipSuccess;
}
inline hipError_t hipStreamCreate(hipStream_t* s) { return hipStreamCreateWithPriority(s, 0, 0); }
inline hipError_t hipStreamDestroy(hipStream_t s) {
  {
    std::lock_guard<std::mutex> lk(fakehip::mu());
    fakehip::streams().erase(s);
  }
  delete s;   // drains: the worker finishes every queued closure first
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t s) {
  s->drain();
  return hipSuccess;
}
// every stream of the calling rank: in the test each rank is a thread standing in for a process, so the "device"
// of a rank is the set of streams its thread created (another rank may destroy its own streams meanwhile)
inline hipError_t hipDeviceSynchronize() {
  std::set<FakeStream*> ss;
  {
    std::lock_guard<std::mutex> lk(fakehip::mu());
    for (FakeStream* s : fakehip::streams())
      if (s->owner == std::this_thread::get_id()) ss.insert(s);
  }
  for (FakeStream* s : ss) s->drain();
  return hipSuccess;
}
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  *e = new FakeEvent();
  return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t e) {
  fake_event_unref(e);
  return hipSuccess;
}
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
  uint64_t gen;
  {
    std::lock_guard<std::mutex> lk(e->mu);
    gen = ++e->recorded;
  }
  ++e->refs;
  s->push([e, gen] {
    {
      std::lock_guard<std::mutex> lk(e->mu);
      e->done = std::max(e->done, gen);
      e->cv.notify_all();
    }
    fake_event_unref(e);
  });
  return hipSuccess;
}
inline hipError_t hipEventQuery(hipEvent_t e) {
  std::lock_guard<std::mutex> lk(e->mu);
  return e->done >= e->recorded ? hipSuccess : hipErrorNotReady;
}
inline hipError_t hipEventSynchronize(hipEvent_t e) {
  std::unique_lock<std::mutex> lk(e->mu);
  const uint64_t gen = e->recorded;
  e->cv.wait(lk, [&] { return e->done >= gen; });
  return hipSuccess;
}
// the stream waits for the event's record as of NOW (later re-records do not move the wait)
inline hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned) {
  uint64_t gen;
  {
    std::lock_guard<std::mutex> lk(e->mu);
    gen = e->recorded;
  }
  ++e->refs;
  s->push([e, gen] {
    {
      std::unique_lock<std::mutex> lk(e->mu);
      e->cv.wait(lk, [&] { return e->done >= gen; });
    }
    fake_event_unref(e);
  });
  return hipSuccess;
}
