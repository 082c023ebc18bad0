// Installs the native allocator (auto_growth.cpp) as PyTorch-ROCm's device allocator WITH its record-stream hook.
//
// torch.cuda.memory.CUDAPluggableAllocator only takes malloc/free, so Tensor.record_stream (used by the executor's
// stream analyzer, AsyncLoad, the stage-3 prefetch stream and c10d's ProcessGroupNCCL for async collectives) was
// a no-op under it: a tensor still read on a side stream could be re-handed out on its allocating stream.  This
// shim builds the pluggable allocator in C++ and sets record_stream_fn -> pd_alloc_record_stream, the
// reference's StreamSafeCUDAAllocator::RecordStream (stream_safe_cuda_allocator.cc) equivalent.
#include <hip/hip_runtime.h>
#include <torch/csrc/cuda/CUDAPluggableAllocator.h>

#include <memory>

extern "C" {
void* pd_alloc_malloc(size_t size, int device, hipStream_t stream);
void pd_alloc_free(void* ptr, size_t size, int device, hipStream_t stream);
void pd_alloc_record_stream(void* ptr, hipStream_t stream);

// 0 on success, 1 if the created allocator is not a CUDAPluggableAllocator (no record-stream hook possible)
int pd_alloc_install_torch() {
  namespace P = torch::cuda::CUDAPluggableAllocator;
  auto a = P::createCustomAllocator(
      [](size_t size, int device, hipStream_t stream) { return pd_alloc_malloc(size, device, stream); },
      [](void* ptr, size_t size, int device, hipStream_t stream) { pd_alloc_free(ptr, size, device, stream); });
  auto pa = std::dynamic_pointer_cast<P::CUDAPluggableAllocator>(a);
  if (!pa) return 1;
  pa->set_record_stream_fn([](void* ptr, hipStream_t stream) { pd_alloc_record_stream(ptr, stream); });
  P::changeCurrentAllocator(a);
  return 0;
}
}
