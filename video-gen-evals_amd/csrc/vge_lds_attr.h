// Host helper of the launch paths that set a kernel's dynamic-LDS limit.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for a kernel on the calling thread's current device, once per device
// (the attribute is per device: a process that moves to another GPU sets it there too; two threads racing here only
// repeat an idempotent call).  One instance per launch site: `static LdsAttrOnce attr; attr(fn, bytes)`.
struct LdsAttrOnce {
  std::atomic<unsigned long long> done{0};
  hipError_t operator()(const void* fn, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_release);
    return e;
  }
};
