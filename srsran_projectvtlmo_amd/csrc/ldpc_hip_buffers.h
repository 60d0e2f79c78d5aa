/* Host-side buffers of the HIP library: device buffers and pinned (page-locked) host buffers that grow on demand.
 * Shared by the decode path (ldpc_hip_api.cpp) and the PDSCH encoder queue (ldpc_hip_enc_queue.cpp). */
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstring>

namespace ldpc_hip {

/* Device buffer that grows on demand. */
struct dev_buffer {
  void*  ptr  = nullptr;
  size_t size = 0;
  ~dev_buffer()
  {
    if (ptr != nullptr) {
      (void)hipFree(ptr);
    }
  }
  hipError_t reserve(size_t n)
  {
    if (n <= size) {
      return hipSuccess;
    }
    if (ptr != nullptr) {
      (void)hipFree(ptr);
      ptr  = nullptr;
      size = 0;
    }
    hipError_t e = hipMalloc(&ptr, n);
    if (e == hipSuccess) {
      size = n;
    }
    return e;
  }
  template <typename T>
  T* as() const
  {
    return static_cast<T*>(ptr);
  }
};

/* pinned (page-locked) host buffer that grows on demand, keeping its first `keep` bytes, mapped into the device address
 * space: `dev` is its device address (the HAL queues' zero-copy batches let kernels read and write it directly).
 * Allocated coherent (fine-grained): the GPU does not cache it, so a kernel's reads see what the host staged and the
 * host sees the kernel's writes once the batch's completion event has fired, without relying on the runtime's
 * system-scope cache maintenance at dispatch boundaries. Each byte crosses PCIe once either way. */
struct pinned_buffer {
  void*  ptr  = nullptr;
  void*  dev  = nullptr;
  size_t size = 0;
  pinned_buffer() = default;
  pinned_buffer(const pinned_buffer&) = delete;
  pinned_buffer& operator=(const pinned_buffer&) = delete;
  ~pinned_buffer()
  {
    if (ptr != nullptr) {
      (void)hipHostFree(ptr);
    }
  }
  hipError_t reserve(size_t n, size_t keep)
  {
    if (n <= size) {
      return hipSuccess;
    }
    n            = std::max(n, 2 * size);
    void*      p = nullptr;
    hipError_t e = hipHostMalloc(&p, n, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) {
      return e;
    }
    if (ptr != nullptr) {
      if (keep != 0) {
        std::memcpy(p, ptr, std::min(keep, size));
      }
      (void)hipHostFree(ptr);
    }
    ptr  = p;
    size = n;
    /* the device address; without one (not expected on ROCm) users fall back to copies */
    if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess) {
      dev = nullptr;
      (void)hipGetLastError();
    }
    return hipSuccess;
  }
  template <typename T>
  T* as() const
  {
    return static_cast<T*>(ptr);
  }
  template <typename T>
  T* dev_as() const
  {
    return static_cast<T*>(dev);
  }
};

} // namespace ldpc_hip
