/* Host-side buffers of the HIP library: device buffers and pinned (page-locked) host buffers that grow on demand.
 * Shared by the decode path (ldpc_hip_api.cpp) and the PDSCH encoder queue (ldpc_hip_enc_queue.cpp). */
#pragma once

#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <mutex>

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

/* Device memory the host writes through the PCIe BAR (fine-grained VRAM the CPU agent is allowed to access: one
 * address for both), for inputs the host stages and a kernel then reads: the host's stores are posted writes, and
 * the kernel reads HBM instead of pinned host memory across PCIe. A one-CB work-queue handoff of 25,344 LLRs took
 * 7.8 us this way against 12.6-14.5 us from pinned memory, 1,248 LLRs 5.6 against 6.5-6.7 us; with the ring word in
 * pinned memory and the payload here, 240,000 items read no stale byte (PCIe keeps the payload's posted writes ahead
 * of the ring word's read completion; tools/ubench/vram_ring.hip, profiles/r06/vram_ring.txt). The host never reads
 * it (uncached reads across PCIe) and orders its stores before the hand-off with an sfence (they may be
 * write-combined). Off with LDPC_HIP_BAR_STAGING=0, and wherever the allocation or the access grant fails (callers
 * then use their pinned staging). Used for the one-CB decode's LLRs (1.5-1.9 us per software-route call). Not for
 * the HAL's staging: host stores into BAR memory ran at ~18 GB/s for C4's 128-CB TB, enqueues 20 -> 88 us against a
 * first dequeue 75 -> 47 us, the slot 30 us slower (profiles/r06/bar_staging_route_ab.json). */
inline bool bar_staging_enabled()
{
  static const bool on = [] {
    const char* v = std::getenv("LDPC_HIP_BAR_STAGING");
    return v == nullptr || std::strcmp(v, "0") != 0;
  }();
  return on;
}

inline hsa_status_t bar_find_cpu(hsa_agent_t agent, void* data)
{
  hsa_device_type_t t{};
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(data) = agent;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct bar_buffer {
  void*  ptr  = nullptr; /* host and device address */
  void*  dev  = nullptr;
  size_t size = 0;
  bar_buffer() = default;
  bar_buffer(const bar_buffer&) = delete;
  bar_buffer& operator=(const bar_buffer&) = delete;
  ~bar_buffer()
  {
    if (ptr != nullptr) {
      (void)hipFree(ptr);
    }
  }
  /* at least n bytes on the current device (the old contents are not kept); an error leaves the buffer as it was */
  hipError_t reserve(size_t n)
  {
    if (n <= size) {
      return hipSuccess;
    }
    if (!bar_staging_enabled()) {
      return hipErrorNotSupported;
    }
    static hsa_agent_t    cpu{};
    static bool           have_cpu = false;
    static std::once_flag once;
    std::call_once(once, [] { have_cpu = hsa_iterate_agents(bar_find_cpu, &cpu) == HSA_STATUS_INFO_BREAK; });
    if (!have_cpu) {
      return hipErrorNotSupported;
    }
    n            = (n + 65535U) & ~static_cast<size_t>(65535U);
    void*      p = nullptr;
    hipError_t e = hipExtMallocWithFlags(&p, n, hipDeviceMallocFinegrained);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return e;
    }
    if (hsa_amd_agents_allow_access(1, &cpu, nullptr, p) != HSA_STATUS_SUCCESS) {
      (void)hipFree(p);
      return hipErrorNotSupported;
    }
    if (ptr != nullptr) {
      (void)hipFree(ptr);
    }
    ptr = dev = p;
    size      = n;
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
