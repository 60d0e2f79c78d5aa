// Diagnostic (not product): a resident "sleeper" grid beside a C2 batch (tools/resident_tax_ab.py), to find what a
// resident work-queue grid costs a concurrent batch launch. Each workgroup reserves `lds` bytes of dynamic LDS (so it
// owns its CU like a work-queue workgroup) and stays for `usec` microseconds (s_memrealtime, 100 MHz). mode:
//   0  wave 0 loops on s_sleep + the clock, the other waves wait at a barrier (an idle work-queue grid, no polling)
//   1  every wave loops on s_sleep + the clock (no barrier)
//   2  as 0, and wave 0 reads a pinned host word (system scope) each loop (the idle poll)
//   3  every wave waits at a barrier until wave 0's s_sleep loop ends, wave 0 with s_sleep 127 (one clock read per
//      ~5 us)
// Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o tools/ubench/libresident_tax.so tools/ubench/resident_tax.hip
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void sleeper(uint64_t ticks, int mode, const uint32_t* host_word, uint32_t* sink)
{
  extern __shared__ uint32_t smem[];
  const uint64_t t0  = __builtin_amdgcn_s_memrealtime();
  uint32_t       acc = 0;
  if (mode == 1) {
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
      __builtin_amdgcn_s_sleep(2);
    }
  } else {
    if (threadIdx.x < 64) {
      while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        if (mode == 2 && host_word != nullptr) {
          acc += __hip_atomic_load(host_word + (threadIdx.x & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (mode == 3) {
          __builtin_amdgcn_s_sleep(127);
        } else {
          __builtin_amdgcn_s_sleep(2);
        }
      }
    }
    __syncthreads();
  }
  smem[threadIdx.x] = acc;
  if (acc == 0xdeadbeefU) {
    sink[blockIdx.x] = smem[threadIdx.x ^ 1];
  }
}

extern "C" int launch_sleeper(void* stream, int nwg, int threads, int lds, double usec, int mode,
                              const uint32_t* host_word, uint32_t* sink)
{
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sleeper),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) {
    return static_cast<int>(e);
  }
  hipLaunchKernelGGL(sleeper, dim3(nwg), dim3(threads), lds, static_cast<hipStream_t>(stream),
                     static_cast<uint64_t>(usec * 100.0), mode, host_word, sink);
  return static_cast<int>(hipGetLastError());
}
