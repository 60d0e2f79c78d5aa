// Diagnostic microbenchmark (round 6): the cost of a work-queue item's completion path. One persistent workgroup
// (256 threads) polls a ring word in pinned memory; per item it writes `out` bytes of results into pinned memory and
// then lane 0 stores the done word. Variants of the completion:
//   0 plain stores, system-scope release fence, done store       (what dwq_loop does today)
//   1 system-coherent stores (buffer stores sc0 sc1), s_waitcnt vmcnt(0), done store, no fence
//   2 no results, release fence, done store
//   3 no results, no fence, done store
// The host spins on the done word, checks every result word equals the item number (results visible when done is),
// and records the round trip. Every spin is bounded (2 s without an item ends the kernel; the host gives up after
// 1 s). Vector memory instructions only.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench/done_path tools/ubench/done_path.hip
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                                                       \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                                                              \
      return 1;                                                                                                        \
    }                                                                                                                  \
  } while (0)

constexpr uint32_t STOP = 0xffffffffU;

__global__ void __launch_bounds__(256) worker(const uint32_t* ring, uint32_t* out, uint32_t out_words, uint32_t* done,
                                              int variant)
{
  __shared__ uint32_t s_seq;
  uint32_t            want = 1;
  uint64_t            last = __builtin_amdgcn_s_memrealtime();
  const uint64_t      p    = reinterpret_cast<uint64_t>(out);
  const uint64_t      lo   = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(p)));
  const uint64_t      hi   = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(p >> 32)));
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(lo | hi << 32), static_cast<short>(0),
                                                    static_cast<int>(out_words * 4U), 0x00020000);
  while (true) {
    if (threadIdx.x == 0) {
      uint32_t v = 0;
      while (true) {
        v = __hip_atomic_load(ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v == want || v == STOP) {
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - last > 200000000ULL) { /* 2 s */
          v = STOP;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_seq = v;
    }
    __syncthreads();
    const uint32_t v = s_seq;
    __syncthreads();
    if (v == STOP) {
      break;
    }
    if (variant <= 1) {
      for (uint32_t i = threadIdx.x; i < out_words; i += blockDim.x) {
        if (variant == 0) {
          out[i] = v;
        } else {
          __builtin_amdgcn_raw_buffer_store_b32(v, rs, static_cast<int>(i * 4U), 0, 17);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      if (variant == 0 || variant == 2) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      }
      __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    last = __builtin_amdgcn_s_memrealtime();
    ++want;
  }
}

int main()
{
  CHECK(hipSetDevice(0));
  constexpr uint32_t OUT_WORDS = 256; /* 1 KB: a one-CB call's packed bits and result */
  uint32_t *ring_h = nullptr, *done_h = nullptr, *out_h = nullptr;
  void *    ring_d = nullptr, *done_d = nullptr, *out_d = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&ring_h), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&done_h), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&out_h), OUT_WORDS * 4, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer(&ring_d, ring_h, 0));
  CHECK(hipHostGetDevicePointer(&done_d, done_h, 0));
  CHECK(hipHostGetDevicePointer(&out_d, out_h, 0));
  const char* names[] = {"plain+release", "sc0sc1 stores", "release only", "done only"};
  for (int rep = 0; rep < 2; ++rep) {
    for (int variant = 0; variant < 4; ++variant) {
      __atomic_store_n(ring_h, 0U, __ATOMIC_RELEASE);
      __atomic_store_n(done_h, 0U, __ATOMIC_RELEASE);
      std::memset(out_h, 0, OUT_WORDS * 4);
      _mm_sfence();
      hipStream_t s;
      CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      hipLaunchKernelGGL(worker, dim3(1), dim3(256), 0, s, static_cast<const uint32_t*>(ring_d),
                         static_cast<uint32_t*>(out_d), OUT_WORDS, static_cast<uint32_t*>(done_d), variant);
      CHECK(hipGetLastError());
      const uint32_t      N = 20000;
      uint64_t            bad = 0;
      std::vector<double> rtt;
      bool                lost = false;
      for (uint32_t k = 1; k <= N; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(ring_h, k, __ATOMIC_RELEASE);
        bool ok = false;
        for (long i = 0;; ++i) {
          if (__atomic_load_n(done_h, __ATOMIC_ACQUIRE) == k) {
            ok = true;
            break;
          }
          if ((i & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
            break;
          }
          _mm_pause();
        }
        if (!ok) {
          lost = true;
          break;
        }
        rtt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        if (variant <= 1) {
          for (uint32_t i = 0; i < OUT_WORDS; ++i) {
            bad += __atomic_load_n(&out_h[i], __ATOMIC_RELAXED) != k ? 1 : 0;
          }
        }
      }
      __atomic_store_n(ring_h, STOP, __ATOMIC_RELEASE);
      _mm_sfence();
      CHECK(hipStreamSynchronize(s));
      CHECK(hipStreamDestroy(s));
      std::sort(rtt.begin(), rtt.end());
      std::printf("%-14s items %u%s: results not visible at done %llu words, round trip p50 %.2f us p90 %.2f us\n",
                  names[variant], N, lost ? " (LOST)" : "", static_cast<unsigned long long>(bad),
                  rtt.empty() ? 0.0 : rtt[rtt.size() / 2], rtt.empty() ? 0.0 : rtt[rtt.size() * 9 / 10]);
    }
  }
  return 0;
}
