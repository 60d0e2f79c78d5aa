// Diagnostic microbenchmark (round 6): which acquire does a persistent workgroup need before reading host-written
// pinned memory it has read before (the work queue's staging buffers are reused item after item)? The host writes a
// 16 KB payload with the iteration number, then a ring word; one persistent workgroup (256 threads) polls the ring
// word, applies the variant's acquire, reads the whole payload (16-byte loads), counts the words that are not the
// iteration number (stale reads), and stores the count and the done word. Variants: 0 no acquire, 1 buffer_inv sc0
// (vector L1 only), 2 the agent-scope acquire fence (what dwq_loop issues), 3 the system-scope acquire fence. Also
// times each handoff and, on the device, the acquire plus reading the payload and a 64 KB device-memory table (the
// decoder's split tables are that size): whether the acquire sends the table reads past the L2. Every spin is bounded (2 s without a new item ends the kernel). Vector loads/stores only.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench/stale_probe tools/ubench/stale_probe.hip
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

constexpr uint32_t STOP  = 0xffffffffU;
constexpr uint32_t BYTES = 16384;

__global__ void __launch_bounds__(256) prober(const uint32_t* ring, const uint4* payload, uint32_t* done,
                                              uint32_t* bad, const uint4* table, uint32_t* ticks,
                                              int variant, int what)
{
  __shared__ uint32_t s_seq, s_bad;
  uint32_t            want = 1;
  uint64_t            last = __builtin_amdgcn_s_memrealtime();
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
      s_bad = 0;
    }
    __syncthreads();
    const uint32_t v = s_seq;
    __syncthreads();
    if (v == STOP) {
      break;
    }
    const uint64_t ta = __builtin_amdgcn_s_memrealtime();
    if (variant == 1) {
      asm volatile("buffer_inv sc0" ::: "memory");
    } else if (variant == 2) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    } else if (variant == 3) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    uint32_t nb = 0;
    if (variant == 4 && (what & 1) != 0) { /* system-coherent loads (sc0 sc1), no acquire: 4 per thread in flight */
      static_assert(BYTES / 16 == 4 * 256, "4 loads per thread");
      uint4 x[4];
      asm volatile("global_load_dwordx4 %0, %4, off sc0 sc1\n\t"
                   "global_load_dwordx4 %1, %5, off sc0 sc1\n\t"
                   "global_load_dwordx4 %2, %6, off sc0 sc1\n\t"
                   "global_load_dwordx4 %3, %7, off sc0 sc1\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
                   : "v"(payload + threadIdx.x), "v"(payload + threadIdx.x + 256), "v"(payload + threadIdx.x + 512),
                     "v"(payload + threadIdx.x + 768)
                   : "memory");
      for (int k = 0; k < 4; ++k) {
        nb += (x[k].x != v) + (x[k].y != v) + (x[k].z != v) + (x[k].w != v);
      }
    }
    for (uint32_t o = threadIdx.x; o < BYTES / 16 && (what & 1) != 0 && variant != 4; o += blockDim.x) {
      const uint4 x = payload[o];
      nb += (x.x != v) + (x.y != v) + (x.z != v) + (x.w != v);
    }
    uint32_t acc = 0;
    for (uint32_t o = threadIdx.x; o < 65536 / 16 && (what & 2) != 0; o += blockDim.x) {
      const uint4 x = table[o];
      acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    nb += acc == 0x9e3779b9U ? 1U : 0U; /* keeps the table loads */
    if (nb != 0) {
      atomicAdd(&s_bad, nb);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      bad[v & 1023]   = s_bad;
      ticks[v & 1023] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime() - ta);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    last = __builtin_amdgcn_s_memrealtime();
    ++want;
  }
}

int main()
{
  CHECK(hipSetDevice(0));
  uint32_t *ring_h = nullptr, *done_h = nullptr, *bad_h = nullptr, *pay_h = nullptr, *tk_h = nullptr;
  void *    ring_d = nullptr, *done_d = nullptr, *bad_d = nullptr, *pay_d = nullptr, *tk_d = nullptr, *table = nullptr;
  CHECK(hipMalloc(&table, 65536));
  CHECK(hipMemset(table, 0x5a, 65536));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&tk_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer(&tk_d, tk_h, 0));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&ring_h), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&done_h), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&bad_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&pay_h), BYTES, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer(&ring_d, ring_h, 0));
  CHECK(hipHostGetDevicePointer(&done_d, done_h, 0));
  CHECK(hipHostGetDevicePointer(&bad_d, bad_h, 0));
  CHECK(hipHostGetDevicePointer(&pay_d, pay_h, 0));
  const char* names[] = {"none", "inv_sc0", "agent", "system", "sc0sc1ld"};
  const char* reads[] = {"", "payload", "table", "both"};
  const int   runs[][2] = {{0, 3}, {1, 3}, {2, 3}, {3, 3}, {0, 2}, {2, 2}, {0, 1}, {2, 1}, {4, 1}, {4, 3}};
  for (const auto& run : runs) {
    const int variant = run[0], what = run[1];
    __atomic_store_n(ring_h, 0U, __ATOMIC_RELEASE);
    __atomic_store_n(done_h, 0U, __ATOMIC_RELEASE);
    std::memset(bad_h, 0, 4096);
    _mm_sfence();
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(prober, dim3(1), dim3(256), 0, s, static_cast<const uint32_t*>(ring_d),
                       static_cast<const uint4*>(pay_d), static_cast<uint32_t*>(done_d), static_cast<uint32_t*>(bad_d),
                       static_cast<const uint4*>(table), static_cast<uint32_t*>(tk_d), variant, what);
    CHECK(hipGetLastError());
    const uint32_t      N = 20000;
    uint64_t            stale_words = 0, stale_items = 0;
    std::vector<double> rtt, dev;
    bool                lost = false;
    for (uint32_t k = 1; k <= N; ++k) {
      const auto t0 = std::chrono::steady_clock::now();
      for (uint32_t i = 0; i < BYTES / 4; ++i) {
        pay_h[i] = k;
      }
      _mm_sfence();
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
      const uint32_t b = __atomic_load_n(&bad_h[k & 1023], __ATOMIC_ACQUIRE);
      stale_words += b;
      stale_items += b != 0 ? 1 : 0;
      dev.push_back(__atomic_load_n(&tk_h[k & 1023], __ATOMIC_ACQUIRE) * 0.01);
    }
    __atomic_store_n(ring_h, STOP, __ATOMIC_RELEASE);
    _mm_sfence();
    CHECK(hipStreamSynchronize(s));
    CHECK(hipStreamDestroy(s));
    std::sort(rtt.begin(), rtt.end());
    std::sort(dev.begin(), dev.end());
    std::printf("%-8s %-7s items %u%s: stale items %llu, stale words %llu, round trip p50 %.2f us, device acquire + "
                "reads p50 %.2f us p90 %.2f us\n",
                names[variant], reads[what], N, lost ? " (LOST)" : "", static_cast<unsigned long long>(stale_items),
                static_cast<unsigned long long>(stale_words), rtt.empty() ? 0.0 : rtt[rtt.size() / 2],
                dev.empty() ? 0.0 : dev[dev.size() / 2], dev.empty() ? 0.0 : dev[dev.size() * 9 / 10]);
  }
  return 0;
}
