// Diagnostic microbenchmark (round 4): host <-> device round trip of a work-queue style handoff, by where the ring
// word and the item's data live. One persistent workgroup (256 threads) polls a ring word; when it reads the next
// sequence number it reads `bytes` of payload (16 B per thread per pass), and lane 0 stores the sequence number into a
// done word in pinned host memory after a system-scope release. The host writes the payload and then the ring word,
// spins on the done word, and records the round trip. Modes:
//   host  : ring word and payload in pinned host memory (hipHostMalloc coherent; the device reads over PCIe)
//   fine  : ring word and payload in device memory from hipExtMallocWithFlags(hipDeviceMallocFinegrained), written by
//           the host through its CPU mapping (only if the allocation has one: hipPointerGetAttributes hostPointer)
//   unc   : as fine with hipDeviceMallocUncached
// Every device spin is bounded (the kernel leaves after 2 s without a new item or on the stop value), and the host
// gives up waiting after 1 s. Vector loads and stores only.
//   hipcc -O3 --offload-arch=gfx950 -o ring_rtt ring_rtt.hip && ./ring_rtt
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <emmintrin.h>

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

__global__ void __launch_bounds__(256) poller(const uint32_t* ring, const uint4* payload, uint32_t bytes,
                                              uint32_t* done, uint32_t* sink)
{
  __shared__ uint32_t s_seq;
  uint32_t            want = 1;
  uint64_t            last = __builtin_amdgcn_s_memrealtime();
  uint32_t            acc  = 0;
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
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    for (uint32_t o = threadIdx.x; o < bytes / 16; o += blockDim.x) {
      const uint4 x = payload[o];
      acc += x.x ^ x.y ^ x.z ^ x.w;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    last = __builtin_amdgcn_s_memrealtime();
    ++want;
  }
  sink[threadIdx.x] = acc;
}

static double median(std::vector<double> v)
{
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static double pct(std::vector<double> v, double p)
{
  std::sort(v.begin(), v.end());
  return v[static_cast<size_t>(p * (v.size() - 1))];
}

/* host write of the payload and ring word: 0 plain stores (memcpy), 1 non-temporal stores (the lines go to memory
 * through write combining, never dirty in a CPU cache the device's read must snoop), 2 plain stores + clflush */
static int g_how = 0;
static void host_copy(uint8_t* dst, const uint8_t* src, uint32_t n)
{
  if (g_how == 1 && (reinterpret_cast<uintptr_t>(dst) & 15U) == 0) {
    uint32_t i = 0;
    for (; i + 16 <= n; i += 16) {
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i)));
    }
    std::memcpy(dst + i, src + i, n - i);
  } else {
    std::memcpy(dst, src, n);
    if (g_how == 2) {
      for (uint32_t i = 0; i < n; i += 64) {
        _mm_clflush(dst + i);
      }
    }
  }
}
static void ring_store(uint32_t* ring, uint32_t v)
{
  if (g_how == 1) {
    _mm_stream_si32(reinterpret_cast<int*>(ring), static_cast<int>(v));
  } else {
    __atomic_store_n(ring, v, __ATOMIC_RELEASE);
    if (g_how == 2) {
      _mm_clflush(ring);
    }
  }
}

int run(const char* mode, uint32_t* ring_h, void* ring_d, uint8_t* pay_h, void* pay_d, uint32_t bytes, uint32_t* done_h,
        uint32_t* done_d, uint32_t* sink)
{
  __atomic_store_n(ring_h, 0U, __ATOMIC_RELEASE);
  __atomic_store_n(done_h, 0U, __ATOMIC_RELEASE);
  _mm_sfence();
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(poller, dim3(1), dim3(256), 0, s, static_cast<const uint32_t*>(ring_d),
                     static_cast<const uint4*>(pay_d), bytes, done_d, sink);
  CHECK(hipGetLastError());
  std::vector<uint8_t> src(bytes, 0x5a);
  std::vector<double>  rtt, wr;
  const int            N = 3000;
  bool                 lost = false;
  for (uint32_t k = 1; k <= N; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    if (bytes != 0) {
      src[0] = static_cast<uint8_t>(k);
      host_copy(pay_h, src.data(), bytes);
      _mm_sfence();
    }
    const auto t1 = std::chrono::steady_clock::now();
    ring_store(ring_h, k);
    _mm_sfence();
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
    const auto t2 = std::chrono::steady_clock::now();
    if (!ok) {
      lost = true;
      break;
    }
    if (k > 200) {
      rtt.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
      wr.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
  }
  __atomic_store_n(ring_h, STOP, __ATOMIC_RELEASE);
  _mm_sfence();
  CHECK(hipStreamSynchronize(s));
  CHECK(hipStreamDestroy(s));
  if (lost) {
    std::printf("%-5s bytes=%6u  LOST (no done word within 1 s)\n", mode, bytes);
    return 1;
  }
  std::printf("%-6s bytes=%6u  round trip p50 %6.2f us  p10 %6.2f  p90 %6.2f   host payload write p50 %6.2f us\n", mode,
              bytes, median(rtt), pct(rtt, 0.1), pct(rtt, 0.9), median(wr));
  return 0;
}

int main()
{
  CHECK(hipSetDevice(0));
  uint32_t* done_h = nullptr;
  void*     done_d = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&done_h), 64, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer(&done_d, done_h, 0));
  uint32_t* sink = nullptr;
  CHECK(hipMalloc(reinterpret_cast<void**>(&sink), 1024));
  const uint32_t sizes[] = {0, 1248, 10752, 25344};
  const size_t   PAY     = 1 << 16;

  /* host-pinned ring and payload */
  uint32_t* ring_h = nullptr;
  uint8_t*  pay_h  = nullptr;
  void *    ring_d = nullptr, *pay_d = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&ring_h), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer(&ring_d, ring_h, 0));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&pay_h), PAY, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer(&pay_d, pay_h, 0));
  const char* hows[] = {"host", "hostnt", "hostfl"};
  for (int how = 0; how < 3; ++how) {
    g_how = how;
    for (uint32_t b : sizes) {
      if (run(hows[how], ring_h, ring_d, pay_h, pay_d, b, done_h, static_cast<uint32_t*>(done_d), sink) != 0) {
        return 1;
      }
    }
  }
  g_how = 0;
  /* device memory with a CPU mapping, if the allocation has one */
  const struct {
    const char* name;
    unsigned    flag;
  } kinds[] = {{"fine", hipDeviceMallocFinegrained}, {"unc", hipDeviceMallocUncached}};
  for (const auto& kd : kinds) {
    void* r = nullptr;
    void* p = nullptr;
    if (hipExtMallocWithFlags(&r, 256, kd.flag) != hipSuccess || hipExtMallocWithFlags(&p, PAY, kd.flag) != hipSuccess) {
      (void)hipGetLastError();
      std::printf("%-5s allocation failed\n", kd.name);
      continue;
    }
    hipPointerAttribute_t ar{}, ap{};
    if (hipPointerGetAttributes(&ar, r) != hipSuccess || hipPointerGetAttributes(&ap, p) != hipSuccess) {
      (void)hipGetLastError();
      std::printf("%-5s no pointer attributes\n", kd.name);
      continue;
    }
    std::printf("%-5s type %d device %p host %p\n", kd.name, static_cast<int>(ar.type), ar.devicePointer,
                ar.hostPointer);
    if (ar.hostPointer == nullptr || ap.hostPointer == nullptr) {
      std::printf("%-5s no CPU mapping: skipped\n", kd.name);
      continue;
    }
    for (uint32_t b : sizes) {
      if (run(kd.name, static_cast<uint32_t*>(ar.hostPointer), ar.devicePointer, static_cast<uint8_t*>(ap.hostPointer),
              ap.devicePointer, b, done_h, static_cast<uint32_t*>(done_d), sink) != 0) {
        return 1;
      }
    }
  }
  return 0;
}
