// Diagnostic microbenchmark (round 6): a work-queue handoff whose ring word and payload live in device memory that
// the host writes through the PCIe BAR, against the pinned-host ring of today. Device memory: fine-grained VRAM
// (hipExtMallocWithFlags hipDeviceMallocFinegrained) made CPU-accessible with hsa_amd_agents_allow_access; a SIGSEGV
// on the host's first store says the BAR does not expose it (reported, nothing else runs in that mode). One persistent
// workgroup (256 threads) polls the ring word with system-scope loads, applies the agent-scope acquire the work queue
// uses, reads `bytes` of payload (16 B per thread per pass) with plain loads, and lane 0 stores the sequence number into a done word in pinned host memory
// after a system-scope release. The host writes the payload, then the ring word, spins on the done word, checks the
// payload checksum the device returned, and records the round trip. Every spin is bounded (2 s on the device, 1 s on
// the host). Modes: host (ring and payload pinned), vram (both in device memory), mix (ring pinned, payload in device
// memory: does the payload arrive before the ring word is seen?), and the host's memcpy bandwidth into each. Vector
// memory instructions only.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench/vram_ring tools/ubench/vram_ring.hip -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <csetjmp>
#include <csignal>
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
                                              uint32_t* done, uint32_t* sums)
{
  __shared__ uint32_t s_seq, s_sum;
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
      s_sum = 0;
    }
    __syncthreads();
    const uint32_t v = s_seq;
    __syncthreads();
    if (v == STOP) {
      break;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    uint32_t acc = 0;
    for (uint32_t o = threadIdx.x; o < bytes / 16; o += blockDim.x) {
      const uint4 x = payload[o];
      acc += x.x + x.y + x.z + x.w;
    }
    if (acc != 0) {
      atomicAdd(&s_sum, acc);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      sums[v & 1023] = s_sum;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    last = __builtin_amdgcn_s_memrealtime();
    ++want;
  }
}

static sigjmp_buf g_jmp;
static void       on_segv(int) { siglongjmp(g_jmp, 1); }

static hsa_status_t find_cpu(hsa_agent_t agent, void* data)
{
  hsa_device_type_t t;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(data) = agent;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

static int run(const char* name, uint32_t* ring_h, const uint32_t* ring_d, uint8_t* pay_h, const uint4* pay_d,
               uint32_t* done_h, uint32_t* done_d, uint32_t* sums_h, uint32_t* sums_d, uint32_t bytes)
{
  __atomic_store_n(ring_h, 0U, __ATOMIC_RELEASE);
  __atomic_store_n(done_h, 0U, __ATOMIC_RELEASE);
  _mm_sfence();
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(poller, dim3(1), dim3(256), 0, s, ring_d, pay_d, bytes, done_d, sums_d);
  CHECK(hipGetLastError());
  std::vector<uint32_t> buf(bytes / 4 + 1);
  std::vector<double>   rtt;
  uint64_t              bad  = 0;
  bool                  lost = false;
  const uint32_t        N    = 20000;
  for (uint32_t k = 1; k <= N; ++k) {
    for (uint32_t i = 0; i < bytes / 4; ++i) {
      buf[i] = k + i;
    }
    uint32_t want = 0;
    for (uint32_t i = 0; i < bytes / 4; ++i) {
      want += buf[i];
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(pay_h, buf.data(), bytes);
    _mm_sfence();
    __atomic_store_n(ring_h, k, __ATOMIC_RELEASE);
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
    if (!ok) {
      lost = true;
      break;
    }
    rtt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    bad += __atomic_load_n(&sums_h[k & 1023], __ATOMIC_ACQUIRE) != want ? 1 : 0;
  }
  __atomic_store_n(ring_h, STOP, __ATOMIC_RELEASE);
  _mm_sfence();
  CHECK(hipStreamSynchronize(s));
  CHECK(hipStreamDestroy(s));
  std::sort(rtt.begin(), rtt.end());
  std::printf("%-5s bytes=%6u  items %u%s  wrong payload sums %llu  round trip p50 %6.2f us  p10 %6.2f  p90 %6.2f\n",
              name, bytes, N, lost ? " (LOST)" : "", static_cast<unsigned long long>(bad),
              rtt.empty() ? 0.0 : rtt[rtt.size() / 2], rtt.empty() ? 0.0 : rtt[rtt.size() / 10],
              rtt.empty() ? 0.0 : rtt[rtt.size() * 9 / 10]);
  return 0;
}

int main()
{
  CHECK(hipSetDevice(0));
  constexpr size_t PAY = 32768;
  uint32_t *done_h = nullptr, *sums_h = nullptr, *ring_h = nullptr;
  uint8_t*  pay_h = nullptr;
  void *    done_d = nullptr, *sums_d = nullptr, *ring_d = nullptr, *pay_d = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&done_h), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&sums_h), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&ring_h), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&pay_h), PAY, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer(&done_d, done_h, 0));
  CHECK(hipHostGetDevicePointer(&sums_d, sums_h, 0));
  CHECK(hipHostGetDevicePointer(&ring_d, ring_h, 0));
  CHECK(hipHostGetDevicePointer(&pay_d, pay_h, 0));
  const uint32_t sizes[] = {0, 1248, 10752, 25344};
  for (uint32_t b : sizes) {
    if (run("host", ring_h, static_cast<const uint32_t*>(ring_d), pay_h, static_cast<const uint4*>(pay_d), done_h,
            static_cast<uint32_t*>(done_d), sums_h, static_cast<uint32_t*>(sums_d), b) != 0) {
      return 1;
    }
  }
  /* device memory the host writes through the BAR */
  void* vram = nullptr;
  CHECK(hipExtMallocWithFlags(&vram, PAY + 4096, hipDeviceMallocFinegrained));
  hsa_agent_t cpu{};
  hsa_iterate_agents(find_cpu, &cpu);
  const hsa_status_t st = hsa_amd_agents_allow_access(1, &cpu, nullptr, vram);
  std::printf("vram %p: hsa_amd_agents_allow_access(cpu) status %d\n", vram, static_cast<int>(st));
  struct sigaction sa {}, old {};
  sa.sa_handler = on_segv;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &old);
  bool mapped = false;
  if (sigsetjmp(g_jmp, 1) == 0) {
    volatile uint32_t* p = static_cast<volatile uint32_t*>(vram);
    p[0]                 = 0x12345678U;
    mapped               = p[0] == 0x12345678U;
  }
  sigaction(SIGSEGV, &old, nullptr);
  if (!mapped) {
    std::printf("vram: the host cannot store to it (SIGSEGV or readback mismatch): BAR mode skipped\n");
    return 0;
  }
  /* host store bandwidth into the BAR-mapped device memory (memcpy + sfence), against pinned host memory */
  {
    void* big = nullptr;
    CHECK(hipExtMallocWithFlags(&big, 2u << 20, hipDeviceMallocFinegrained));
    if (hsa_amd_agents_allow_access(1, &cpu, nullptr, big) == HSA_STATUS_SUCCESS) {
      uint8_t* pin = nullptr;
      CHECK(hipHostMalloc(reinterpret_cast<void**>(&pin), 2u << 20, hipHostMallocMapped | hipHostMallocCoherent));
      std::vector<uint8_t> src(2u << 20, 7);
      /* 128 codeblocks of 9,760 LLRs one after another (C4's 128-CB TB as the HAL enqueues it), by memcpy and by
       * 32-byte non-temporal stores */
      for (int mode = 0; mode < 2; ++mode) {
        std::vector<double> t;
        for (int r = 0; r < 50; ++r) {
          const auto t0 = std::chrono::steady_clock::now();
          for (uint32_t cb = 0; cb < 128; ++cb) {
            uint8_t*       d  = static_cast<uint8_t*>(big) + cb * 9760u;
            const uint8_t* sp = src.data() + cb * 9760u;
            if (mode == 0) {
              std::memcpy(d, sp, 9760);
            } else {
              uint32_t i = 0;
              for (; i < 9760u && (reinterpret_cast<uintptr_t>(d + i) & 31U) != 0; ++i) {
                d[i] = sp[i];
              }
              for (; i + 32 <= 9760u; i += 32) {
                _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i),
                                    _mm256_loadu_si256(reinterpret_cast<const __m256i*>(sp + i)));
              }
              for (; i < 9760u; ++i) {
                d[i] = sp[i];
              }
            }
          }
          _mm_sfence();
          t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(t.begin(), t.end());
        std::printf("host 128 x 9760 B into vram by %s: p50 %8.2f us (%.1f GB/s)\n", mode == 0 ? "memcpy" : "stream",
                    t[t.size() / 2], 128 * 9760 / (t[t.size() / 2] * 1e3));
      }
      for (uint32_t n : {1248u, 10752u, 25344u, 131072u, 1310720u}) {
        for (int dst = 0; dst < 2; ++dst) {
          uint8_t*            d = dst == 0 ? static_cast<uint8_t*>(big) : pin;
          std::vector<double> t;
          for (int r = 0; r < 200; ++r) {
            const auto t0 = std::chrono::steady_clock::now();
            std::memcpy(d, src.data(), n);
            _mm_sfence();
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
          }
          std::sort(t.begin(), t.end());
          std::printf("host memcpy %-6s %8u B: p50 %8.2f us (%.1f GB/s)\n", dst == 0 ? "vram" : "pinned", n,
                      t[t.size() / 2], n / (t[t.size() / 2] * 1e3));
        }
      }
      CHECK(hipHostFree(pin));
    }
    CHECK(hipFree(big));
  }
  uint32_t* vring = static_cast<uint32_t*>(vram);
  uint8_t*  vpay  = static_cast<uint8_t*>(vram) + 4096;
  for (uint32_t b : sizes) {
    if (run("vram", vring, vring, vpay, reinterpret_cast<const uint4*>(vpay), done_h, static_cast<uint32_t*>(done_d),
            sums_h, static_cast<uint32_t*>(sums_d), b) != 0) {
      return 1;
    }
  }
  /* mix: the ring word in pinned host memory (as the work queue's ring), the payload in the BAR-written device memory */
  for (int rep = 0; rep < 3; ++rep) {
    for (uint32_t b : sizes) {
      if (run("mix", ring_h, static_cast<const uint32_t*>(ring_d), vpay, reinterpret_cast<const uint4*>(vpay), done_h,
              static_cast<uint32_t*>(done_d), sums_h, static_cast<uint32_t*>(sums_d), b) != 0) {
        return 1;
      }
    }
  }
  return 0;
}
