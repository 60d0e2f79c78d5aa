// Diagnostic microbenchmark (round 6): latency of a workgroup's first read of N bytes from pinned host memory, as
// the one-codeblock work-queue prologue issues it (16-byte loads, up to four in flight per thread), with and without
// an agent-scope acquire fence before it and with HBM table loads in flight beside it. One kernel launch per
// measurement; the kernel stamps s_memrealtime (100 MHz) before the loads and after s_waitcnt, lane 0 writes the
// difference. Vector loads/stores only.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench/pinned_read tools/ubench/pinned_read.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                                                       \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                                                              \
      return 1;                                                                                                        \
    }                                                                                                                  \
  } while (0)

// mode bit 0: agent-scope acquire fence first; bit 1: HBM table loads (tab4, ntab 16-byte chunks) in flight too;
// bit 2: the host buffer read with system-scope atomic-style loads of one dword per lane instead of 16-byte loads
__global__ void reader(const uint4* __restrict__ src, uint32_t n16, const uint4* __restrict__ tab4, uint32_t ntab,
                       int mode, uint32_t* __restrict__ out, uint4* __restrict__ sink)
{
  __shared__ uint4 s[1024];
  const uint32_t tid = threadIdx.x, nth = blockDim.x;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (mode & 1) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  uint4 v[4], t[3];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint32_t i = tid + u * nth;
    v[u]             = i < n16 ? src[i] : make_uint4(0, 0, 0, 0);
  }
  if (mode & 2) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const uint32_t j = tid + u * nth;
      t[u]             = j < ntab ? tab4[j] : make_uint4(0, 0, 0, 0);
    }
  } else {
    t[0] = t[1] = t[2] = make_uint4(0, 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  uint4          acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    acc.x ^= v[u].x;
    acc.y ^= v[u].y;
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    acc.z ^= t[u].z;
    acc.w ^= t[u].w;
  }
  s[tid] = acc;
  __syncthreads();
  if (tid == 0) {
    out[0] = static_cast<uint32_t>(t1 - t0);
  }
  if (acc.x == 0x12345678U && acc.y == 0x9abcdef0U) {
    sink[tid] = s[(tid + 1) % nth];
  }
}

/* bandwidth mode: `blocks` workgroups each read `per` bytes of pinned memory (16-byte loads, up to four in flight per
 * thread and pass) once, as the HAL's fused launch reads a large TB's staged LLRs; the kernel time gives GB/s */
__global__ void bw_reader(const uint4* __restrict__ src, uint32_t per16, uint4* __restrict__ sink)
{
  const uint4* b   = src + static_cast<size_t>(blockIdx.x) * per16;
  uint4        acc = make_uint4(0, 0, 0, 0);
  for (uint32_t i0 = threadIdx.x; i0 < per16; i0 += 4U * blockDim.x) {
    uint4 v[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t i = i0 + u * blockDim.x;
      v[u]             = i < per16 ? b[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      acc.x ^= v[u].x;
      acc.y ^= v[u].y;
      acc.z ^= v[u].z;
      acc.w ^= v[u].w;
    }
  }
  if (acc.x == 0x12345678U && acc.y == 0x9abcdef0U) {
    sink[threadIdx.x] = acc;
  }
}

static int bandwidth(const void* hdev, uint4* sink)
{
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const struct {
    uint32_t blocks, per, threads;
  } cases[] = {{128, 9728, 768}, {128, 9728, 256}, {256, 4864, 256}, {512, 2432, 256}, {1024, 1216, 256},
               {64, 19456, 768}, {128, 9728, 1024}};
  for (const auto& c : cases) {
    std::vector<float> t;
    for (int rep = 0; rep < 30; ++rep) {
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(bw_reader, dim3(c.blocks), dim3(c.threads), 0, 0, static_cast<const uint4*>(hdev),
                         c.per / 16, sink);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep >= 5) {
        t.push_back(ms);
      }
    }
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2] * 1e3, bytes = static_cast<double>(c.blocks) * c.per;
    std::printf("bandwidth: %4u workgroups x %6u B (%4u threads): %7.1f us, %5.1f GB/s\n", c.blocks, c.per, c.threads,
                us, bytes / us / 1e3);
  }
  return 0;
}

int main()
{
  const uint32_t sizes[] = {1248, 1800, 9728, 25344};
  uint8_t*       host    = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&host), 4 << 20, hipHostMallocMapped | hipHostMallocCoherent));
  for (int i = 0; i < (4 << 20); ++i) {
    host[i] = static_cast<uint8_t>(i * 7 + 1);
  }
  void* hdev = nullptr;
  CHECK(hipHostGetDevicePointer(&hdev, host, 0));
  uint4*    tab  = nullptr;
  uint32_t* out  = nullptr;
  uint4*    sink = nullptr;
  CHECK(hipMalloc(&tab, 1 << 20));
  CHECK(hipMemset(tab, 1, 1 << 20));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMalloc(&sink, 1 << 16));
  if (bandwidth(hdev, sink) != 0) {
    return 1;
  }
  for (int threads : {128, 256, 768}) {
    for (int mode = 0; mode < 4; ++mode) {
      for (uint32_t n : sizes) {
        std::vector<uint32_t> t;
        for (int rep = 0; rep < 40; ++rep) {
          hipLaunchKernelGGL(reader, dim3(1), dim3(threads), 0, 0, static_cast<const uint4*>(hdev), (n + 15) / 16,
                             tab, 324U, mode, out, sink);
          uint32_t v = 0;
          CHECK(hipMemcpy(&v, out, 4, hipMemcpyDeviceToHost));
          if (rep >= 5) {
            t.push_back(v);
          }
        }
        std::sort(t.begin(), t.end());
        std::printf("threads %4d fence %d tables %d bytes %6u: loads returned p50 %5.2f us p10 %5.2f p90 %5.2f\n",
                    threads, mode & 1, (mode >> 1) & 1, n, t[t.size() / 2] * 0.01, t[t.size() / 10] * 0.01,
                    t[t.size() * 9 / 10] * 0.01);
      }
    }
  }
  return 0;
}
