// Diagnostic microbenchmark (round 2): LDS pipe cost of ds_write_b8 as a function of the active lanes (EXEC = all,
// upper half, lower 8, none) -- whether a partial-wave write is cheaper than a full one. Same harness as lds2.hip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define WR(op) asm volatile("s_mov_b64 exec, %5\n" REP8(op " %0, %4\n " op " %1, %4\n " op " %2, %4\n " op " %3, %4\n " op " %0, %4 offset:16384\n " op " %1, %4 offset:16384\n " op " %2, %4 offset:16384\n " op " %3, %4 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)\n s_mov_b64 exec, -1" \
                   :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(lane), "s"(mask) : "memory")

template <int M>
__global__ void kern(uint32_t* out, uint64_t* t, int n)
{
  extern __shared__ uint8_t lds[];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x) reinterpret_cast<uint32_t*>(lds)[i] = i;
  __syncthreads();
  uint32_t a0 = wave * 397 + lane + 3, a1 = a0 + 4099, a2 = a0 + 8191, a3 = a0 + 12301;
  const uint64_t mask = M == 0 ? ~0ULL : M == 1 ? 0xffffffff00000000ULL : M == 2 ? 0xffULL : M == 3 ? 0ULL
                                                                          : 0x5555555555555555ULL;
  uint64_t tb = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    WR("ds_write_b8");
  }
  uint64_t te = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a0;
  if (lane == 0) t[wave] = te - tb;
}

template <int M>
void run(const char* name, int waves)
{
  uint32_t* out;
  uint64_t* t;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMalloc(&t, 64 * 8);
  const int n = 64, threads = 64 * waves;
  hipLaunchKernelGGL((kern<M>), dim3(1), dim3(threads), 65536, 0, out, t, n);
  hipLaunchKernelGGL((kern<M>), dim3(1), dim3(threads), 65536, 0, out, t, n);
  (void)hipDeviceSynchronize();
  uint64_t ht[64];
  (void)hipMemcpy(ht, t, 64 * 8, hipMemcpyDeviceToHost);
  uint64_t mx = 0;
  for (int w = 0; w < waves; ++w) mx = ht[w] > mx ? ht[w] : mx;
  std::printf("ds_write_b8 exec=%-14s waves %2d: %.2f ticks per wave-instruction per CU\n", name, waves,
              mx / (double(n) * 64 * waves));
  (void)hipFree(out);
  (void)hipFree(t);
}

int main()
{
  for (int w : {4, 12}) {
    run<0>("all", w);
    run<1>("upper 32", w);
    run<2>("lower 8", w);
    run<3>("none", w);
    run<4>("even lanes", w);
  }
  return 0;
}
