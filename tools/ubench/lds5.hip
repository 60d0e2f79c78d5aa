// Diagnostic microbenchmark (round 3): LDS pipe cost of byte reads and writes as a function of which lane touches
// which byte of a 64-byte window (the decoder's rotated columns: a wave's 64 check nodes read and write 64 consecutive
// bytes at an unaligned base; the lane -> check node map is free to choose). One workgroup of W waves, each issuing
// n x 64 LDS instructions at 4 window bases; prints LDS ticks per wave-instruction per CU.
//   identity : lane l -> byte l
//   quarter  : lane l -> byte 4 (l % 16) + l / 16      (each 16-lane quarter touches 16 distinct dwords)
//   half     : lane l -> byte 2 (l % 32) + l / 32      (each 32-lane half touches 2 bytes of 16 dwords)
//   half32   : lane l -> 32 (l / 32) + 4 (l % 8) + (l / 8) % 4   (split rows: per half-wave the quarter pattern)
//   dword    : lane l -> byte 4 l                      (one dword per lane, a 256-byte window: the bound)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP8(x) x x x x x x x x

__device__ uint32_t perm(int P, uint32_t l)
{
  switch (P) {
  case 1: return 4 * (l % 16) + l / 16;
  case 2: return 2 * (l % 32) + l / 32;
  case 3: return 32 * (l / 32) + 4 * (l % 8) + (l / 8) % 4;
  case 4: return 4 * l;
  default: return l;
  }
}

template <int OP, int P>
__global__ void kern(uint32_t* out, uint64_t* t, int n)
{
  extern __shared__ uint8_t lds[];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x) reinterpret_cast<uint32_t*>(lds)[i] = i;
  __syncthreads();
  const uint32_t o  = perm(P, lane);
  uint32_t       a0 = wave * 397 + o + 3, a1 = a0 + 4099, a2 = a0 + 8191, a3 = a0 + 12301;
  uint32_t       r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
  uint64_t       t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (OP == 0) {
      asm volatile(REP8("ds_read_i8 %0, %8\n ds_read_i8 %1, %9\n ds_read_i8 %2, %10\n ds_read_i8 %3, %11\n ds_read_i8 %4, %8 offset:16384\n ds_read_i8 %5, %9 offset:16384\n ds_read_i8 %6, %10 offset:16384\n ds_read_i8 %7, %11 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                   : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
    } else {
      asm volatile(REP8("ds_write_b8 %0, %4\n ds_write_b8 %1, %4\n ds_write_b8 %2, %4\n ds_write_b8 %3, %4\n ds_write_b8 %0, %4 offset:16384\n ds_write_b8 %1, %4 offset:16384\n ds_write_b8 %2, %4 offset:16384\n ds_write_b8 %3, %4 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(lane) : "memory");
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
  if (lane == 0) t[wave] = t1 - t0;
}

template <int OP, int P>
void run(const char* name, int waves)
{
  uint32_t* out;
  uint64_t* t;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&t, 64 * 8);
  const int n = 64, threads = 64 * waves;
  hipLaunchKernelGGL((kern<OP, P>), dim3(1), dim3(threads), 65536, 0, out, t, n);
  hipLaunchKernelGGL((kern<OP, P>), dim3(1), dim3(threads), 65536, 0, out, t, n);
  hipDeviceSynchronize();
  uint64_t ht[64];
  hipMemcpy(ht, t, 64 * 8, hipMemcpyDeviceToHost);
  uint64_t mx = 0;
  for (int w = 0; w < waves; ++w) mx = ht[w] > mx ? ht[w] : mx;
  std::printf("%-12s %-9s waves %2d: %.2f ticks per wave-instruction per CU\n", OP ? "ds_write_b8" : "ds_read_i8",
              name, waves, mx / (double(n) * 64 * waves));
  hipFree(out);
  hipFree(t);
}

template <int OP>
void all(int w)
{
  run<OP, 0>("identity", w);
  run<OP, 1>("quarter", w);
  run<OP, 2>("half", w);
  run<OP, 3>("half32", w);
  run<OP, 4>("dword", w);
}

int main()
{
  for (int w : {4, 12}) {
    all<0>(w);
    all<1>(w);
  }
  return 0;
}
