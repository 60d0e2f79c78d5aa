// Diagnostic microbenchmark: VALU issue cost per wave-instruction for the ops the decoder uses, with W waves per
// SIMD (1 workgroup of 4*W waves on one CU). Prints cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int OP>
__global__ void kern(uint32_t* out, uint64_t* t, int n)
{
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a ^ 0x55, d = a + 7, e = a * 5, f = a + 11, g = a ^ 0x77, h = a + 2;
  __syncthreads();
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (OP == 0) {
      asm volatile(REP64("v_add_u32 %0, %0, %1\n v_add_u32 %2, %2, %3\n v_add_u32 %4, %4, %5\n v_add_u32 %6, %6, %7\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    } else if (OP == 1) {
      asm volatile(REP64("v_pk_add_u16 %0, %0, %1\n v_pk_add_u16 %2, %2, %3\n v_pk_add_u16 %4, %4, %5\n v_pk_add_u16 %6, %6, %7\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    } else if (OP == 2) {
      asm volatile(REP64("v_med3_i32 %0, %0, %1, %2\n v_med3_i32 %2, %2, %3, %4\n v_med3_i32 %4, %4, %5, %6\n v_med3_i32 %6, %6, %7, %0\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    } else if (OP == 3) {
      asm volatile(REP64("v_pk_max_i16 %0, %0, %1\n v_pk_max_i16 %2, %2, %3\n v_pk_max_i16 %4, %4, %5\n v_pk_max_i16 %6, %6, %7\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    } else if (OP == 4) {
      asm volatile(REP64("v_xor_b32 %0, %0, %1\n v_xor_b32 %2, %2, %3\n v_xor_b32 %4, %4, %5\n v_xor_b32 %6, %6, %7\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    } else if (OP == 5) { /* dependent chain, one register */
      asm volatile(REP64("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n")
                   : "+v"(a), "+v"(b));
    } else if (OP == 6) {
      asm volatile(REP64("v_pk_mad_u16 %0, %0, %1, %2\n v_pk_mad_u16 %2, %2, %3, %4\n v_pk_mad_u16 %4, %4, %5, %6\n v_pk_mad_u16 %6, %6, %7, %0\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    } else if (OP == 7) {
      asm volatile(REP64("v_readlane_b32 s0, %0, 3\n v_readlane_b32 s1, %2, 5\n v_readlane_b32 s2, %4, 7\n v_readlane_b32 s3, %6, 9\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : : "s0", "s1", "s2", "s3");
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h;
  if ((threadIdx.x & 63) == 0) {
    t[threadIdx.x >> 6] = t1 - t0;
  }
}

template <int OP>
void run(const char* name, int waves_per_simd)
{
  uint32_t* out;
  uint64_t* t;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&t, 64 * 8);
  const int n = 64, threads = 256 * waves_per_simd;
  hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 0, 0, out, t, n);
  hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 0, 0, out, t, n);
  hipDeviceSynchronize();
  uint64_t ht[64];
  hipMemcpy(ht, t, 64 * 8, hipMemcpyDeviceToHost);
  uint64_t mx = 0;
  for (int w = 0; w < threads / 64; ++w) {
    mx = ht[w] > mx ? ht[w] : mx;
  }
  const double instr_per_simd = double(n) * 256.0 * waves_per_simd;
  std::printf("%-14s waves/SIMD %d: %.2f ticks per wave-instruction per SIMD\n", name, waves_per_simd, mx / instr_per_simd);
  hipFree(out);
  hipFree(t);
}

int main()
{
  for (int w : {1, 2, 3, 4}) {
    run<0>("v_add_u32", w);
    run<1>("v_pk_add_u16", w);
    run<2>("v_med3_i32", w);
    run<3>("v_pk_max_i16", w);
    run<4>("v_xor_b32", w);
    run<5>("dep v_add_u32", w);
    run<6>("v_pk_mad_u16", w);
    run<7>("v_readlane", w);
  }
  return 0;
}
