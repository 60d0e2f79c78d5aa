// Diagnostic microbenchmark (round 2 variant of lds.hip: 16-bit and d16 forms): LDS pipe cost of the decoder's access patterns. One workgroup (one CU) of W waves, each
// issuing n x 64 LDS instructions (8 independent streams, waits only at the end of each block of 8). Prints LDS cycles
// per wave-instruction per CU (total ticks / total wave-instructions of all waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x

template <int OP>
__global__ void kern(uint32_t* out, uint64_t* t, int n)
{
  extern __shared__ uint8_t lds[];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x) reinterpret_cast<uint32_t*>(lds)[i] = i;
  __syncthreads();
  /* byte addresses: 64 consecutive bytes per wave at a wave-dependent, unaligned base (like a rotated column) */
  uint32_t a0 = wave * 397 + lane + 3, a1 = a0 + 4099, a2 = a0 + 8191, a3 = a0 + 12301;
  uint32_t w0 = (wave * 64 + lane) * 4, w1 = w0 + 8192, w2 = w0 + 16384, w3 = w0 + 24576;
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (OP == 0) {
      asm volatile(REP8("ds_read_i8 %0, %8\n ds_read_i8 %1, %9\n ds_read_i8 %2, %10\n ds_read_i8 %3, %11\n ds_read_i8 %4, %8 offset:16384\n ds_read_i8 %5, %9 offset:16384\n ds_read_i8 %6, %10 offset:16384\n ds_read_i8 %7, %11 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                   : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
    } else if (OP == 1) {
      asm volatile(REP8("ds_read_u16 %0, %8\n ds_read_u16 %1, %9\n ds_read_u16 %2, %10\n ds_read_u16 %3, %11\n ds_read_u16 %4, %8 offset:16384\n ds_read_u16 %5, %9 offset:16384\n ds_read_u16 %6, %10 offset:16384\n ds_read_u16 %7, %11 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                   : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
    } else if (OP == 2) {
      asm volatile(REP8("ds_read_i8_d16_hi %0, %8\n ds_read_i8_d16_hi %1, %9\n ds_read_i8_d16_hi %2, %10\n ds_read_i8_d16_hi %3, %11\n ds_read_i8_d16_hi %4, %8 offset:16384\n ds_read_i8_d16_hi %5, %9 offset:16384\n ds_read_i8_d16_hi %6, %10 offset:16384\n ds_read_i8_d16_hi %7, %11 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                   : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
    } else if (OP == 3) {
      asm volatile(REP8("ds_read_b32 %0, %8\n ds_read_b32 %1, %9\n ds_read_b32 %2, %10\n ds_read_b32 %3, %11\n ds_read_b32 %4, %8 offset:16384\n ds_read_b32 %5, %9 offset:16384\n ds_read_b32 %6, %10 offset:16384\n ds_read_b32 %7, %11 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                   : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
    } else if (OP == 4) {
      asm volatile(REP8("ds_write_b8 %0, %4\n ds_write_b8 %1, %4\n ds_write_b8 %2, %4\n ds_write_b8 %3, %4\n ds_write_b8 %0, %4 offset:16384\n ds_write_b8 %1, %4 offset:16384\n ds_write_b8 %2, %4 offset:16384\n ds_write_b8 %3, %4 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(lane) : "memory");
    } else if (OP == 5) {
      asm volatile(REP8("ds_write_b16 %0, %4\n ds_write_b16 %1, %4\n ds_write_b16 %2, %4\n ds_write_b16 %3, %4\n ds_write_b16 %0, %4 offset:16384\n ds_write_b16 %1, %4 offset:16384\n ds_write_b16 %2, %4 offset:16384\n ds_write_b16 %3, %4 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(lane) : "memory");
    } else if (OP == 6) {
      asm volatile(REP8("ds_write_b8_d16_hi %0, %4\n ds_write_b8_d16_hi %1, %4\n ds_write_b8_d16_hi %2, %4\n ds_write_b8_d16_hi %3, %4\n ds_write_b8_d16_hi %0, %4 offset:16384\n ds_write_b8_d16_hi %1, %4 offset:16384\n ds_write_b8_d16_hi %2, %4 offset:16384\n ds_write_b8_d16_hi %3, %4 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(lane) : "memory");
    } else if (OP == 7) {
      asm volatile(REP8("ds_write_b32 %0, %4\n ds_write_b32 %1, %4\n ds_write_b32 %2, %4\n ds_write_b32 %3, %4\n ds_write_b32 %0, %4 offset:16384\n ds_write_b32 %1, %4 offset:16384\n ds_write_b32 %2, %4 offset:16384\n ds_write_b32 %3, %4 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)"
                   :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(lane) : "memory");
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
  if (lane == 0) t[wave] = t1 - t0;
}

template <int OP>
void run(const char* name, int waves, int per)
{
  uint32_t* out;
  uint64_t* t;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&t, 64 * 8);
  const int n = 64, threads = 64 * waves;
  hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 65536, 0, out, t, n);
  hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 65536, 0, out, t, n);
  hipDeviceSynchronize();
  uint64_t ht[64];
  hipMemcpy(ht, t, 64 * 8, hipMemcpyDeviceToHost);
  uint64_t mx = 0;
  for (int w = 0; w < waves; ++w) mx = ht[w] > mx ? ht[w] : mx;
  const double instr = double(n) * per * waves;
  std::printf("%-22s waves %2d: %.2f ticks per wave-instruction per CU\n", name, waves, mx / instr);
  hipFree(out);
  hipFree(t);
}

int main()
{
  for (int w : {4, 8, 12, 16}) {
    run<0>("ds_read_i8", w, 64);
    run<1>("ds_read_u16 (odd addr)", w, 64);
    run<2>("ds_read_i8_d16_hi", w, 64);
    run<3>("ds_read_b32 (unaligned)", w, 64);
    run<4>("ds_write_b8", w, 64);
    run<5>("ds_write_b16 (odd addr)", w, 64);
    run<6>("ds_write_b8_d16_hi", w, 64);
    run<7>("ds_write_b32 (unaligned)", w, 64);
  }
  return 0;
}
