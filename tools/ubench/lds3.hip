// Diagnostic microbenchmark (round 2): LDS pipe cost of 16/32-bit accesses at ALIGNED strided addresses (one soft value
// per 2 or 4 bytes, wrapped rotation like a shifted column). Same harness as lds2.hip: one workgroup of W waves, 8
// independent streams, LDS cycles per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define RD(op) asm volatile(REP8(op " %0, %8\n " op " %1, %9\n " op " %2, %10\n " op " %3, %11\n " op " %4, %8 offset:16384\n " op " %5, %9 offset:16384\n " op " %6, %10 offset:16384\n " op " %7, %11 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)" \
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(a0), "v"(a1), "v"(a2), "v"(a3))
#define WR(op) asm volatile(REP8(op " %0, %4\n " op " %1, %4\n " op " %2, %4\n " op " %3, %4\n " op " %0, %4 offset:16384\n " op " %1, %4 offset:16384\n " op " %2, %4 offset:16384\n " op " %3, %4 offset:16384\n s_waitcnt lgkmcnt(8)\n") "s_waitcnt lgkmcnt(0)" \
                   :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(lane) : "memory")

template <int OP, int STRIDE>
__global__ void kern(uint32_t* out, uint64_t* t, int n)
{
  extern __shared__ uint8_t lds[];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x) reinterpret_cast<uint32_t*>(lds)[i] = i;
  __syncthreads();
  const uint32_t t0i = wave * 64 + lane;
  auto rot = [&](uint32_t r, uint32_t base) { return ((t0i + r) % 384U) * STRIDE + base; };
  uint32_t a0 = rot(37, 0), a1 = rot(101, 1536 * STRIDE / 4), a2 = rot(250, 3072 * STRIDE / 4), a3 = rot(383, 4608 * STRIDE / 4);
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
  uint64_t tb = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (OP == 0) RD("ds_read_u16");
    else if (OP == 1) RD("ds_read_u16_d16_hi");
    else if (OP == 2) RD("ds_read_b32");
    else if (OP == 3) RD("ds_read_i8");
    else if (OP == 4) WR("ds_write_b16");
    else if (OP == 5) WR("ds_write_b16_d16_hi");
    else if (OP == 6) WR("ds_write_b32");
    else if (OP == 7) WR("ds_write_b8");
  }
  uint64_t te = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
  if (lane == 0) t[wave] = te - tb;
}

template <int OP, int STRIDE>
void run(const char* name, int waves)
{
  uint32_t* out;
  uint64_t* t;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&t, 64 * 8);
  const int n = 64, threads = 64 * waves;
  hipLaunchKernelGGL((kern<OP, STRIDE>), dim3(1), dim3(threads), 65536, 0, out, t, n);
  hipLaunchKernelGGL((kern<OP, STRIDE>), dim3(1), dim3(threads), 65536, 0, out, t, n);
  hipDeviceSynchronize();
  uint64_t ht[64];
  hipMemcpy(ht, t, 64 * 8, hipMemcpyDeviceToHost);
  uint64_t mx = 0;
  for (int w = 0; w < waves; ++w) mx = ht[w] > mx ? ht[w] : mx;
  std::printf("%-22s stride %d waves %2d: %.2f ticks per wave-instruction per CU\n", name, STRIDE, waves,
              mx / (double(n) * 64 * waves));
  hipFree(out);
  hipFree(t);
}

int main()
{
  for (int w : {4, 12}) {
    run<0, 4>("ds_read_u16", w);
    run<1, 4>("ds_read_u16_d16_hi", w);
    run<2, 4>("ds_read_b32", w);
    run<3, 4>("ds_read_i8", w);
    run<4, 4>("ds_write_b16", w);
    run<5, 4>("ds_write_b16_d16_hi", w);
    run<6, 4>("ds_write_b32", w);
    run<7, 4>("ds_write_b8", w);
    run<0, 2>("ds_read_u16", w);
    run<1, 2>("ds_read_u16_d16_hi", w);
    run<4, 2>("ds_write_b16", w);
    run<5, 2>("ds_write_b16_d16_hi", w);
    run<7, 2>("ds_write_b8", w);
    run<3, 1>("ds_read_i8", w);
    run<7, 1>("ds_write_b8", w);
  }
  return 0;
}
