// Diagnostic microbenchmark: issue cost per wave-instruction per SIMD of the encodings the specialised decoder uses
// (SDWA, VOPC, VOP3, DPP), W = 1..4 waves per SIMD. hipcc -O3 --offload-arch=gfx950 -o valu2 valu2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)

#define OPS(X)                                                                                                         \
  X(0, "v_add_u32 (VOP2)", "v_add_u32 %0, %0, %1\n v_add_u32 %2, %2, %3\n v_add_u32 %4, %4, %5\n v_add_u32 %6, %6, %7\n") \
  X(1, "v_sub_u32_sdwa sext b", "v_sub_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa %2, %2, sext(%3) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa %4, %4, sext(%5) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa %6, %6, sext(%7) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n") \
  X(2, "v_mul_i32_i24_sdwa dst byte", "v_mul_i32_i24_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa %2, %3, %4 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa %4, %5, %6 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa %6, %7, %0 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n") \
  X(3, "v_mul_i32_i24_e32", "v_mul_i32_i24_e32 %0, %0, %1\n v_mul_i32_i24_e32 %2, %2, %3\n v_mul_i32_i24_e32 %4, %4, %5\n v_mul_i32_i24_e32 %6, %6, %7\n") \
  X(4, "v_cmp_eq_u32 + cndmask vcc", "v_cmp_eq_u32_e32 vcc, %0, %1\n v_cndmask_b32_e32 %2, %2, %3, vcc\n v_cmp_eq_u32_e32 vcc, %4, %5\n v_cndmask_b32_e32 %6, %6, %7, vcc\n") \
  X(5, "v_lshl_add_u32 (VOP3)", "v_lshl_add_u32 %0, %0, 9, %1\n v_lshl_add_u32 %2, %2, 9, %3\n v_lshl_add_u32 %4, %4, 9, %5\n v_lshl_add_u32 %6, %6, 9, %7\n") \
  X(6, "v_med3_u32 (VOP3)", "v_med3_u32 %0, %0, %1, %2\n v_med3_u32 %2, %2, %3, %4\n v_med3_u32 %4, %4, %5, %6\n v_med3_u32 %6, %6, %7, %0\n") \
  X(7, "v_min_u32_e32", "v_min_u32_e32 %0, %0, %1\n v_min_u32_e32 %2, %2, %3\n v_min_u32_e32 %4, %4, %5\n v_min_u32_e32 %6, %6, %7\n") \
  X(8, "v_or_b32_sdwa sext b3", "v_or_b32_sdwa %0, sext(%1), 1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD\n v_or_b32_sdwa %2, sext(%3), 1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD\n v_or_b32_sdwa %4, sext(%5), 1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD\n v_or_b32_sdwa %6, sext(%7), 1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD\n") \
  X(9, "v_max_i16_e32", "v_max_i16_e32 %0, %0, %1\n v_max_i16_e32 %2, %2, %3\n v_max_i16_e32 %4, %4, %5\n v_max_i16_e32 %6, %6, %7\n") \
  X(10, "v_mov_b32_dpp row_shr", "v_mov_b32_dpp %0, %1 row_shr:1\n v_mov_b32_dpp %2, %3 row_shr:1\n v_mov_b32_dpp %4, %5 row_shr:1\n v_mov_b32_dpp %6, %7 row_shr:1\n") \
  X(11, "v_add3_u32 (VOP3)", "v_add3_u32 %0, %0, %1, %2\n v_add3_u32 %2, %2, %3, %4\n v_add3_u32 %4, %4, %5, %6\n v_add3_u32 %6, %6, %7, %0\n") \
  X(12, "v_xor_b32_sdwa w1", "v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n v_xor_b32_sdwa %2, %2, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n v_xor_b32_sdwa %4, %4, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n v_xor_b32_sdwa %6, %6, %7 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n") \
  X(13, "v_max_i32_e32", "v_max_i32_e32 %0, %0, %1\n v_max_i32_e32 %2, %2, %3\n v_max_i32_e32 %4, %4, %5\n v_max_i32_e32 %6, %6, %7\n") \
  X(14, "v_sub_u32 e64 (VOP3 enc)", "v_sub_u32_e64 %0, %0, %1\n v_sub_u32_e64 %2, %2, %3\n v_sub_u32_e64 %4, %4, %5\n v_sub_u32_e64 %6, %6, %7\n") \
  X(15, "v_pk_sub_i16 clamp", "v_pk_sub_i16 %0, %0, %1 clamp\n v_pk_sub_i16 %2, %2, %3 clamp\n v_pk_sub_i16 %4, %4, %5 clamp\n v_pk_sub_i16 %6, %6, %7 clamp\n") \
  X(16, "v_perm_b32", "v_perm_b32 %0, %0, %1, %2\n v_perm_b32 %2, %2, %3, %4\n v_perm_b32 %4, %4, %5, %6\n v_perm_b32 %6, %6, %7, %0\n") \
  X(17, "v_sad_u8", "v_sad_u8 %0, %0, %1, %2\n v_sad_u8 %2, %2, %3, %4\n v_sad_u8 %4, %4, %5, %6\n v_sad_u8 %6, %6, %7, %0\n") \
  X(18, "v_dot4_i32_i8", "v_dot4_i32_i8 %0, %0, %1, %2\n v_dot4_i32_i8 %2, %2, %3, %4\n v_dot4_i32_i8 %4, %4, %5, %6\n v_dot4_i32_i8 %6, %6, %7, %0\n") \
  X(19, "v_add_u16_sdwa b", "v_add_u16_sdwa %0, %0, sext(%1) dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:BYTE_0\n v_add_u16_sdwa %2, %2, sext(%3) dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:BYTE_0\n v_add_u16_sdwa %4, %4, sext(%5) dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:BYTE_0\n v_add_u16_sdwa %6, %6, sext(%7) dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:BYTE_0\n")

#define KER(id, name, body)                                                                                            \
  else if (OP == id) { asm volatile(REP32(body) : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : : "vcc"); }

template <int OP>
__global__ void kern(uint32_t* out, uint64_t* t, int n)
{
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a ^ 0x55, d = a + 7, e = a * 5, f = a + 11, g = a ^ 0x77, h = a + 2;
  __syncthreads();
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (false) {
    }
    OPS(KER)
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h;
  if ((threadIdx.x & 63) == 0) {
    t[threadIdx.x >> 6] = t1 - t0;
  }
}

template <int OP>
void run(const char* name)
{
  uint32_t* out;
  uint64_t* t;
  hipMalloc(&out, 1 << 20);
  hipMalloc(&t, 64 * 8);
  std::printf("%-30s", name);
  for (int w = 1; w <= 4; ++w) {
    const int n = 64, threads = 256 * w;
    hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 0, 0, out, t, n);
    hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 0, 0, out, t, n);
    hipDeviceSynchronize();
    uint64_t ht[64];
    hipMemcpy(ht, t, 64 * 8, hipMemcpyDeviceToHost);
    uint64_t mx = 0;
    for (int q = 0; q < threads / 64; ++q) {
      mx = ht[q] > mx ? ht[q] : mx;
    }
    std::printf("  %5.2f", mx / (double(n) * 128.0 * w));
  }
  std::printf("\n");
  hipFree(out);
  hipFree(t);
}

#define RUN(id, name, body) run<id>(name);
int main()
{
  std::printf("%-30s  cycles per wave-instruction per SIMD at 1, 2, 3, 4 waves/SIMD\n", "instruction");
  OPS(RUN)
  return 0;
}
