// Diagnostic microbenchmark (round 2: independent chains for 3-operand ops, packed f16): issue cost per wave-instruction per SIMD of the encodings the specialised decoder uses
// (SDWA, VOPC, VOP3, DPP), W = 1..4 waves per SIMD. hipcc -O3 --offload-arch=gfx950 -o valu2 valu2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)

#define OPS(X) \
  X(0, "v_add_u32", "v_add_u32 %0, %0, %1\n v_add_u32 %2, %2, %1\n v_add_u32 %4, %4, %1\n v_add_u32 %6, %6, %1\n ") \
  X(1, "v_pk_add_f16", "v_pk_add_f16 %0, %0, %1\n v_pk_add_f16 %2, %2, %1\n v_pk_add_f16 %4, %4, %1\n v_pk_add_f16 %6, %6, %1\n ") \
  X(2, "v_pk_min_f16", "v_pk_min_f16 %0, %0, %1\n v_pk_min_f16 %2, %2, %1\n v_pk_min_f16 %4, %4, %1\n v_pk_min_f16 %6, %6, %1\n ") \
  X(3, "v_pk_max_f16", "v_pk_max_f16 %0, %0, %1\n v_pk_max_f16 %2, %2, %1\n v_pk_max_f16 %4, %4, %1\n v_pk_max_f16 %6, %6, %1\n ") \
  X(4, "v_pk_mul_f16", "v_pk_mul_f16 %0, %0, %1\n v_pk_mul_f16 %2, %2, %1\n v_pk_mul_f16 %4, %4, %1\n v_pk_mul_f16 %6, %6, %1\n ") \
  X(5, "v_pk_fma_f16", "v_pk_fma_f16 %0, %0, %1, %3\n v_pk_fma_f16 %2, %2, %1, %3\n v_pk_fma_f16 %4, %4, %1, %3\n v_pk_fma_f16 %6, %6, %1, %3\n ") \
  X(6, "v_pk_add_f16 neg_hi", "v_pk_add_f16 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]\n v_pk_add_f16 %2, %2, %1 neg_lo:[0,1] neg_hi:[0,1]\n v_pk_add_f16 %4, %4, %1 neg_lo:[0,1] neg_hi:[0,1]\n v_pk_add_f16 %6, %6, %1 neg_lo:[0,1] neg_hi:[0,1]\n ") \
  X(7, "v_pk_max_f16 clamp", "v_pk_max_f16 %0, %0, %1 clamp\n v_pk_max_f16 %2, %2, %1 clamp\n v_pk_max_f16 %4, %4, %1 clamp\n v_pk_max_f16 %6, %6, %1 clamp\n ") \
  X(8, "v_med3_f16", "v_med3_f16 %0, %0, %1, %3\n v_med3_f16 %2, %2, %1, %3\n v_med3_f16 %4, %4, %1, %3\n v_med3_f16 %6, %6, %1, %3\n ") \
  X(9, "v_med3_f32", "v_med3_f32 %0, %0, %1, %3\n v_med3_f32 %2, %2, %1, %3\n v_med3_f32 %4, %4, %1, %3\n v_med3_f32 %6, %6, %1, %3\n ") \
  X(10, "v_med3_i32 indep", "v_med3_i32 %0, %0, %1, %3\n v_med3_i32 %2, %2, %1, %3\n v_med3_i32 %4, %4, %1, %3\n v_med3_i32 %6, %6, %1, %3\n ") \
  X(11, "v_med3_u32 indep", "v_med3_u32 %0, %0, %1, %3\n v_med3_u32 %2, %2, %1, %3\n v_med3_u32 %4, %4, %1, %3\n v_med3_u32 %6, %6, %1, %3\n ") \
  X(12, "v_min3_f32", "v_min3_f32 %0, %0, %1, %3\n v_min3_f32 %2, %2, %1, %3\n v_min3_f32 %4, %4, %1, %3\n v_min3_f32 %6, %6, %1, %3\n ") \
  X(13, "v_min3_u32", "v_min3_u32 %0, %0, %1, %3\n v_min3_u32 %2, %2, %1, %3\n v_min3_u32 %4, %4, %1, %3\n v_min3_u32 %6, %6, %1, %3\n ") \
  X(14, "v_lshl_add_u32 indep", "v_lshl_add_u32 %0, %0, 9, %1\n v_lshl_add_u32 %2, %2, 9, %1\n v_lshl_add_u32 %4, %4, 9, %1\n v_lshl_add_u32 %6, %6, 9, %1\n ") \
  X(15, "v_add3_u32 indep", "v_add3_u32 %0, %0, %1, %3\n v_add3_u32 %2, %2, %1, %3\n v_add3_u32 %4, %4, %1, %3\n v_add3_u32 %6, %6, %1, %3\n ") \
  X(16, "v_perm_b32 indep", "v_perm_b32 %0, %0, %1, %3\n v_perm_b32 %2, %2, %1, %3\n v_perm_b32 %4, %4, %1, %3\n v_perm_b32 %6, %6, %1, %3\n ") \
  X(18, "v_cndmask_b32_e64 s", "v_cndmask_b32_e64 %0, %0, %1, s[20:21]\n v_cndmask_b32_e64 %2, %2, %1, s[20:21]\n v_cndmask_b32_e64 %4, %4, %1, s[20:21]\n v_cndmask_b32_e64 %6, %6, %1, s[20:21]\n ") \
  X(19, "v_cmp_eq_u32_e64 s", "v_cmp_eq_u32_e64 s[20:21], %0, %1\n v_cmp_eq_u32_e64 s[20:21], %2, %1\n v_cmp_eq_u32_e64 s[20:21], %4, %1\n v_cmp_eq_u32_e64 s[20:21], %6, %1\n ") \
  X(20, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1\n v_pk_add_u16 %2, %2, %1\n v_pk_add_u16 %4, %4, %1\n v_pk_add_u16 %6, %6, %1\n ") \
  X(21, "v_pk_min_i16", "v_pk_min_i16 %0, %0, %1\n v_pk_min_i16 %2, %2, %1\n v_pk_min_i16 %4, %4, %1\n v_pk_min_i16 %6, %6, %1\n ") \
  X(22, "v_max_i32_sdwa dst w1", "v_max_i32_sdwa %0, %1, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_max_i32_sdwa %2, %1, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_max_i32_sdwa %4, %1, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_max_i32_sdwa %6, %1, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n ") \
  X(23, "v_min_i32_sdwa b0 b1", "v_min_i32_sdwa %0, sext(%1), sext(%3) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1\n v_min_i32_sdwa %2, sext(%1), sext(%3) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1\n v_min_i32_sdwa %4, sext(%1), sext(%3) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1\n v_min_i32_sdwa %6, sext(%1), sext(%3) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1\n ") \
  X(24, "v_max_f16 sdwa w1", "v_max_f16_sdwa %0, %1, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_f16_sdwa %2, %1, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_f16_sdwa %4, %1, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_f16_sdwa %6, %1, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n ") \
  X(25, "v_mul_i32_i24_e64", "v_mul_i32_i24_e64 %0, %0, %1\n v_mul_i32_i24_e64 %2, %2, %1\n v_mul_i32_i24_e64 %4, %4, %1\n v_mul_i32_i24_e64 %6, %6, %1\n ") \
  X(26, "v_pk_mul_lo_u16", "v_pk_mul_lo_u16 %0, %0, %1\n v_pk_mul_lo_u16 %2, %2, %1\n v_pk_mul_lo_u16 %4, %4, %1\n v_pk_mul_lo_u16 %6, %6, %1\n ") \
  X(27, "v_cvt_pk_i16_i32", "v_cvt_pk_i16_i32 %0, %0, %1\n v_cvt_pk_i16_i32 %2, %2, %1\n v_cvt_pk_i16_i32 %4, %4, %1\n v_cvt_pk_i16_i32 %6, %6, %1\n ") \
  X(28, "v_dot2_f32_f16", "v_dot2_f32_f16 %0, %0, %1, %3\n v_dot2_f32_f16 %2, %2, %1, %3\n v_dot2_f32_f16 %4, %4, %1, %3\n v_dot2_f32_f16 %6, %6, %1, %3\n ") \
  X(29, "v_mad_u32_u24", "v_mad_u32_u24 %0, %0, %1, %3\n v_mad_u32_u24 %2, %2, %1, %3\n v_mad_u32_u24 %4, %4, %1, %3\n v_mad_u32_u24 %6, %6, %1, %3\n ") \
  X(30, "v_bfi_b32", "v_bfi_b32 %0, %0, %1, %3\n v_bfi_b32 %2, %2, %1, %3\n v_bfi_b32 %4, %4, %1, %3\n v_bfi_b32 %6, %6, %1, %3\n ") \
  X(31, "v_alignbyte_b32", "v_alignbyte_b32 %0, %0, %1, 1\n v_alignbyte_b32 %2, %2, %1, 1\n v_alignbyte_b32 %4, %4, %1, 1\n v_alignbyte_b32 %6, %6, %1, 1\n ") \
  X(32, "v_and_or_b32 indep", "v_and_or_b32 %0, %0, %1, %3\n v_and_or_b32 %2, %2, %1, %3\n v_and_or_b32 %4, %4, %1, %3\n v_and_or_b32 %6, %6, %1, %3\n ") \
  X(33, "v_or3_b32", "v_or3_b32 %0, %0, %1, %3\n v_or3_b32 %2, %2, %1, %3\n v_or3_b32 %4, %4, %1, %3\n v_or3_b32 %6, %6, %1, %3\n ") \
  X(34, "v_sub_i32 clamp", "v_sub_i32 %0, %0, %1 clamp\n v_sub_i32 %2, %2, %1 clamp\n v_sub_i32 %4, %4, %1 clamp\n v_sub_i32 %6, %6, %1 clamp\n ") \

#define KER(id, name, body)                                                                                            \
  else if (OP == id) { asm volatile(REP32(body) : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : : "vcc", "s20", "s21", "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55"); }

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
