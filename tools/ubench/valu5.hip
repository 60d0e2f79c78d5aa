// Diagnostic microbenchmark (round 2): VALU issue cost with explicit VGPR banks (bank = reg % 4).
// "CONFLICT": the sources share the destination's bank. hipcc -O3 --offload-arch=gfx950 -o valu5 valu5.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)
#define OPS(X) \
  X(0, "v_add_u32", "v_add_u32 v16, v16, v25\n v_add_u32 v17, v17, v26\n v_add_u32 v18, v18, v27\n v_add_u32 v19, v19, v24\n ") \
  X(1, "v_add_u32 CONFLICT", "v_add_u32 v16, v16, v24\n v_add_u32 v17, v17, v25\n v_add_u32 v18, v18, v26\n v_add_u32 v19, v19, v27\n ") \
  X(2, "v_min_i32", "v_min_i32 v16, v16, v25\n v_min_i32 v17, v17, v26\n v_min_i32 v18, v18, v27\n v_min_i32 v19, v19, v24\n ") \
  X(3, "v_min_i32 CONFLICT", "v_min_i32 v16, v16, v24\n v_min_i32 v17, v17, v25\n v_min_i32 v18, v18, v26\n v_min_i32 v19, v19, v27\n ") \
  X(4, "v_max_f32", "v_max_f32 v16, v16, v25\n v_max_f32 v17, v17, v26\n v_max_f32 v18, v18, v27\n v_max_f32 v19, v19, v24\n ") \
  X(5, "v_max_f32 CONFLICT", "v_max_f32 v16, v16, v24\n v_max_f32 v17, v17, v25\n v_max_f32 v18, v18, v26\n v_max_f32 v19, v19, v27\n ") \
  X(6, "v_lshlrev_b32", "v_lshlrev_b32 v16, v25, v16\n v_lshlrev_b32 v17, v26, v17\n v_lshlrev_b32 v18, v27, v18\n v_lshlrev_b32 v19, v24, v19\n ") \
  X(7, "v_lshlrev_b32 CONFLICT", "v_lshlrev_b32 v16, v24, v16\n v_lshlrev_b32 v17, v25, v17\n v_lshlrev_b32 v18, v26, v18\n v_lshlrev_b32 v19, v27, v19\n ") \
  X(8, "v_mul_u32_u24", "v_mul_u32_u24 v16, v16, v25\n v_mul_u32_u24 v17, v17, v26\n v_mul_u32_u24 v18, v18, v27\n v_mul_u32_u24 v19, v19, v24\n ") \
  X(9, "v_mul_u32_u24 CONFLICT", "v_mul_u32_u24 v16, v16, v24\n v_mul_u32_u24 v17, v17, v25\n v_mul_u32_u24 v18, v18, v26\n v_mul_u32_u24 v19, v19, v27\n ") \
  X(10, "v_cndmask_b32 vcc", "v_cndmask_b32 v16, v16, v25, vcc\n v_cndmask_b32 v17, v17, v26, vcc\n v_cndmask_b32 v18, v18, v27, vcc\n v_cndmask_b32 v19, v19, v24, vcc\n ") \
  X(11, "v_cndmask_b32 vcc CONFLICT", "v_cndmask_b32 v16, v16, v24, vcc\n v_cndmask_b32 v17, v17, v25, vcc\n v_cndmask_b32 v18, v18, v26, vcc\n v_cndmask_b32 v19, v19, v27, vcc\n ") \
  X(12, "v_cmp_eq_u32 vcc", "v_cmp_eq_u32 vcc, v16, v25\n v_cmp_eq_u32 vcc, v17, v26\n v_cmp_eq_u32 vcc, v18, v27\n v_cmp_eq_u32 vcc, v19, v24\n ") \
  X(13, "v_cmp_eq_u32 vcc CONFLICT", "v_cmp_eq_u32 vcc, v16, v24\n v_cmp_eq_u32 vcc, v17, v25\n v_cmp_eq_u32 vcc, v18, v26\n v_cmp_eq_u32 vcc, v19, v27\n ") \
  X(14, "v_med3_i32", "v_med3_i32 v16, v16, v25, v30\n v_med3_i32 v17, v17, v26, v31\n v_med3_i32 v18, v18, v27, v28\n v_med3_i32 v19, v19, v24, v29\n ") \
  X(15, "v_med3_i32 CONFLICT", "v_med3_i32 v16, v16, v24, v28\n v_med3_i32 v17, v17, v25, v29\n v_med3_i32 v18, v18, v26, v30\n v_med3_i32 v19, v19, v27, v31\n ") \
  X(16, "v_med3_f32", "v_med3_f32 v16, v16, v25, v30\n v_med3_f32 v17, v17, v26, v31\n v_med3_f32 v18, v18, v27, v28\n v_med3_f32 v19, v19, v24, v29\n ") \
  X(17, "v_med3_f32 CONFLICT", "v_med3_f32 v16, v16, v24, v28\n v_med3_f32 v17, v17, v25, v29\n v_med3_f32 v18, v18, v26, v30\n v_med3_f32 v19, v19, v27, v31\n ") \
  X(18, "v_min3_u32", "v_min3_u32 v16, v16, v25, v30\n v_min3_u32 v17, v17, v26, v31\n v_min3_u32 v18, v18, v27, v28\n v_min3_u32 v19, v19, v24, v29\n ") \
  X(19, "v_min3_u32 CONFLICT", "v_min3_u32 v16, v16, v24, v28\n v_min3_u32 v17, v17, v25, v29\n v_min3_u32 v18, v18, v26, v30\n v_min3_u32 v19, v19, v27, v31\n ") \
  X(20, "v_lshl_add_u32", "v_lshl_add_u32 v16, v16, 9, v25\n v_lshl_add_u32 v17, v17, 9, v26\n v_lshl_add_u32 v18, v18, 9, v27\n v_lshl_add_u32 v19, v19, 9, v24\n ") \
  X(21, "v_lshl_add_u32 CONFLICT", "v_lshl_add_u32 v16, v16, 9, v24\n v_lshl_add_u32 v17, v17, 9, v25\n v_lshl_add_u32 v18, v18, 9, v26\n v_lshl_add_u32 v19, v19, 9, v27\n ") \
  X(22, "v_add3_u32", "v_add3_u32 v16, v16, v25, v30\n v_add3_u32 v17, v17, v26, v31\n v_add3_u32 v18, v18, v27, v28\n v_add3_u32 v19, v19, v24, v29\n ") \
  X(23, "v_add3_u32 CONFLICT", "v_add3_u32 v16, v16, v24, v28\n v_add3_u32 v17, v17, v25, v29\n v_add3_u32 v18, v18, v26, v30\n v_add3_u32 v19, v19, v27, v31\n ") \
  X(24, "v_perm_b32", "v_perm_b32 v16, v16, v25, v30\n v_perm_b32 v17, v17, v26, v31\n v_perm_b32 v18, v18, v27, v28\n v_perm_b32 v19, v19, v24, v29\n ") \
  X(25, "v_perm_b32 CONFLICT", "v_perm_b32 v16, v16, v24, v28\n v_perm_b32 v17, v17, v25, v29\n v_perm_b32 v18, v18, v26, v30\n v_perm_b32 v19, v19, v27, v31\n ") \
  X(26, "v_bfe_i32", "v_bfe_i32 v16, v16, 8, 8\n v_bfe_i32 v17, v17, 8, 8\n v_bfe_i32 v18, v18, 8, 8\n v_bfe_i32 v19, v19, 8, 8\n ") \
  X(27, "v_bfe_i32 CONFLICT", "v_bfe_i32 v16, v16, 8, 8\n v_bfe_i32 v17, v17, 8, 8\n v_bfe_i32 v18, v18, 8, 8\n v_bfe_i32 v19, v19, 8, 8\n ") \
  X(28, "v_pk_add_f16", "v_pk_add_f16 v16, v16, v25\n v_pk_add_f16 v17, v17, v26\n v_pk_add_f16 v18, v18, v27\n v_pk_add_f16 v19, v19, v24\n ") \
  X(29, "v_pk_add_f16 CONFLICT", "v_pk_add_f16 v16, v16, v24\n v_pk_add_f16 v17, v17, v25\n v_pk_add_f16 v18, v18, v26\n v_pk_add_f16 v19, v19, v27\n ") \
  X(30, "v_pk_max_i16", "v_pk_max_i16 v16, v16, v25\n v_pk_max_i16 v17, v17, v26\n v_pk_max_i16 v18, v18, v27\n v_pk_max_i16 v19, v19, v24\n ") \
  X(31, "v_pk_max_i16 CONFLICT", "v_pk_max_i16 v16, v16, v24\n v_pk_max_i16 v17, v17, v25\n v_pk_max_i16 v18, v18, v26\n v_pk_max_i16 v19, v19, v27\n ") \
  X(32, "v_pk_fma_f16", "v_pk_fma_f16 v16, v16, v25, v30\n v_pk_fma_f16 v17, v17, v26, v31\n v_pk_fma_f16 v18, v18, v27, v28\n v_pk_fma_f16 v19, v19, v24, v29\n ") \
  X(33, "v_pk_fma_f16 CONFLICT", "v_pk_fma_f16 v16, v16, v24, v28\n v_pk_fma_f16 v17, v17, v25, v29\n v_pk_fma_f16 v18, v18, v26, v30\n v_pk_fma_f16 v19, v19, v27, v31\n ") \
  X(34, "v_sub_u32_sdwa sext b1", "v_sub_u32_sdwa v16, v16, sext(v25) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa v17, v17, sext(v26) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa v18, v18, sext(v27) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa v19, v19, sext(v24) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n ") \
  X(35, "v_sub_u32_sdwa sext b1 CONFLICT", "v_sub_u32_sdwa v16, v16, sext(v24) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa v17, v17, sext(v25) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa v18, v18, sext(v26) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n v_sub_u32_sdwa v19, v19, sext(v27) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n ") \
  X(36, "v_mul_i32_i24_sdwa dst b1", "v_mul_i32_i24_sdwa v16, v25, v30 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa v17, v26, v31 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa v18, v27, v28 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa v19, v24, v29 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n ") \
  X(37, "v_mul_i32_i24_sdwa dst b1 CONFLICT", "v_mul_i32_i24_sdwa v16, v24, v28 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa v17, v25, v29 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa v18, v26, v30 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n v_mul_i32_i24_sdwa v19, v27, v31 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n ") \
  X(38, "v_max_i16_sdwa dst w1", "v_max_i16_sdwa v16, v25, v30 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_i16_sdwa v17, v26, v31 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_i16_sdwa v18, v27, v28 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_i16_sdwa v19, v24, v29 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n ") \
  X(39, "v_max_i16_sdwa dst w1 CONFLICT", "v_max_i16_sdwa v16, v24, v28 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_i16_sdwa v17, v25, v29 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_i16_sdwa v18, v26, v30 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n v_max_i16_sdwa v19, v27, v31 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n ") \
  X(40, "v_add_u32_dpp", "v_add_u32_dpp v16, v25, v16 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp v17, v26, v17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp v18, v27, v18 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp v19, v24, v19 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n ") \
  X(41, "v_add_u32_dpp CONFLICT", "v_add_u32_dpp v16, v24, v16 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp v17, v25, v17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp v18, v26, v18 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp v19, v27, v19 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n ") \
  X(42, "v_sub_u32_e64", "v_sub_u32_e64 v16, v16, v25\n v_sub_u32_e64 v17, v17, v26\n v_sub_u32_e64 v18, v18, v27\n v_sub_u32_e64 v19, v19, v24\n ") \
  X(43, "v_sub_u32_e64 CONFLICT", "v_sub_u32_e64 v16, v16, v24\n v_sub_u32_e64 v17, v17, v25\n v_sub_u32_e64 v18, v18, v26\n v_sub_u32_e64 v19, v19, v27\n ") \
  X(44, "v_fma_f32", "v_fma_f32 v16, v16, v25, v30\n v_fma_f32 v17, v17, v26, v31\n v_fma_f32 v18, v18, v27, v28\n v_fma_f32 v19, v19, v24, v29\n ") \
  X(45, "v_fma_f32 CONFLICT", "v_fma_f32 v16, v16, v24, v28\n v_fma_f32 v17, v17, v25, v29\n v_fma_f32 v18, v18, v26, v30\n v_fma_f32 v19, v19, v27, v31\n ") \
  X(46, "v_xor_b32", "v_xor_b32 v16, v16, v25\n v_xor_b32 v17, v17, v26\n v_xor_b32 v18, v18, v27\n v_xor_b32 v19, v19, v24\n ") \
  X(47, "v_xor_b32 CONFLICT", "v_xor_b32 v16, v16, v24\n v_xor_b32 v17, v17, v25\n v_xor_b32 v18, v18, v26\n v_xor_b32 v19, v19, v27\n ") \
  X(48, "v_min_u32", "v_min_u32 v16, v16, v25\n v_min_u32 v17, v17, v26\n v_min_u32 v18, v18, v27\n v_min_u32 v19, v19, v24\n ") \
  X(49, "v_min_u32 CONFLICT", "v_min_u32 v16, v16, v24\n v_min_u32 v17, v17, v25\n v_min_u32 v18, v18, v26\n v_min_u32 v19, v19, v27\n ") \
  X(50, "v_max_i32", "v_max_i32 v16, v16, v25\n v_max_i32 v17, v17, v26\n v_max_i32 v18, v18, v27\n v_max_i32 v19, v19, v24\n ") \
  X(51, "v_max_i32 CONFLICT", "v_max_i32 v16, v16, v24\n v_max_i32 v17, v17, v25\n v_max_i32 v18, v18, v26\n v_max_i32 v19, v19, v27\n ") \
  X(52, "v_mul_i32_i24", "v_mul_i32_i24 v16, v16, v25\n v_mul_i32_i24 v17, v17, v26\n v_mul_i32_i24 v18, v18, v27\n v_mul_i32_i24 v19, v19, v24\n ") \
  X(53, "v_mul_i32_i24 CONFLICT", "v_mul_i32_i24 v16, v16, v24\n v_mul_i32_i24 v17, v17, v25\n v_mul_i32_i24 v18, v18, v26\n v_mul_i32_i24 v19, v19, v27\n ") \
  X(54, "v_max_i16", "v_max_i16 v16, v16, v25\n v_max_i16 v17, v17, v26\n v_max_i16 v18, v18, v27\n v_max_i16 v19, v19, v24\n ") \
  X(55, "v_max_i16 CONFLICT", "v_max_i16 v16, v16, v24\n v_max_i16 v17, v17, v25\n v_max_i16 v18, v18, v26\n v_max_i16 v19, v19, v27\n ") \

#define KER(id, name, body) else if (OP == id) { asm volatile(REP32(body) ::: "vcc", "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31"); }

template <int OP>
__global__ void kern(uint64_t* t, int n)
{
  asm volatile("v_mov_b32 v16, 1\n v_mov_b32 v17, 2\n v_mov_b32 v18, 3\n v_mov_b32 v19, 4\n v_mov_b32 v24, 5\n v_mov_b32 v25, 6\n v_mov_b32 v26, 7\n v_mov_b32 v27, 8\n v_mov_b32 v28, 9\n v_mov_b32 v29, 10\n v_mov_b32 v30, 11\n v_mov_b32 v31, 12\n s_mov_b64 vcc, -1" ::: "vcc", "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31");
  __syncthreads();
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (false) { }
    OPS(KER)
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) t[threadIdx.x >> 6] = t1 - t0;
}

template <int OP>
void run(const char* name)
{
  uint64_t* t;
  (void)hipMalloc(&t, 64 * 8);
  std::printf("%-34s", name);
  for (int w = 1; w <= 4; ++w) {
    const int n = 64, threads = 256 * w;
    hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 0, 0, t, n);
    hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(threads), 0, 0, t, n);
    (void)hipDeviceSynchronize();
    uint64_t ht[64];
    (void)hipMemcpy(ht, t, 64 * 8, hipMemcpyDeviceToHost);
    uint64_t mx = 0;
    for (int q = 0; q < threads / 64; ++q) mx = ht[q] > mx ? ht[q] : mx;
    std::printf("  %5.2f", mx / (double(n) * 128.0 * w));
  }
  std::printf("\n");
  (void)hipFree(t);
}
#define RUN(id, name, body) run<id>(name);
int main()
{
  std::printf("%-34s  cycles per wave-instruction per SIMD at 1, 2, 3, 4 waves/SIMD\n", "instruction");
  OPS(RUN)
  return 0;
}
