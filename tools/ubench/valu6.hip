// Diagnostic microbenchmark (round 2): more VALU issue costs (explicit VGPRs) + 16-bit/d16 semantics checks.
// hipcc -O3 --offload-arch=gfx950 -o valu6 valu6.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)
#define OPS(X) \
  X(0, "v_add_u32", "v_add_u32 v16, v16, v25\n v_add_u32 v17, v17, v26\n v_add_u32 v18, v18, v27\n v_add_u32 v19, v19, v24\n ") \
  X(1, "v_min_u16", "v_min_u16 v16, v16, v25\n v_min_u16 v17, v17, v26\n v_min_u16 v18, v18, v27\n v_min_u16 v19, v19, v24\n ") \
  X(2, "v_min_i16", "v_min_i16 v16, v16, v25\n v_min_i16 v17, v17, v26\n v_min_i16 v18, v18, v27\n v_min_i16 v19, v19, v24\n ") \
  X(3, "v_min_f16", "v_min_f16 v16, v16, v25\n v_min_f16 v17, v17, v26\n v_min_f16 v18, v18, v27\n v_min_f16 v19, v19, v24\n ") \
  X(4, "v_sub_f16", "v_sub_f16 v16, v16, v25\n v_sub_f16 v17, v17, v26\n v_sub_f16 v18, v18, v27\n v_sub_f16 v19, v19, v24\n ") \
  X(5, "v_mul_f16", "v_mul_f16 v16, v16, v25\n v_mul_f16 v17, v17, v26\n v_mul_f16 v18, v18, v27\n v_mul_f16 v19, v19, v24\n ") \
  X(6, "v_mul_lo_u16", "v_mul_lo_u16 v16, v16, v25\n v_mul_lo_u16 v17, v17, v26\n v_mul_lo_u16 v18, v18, v27\n v_mul_lo_u16 v19, v19, v24\n ") \
  X(7, "v_lshrrev_b32", "v_lshrrev_b32 v16, v25, v16\n v_lshrrev_b32 v17, v26, v17\n v_lshrrev_b32 v18, v27, v18\n v_lshrrev_b32 v19, v24, v19\n ") \
  X(8, "v_lshrrev_b16", "v_lshrrev_b16 v16, v25, v16\n v_lshrrev_b16 v17, v26, v17\n v_lshrrev_b16 v18, v27, v18\n v_lshrrev_b16 v19, v24, v19\n ") \
  X(9, "v_ashrrev_i16", "v_ashrrev_i16 v16, v25, v16\n v_ashrrev_i16 v17, v26, v17\n v_ashrrev_i16 v18, v27, v18\n v_ashrrev_i16 v19, v24, v19\n ") \
  X(10, "v_lshlrev_b16", "v_lshlrev_b16 v16, v25, v16\n v_lshlrev_b16 v17, v26, v17\n v_lshlrev_b16 v18, v27, v18\n v_lshlrev_b16 v19, v24, v19\n ") \
  X(11, "v_sub_u16_e64", "v_sub_u16_e64 v16, v16, v25\n v_sub_u16_e64 v17, v17, v26\n v_sub_u16_e64 v18, v18, v27\n v_sub_u16_e64 v19, v19, v24\n ") \
  X(15, "v_max_i16_e64 const", "v_max_i16 v16, 0xff88, v16\n v_max_i16 v17, 0xff88, v17\n v_max_i16 v18, 0xff88, v18\n v_max_i16 v19, 0xff88, v19\n ") \
  X(16, "v_mad_u16", "v_mad_u16 v16, v16, v25, v30\n v_mad_u16 v17, v17, v26, v31\n v_mad_u16 v18, v18, v27, v28\n v_mad_u16 v19, v19, v24, v29\n ") \
  X(17, "v_mad_i16", "v_mad_i16 v16, v16, v25, v30\n v_mad_i16 v17, v17, v26, v31\n v_mad_i16 v18, v18, v27, v28\n v_mad_i16 v19, v19, v24, v29\n ") \
  X(18, "v_mad_u32_u16", "v_mad_u32_u16 v16, v16, v25, v30\n v_mad_u32_u16 v17, v17, v26, v31\n v_mad_u32_u16 v18, v18, v27, v28\n v_mad_u32_u16 v19, v19, v24, v29\n ") \
  X(19, "v_add_co_u32 vcc", "v_add_co_u32 v16, vcc, v16, v25\n v_add_co_u32 v17, vcc, v17, v26\n v_add_co_u32 v18, vcc, v18, v27\n v_add_co_u32 v19, vcc, v19, v24\n ") \
  X(20, "v_not_b32", "v_not_b32 v16, v25\n v_not_b32 v17, v26\n v_not_b32 v18, v27\n v_not_b32 v19, v24\n ") \
  X(21, "v_and_b32_e64", "v_and_b32_e64 v16, v16, v25\n v_and_b32_e64 v17, v17, v26\n v_and_b32_e64 v18, v18, v27\n v_and_b32_e64 v19, v19, v24\n ") \
  X(22, "v_subrev_u16", "v_subrev_u16 v16, v16, v25\n v_subrev_u16 v17, v17, v26\n v_subrev_u16 v18, v18, v27\n v_subrev_u16 v19, v19, v24\n ") \
  X(23, "v_max_u32", "v_max_u32 v16, v16, v25\n v_max_u32 v17, v17, v26\n v_max_u32 v18, v18, v27\n v_max_u32 v19, v19, v24\n ") \
  X(24, "v_cvt_f32_f16", "v_cvt_f32_f16 v16, v25\n v_cvt_f32_f16 v17, v26\n v_cvt_f32_f16 v18, v27\n v_cvt_f32_f16 v19, v24\n ") \
  X(25, "v_fmac_f32", "v_fmac_f32 v16, v25, v30\n v_fmac_f32 v17, v26, v31\n v_fmac_f32 v18, v27, v28\n v_fmac_f32 v19, v24, v29\n ") \
  X(26, "v_fmamk_f32", "v_fmamk_f32 v16, v25, 0x3f800000, v30\n v_fmamk_f32 v17, v26, 0x3f800000, v31\n v_fmamk_f32 v18, v27, 0x3f800000, v28\n v_fmamk_f32 v19, v24, 0x3f800000, v29\n ") \
  X(27, "v_add_u32 literal", "v_add_u32 v16, 0x12345, v16\n v_add_u32 v17, 0x12345, v17\n v_add_u32 v18, 0x12345, v18\n v_add_u32 v19, 0x12345, v19\n ") \
  X(28, "v_xor_b32 literal", "v_xor_b32 v16, 0x12345, v16\n v_xor_b32 v17, 0x12345, v17\n v_xor_b32 v18, 0x12345, v18\n v_xor_b32 v19, 0x12345, v19\n ") \
  X(29, "v_cndmask vcc(vcmp)", "v_cndmask_b32 v16, v16, v25, vcc\n v_cndmask_b32 v17, v17, v26, vcc\n v_cndmask_b32 v18, v18, v27, vcc\n v_cndmask_b32 v19, v19, v24, vcc\n ") \
  X(30, "v_cndmask_e64 sgpr", "v_cndmask_b32_e64 v16, v16, v25, s[20:21]\n v_cndmask_b32_e64 v17, v17, v26, s[20:21]\n v_cndmask_b32_e64 v18, v18, v27, s[20:21]\n v_cndmask_b32_e64 v19, v19, v24, s[20:21]\n ") \
  X(31, "v_cmp_gt_u16 vcc", "v_cmp_gt_u16 vcc, v16, v25\n v_cmp_gt_u16 vcc, v17, v26\n v_cmp_gt_u16 vcc, v18, v27\n v_cmp_gt_u16 vcc, v19, v24\n ") \
  X(32, "v_cmpx? v_cmp_lt_i32 e64", "v_cmp_lt_i32_e64 s[22:23], v16, v25\n v_cmp_lt_i32_e64 s[22:23], v17, v26\n v_cmp_lt_i32_e64 s[22:23], v18, v27\n v_cmp_lt_i32_e64 s[22:23], v19, v24\n ") \
  X(33, "v_sad_u16", "v_sad_u16 v16, v16, v25, v30\n v_sad_u16 v17, v17, v26, v31\n v_sad_u16 v18, v18, v27, v28\n v_sad_u16 v19, v19, v24, v29\n ") \
  X(34, "v_max_f16 e64 clamp", "v_max_f16_e64 v16, v16, v25 clamp\n v_max_f16_e64 v17, v17, v26 clamp\n v_max_f16_e64 v18, v18, v27 clamp\n v_max_f16_e64 v19, v19, v24 clamp\n ") \
  X(35, "v_add_f16 e64 clamp", "v_add_f16_e64 v16, v16, v25 clamp\n v_add_f16_e64 v17, v17, v26 clamp\n v_add_f16_e64 v18, v18, v27 clamp\n v_add_f16_e64 v19, v19, v24 clamp\n ") \
  X(36, "v_fma_f16", "v_fma_f16 v16, v16, v25, v30\n v_fma_f16 v17, v17, v26, v31\n v_fma_f16 v18, v18, v27, v28\n v_fma_f16 v19, v19, v24, v29\n ") \
  X(37, "v_pk_add_u16 op_sel", "v_pk_add_u16 v16, v16, v25 op_sel:[0,1] op_sel_hi:[1,0]\n v_pk_add_u16 v17, v17, v26 op_sel:[0,1] op_sel_hi:[1,0]\n v_pk_add_u16 v18, v18, v27 op_sel:[0,1] op_sel_hi:[1,0]\n v_pk_add_u16 v19, v19, v24 op_sel:[0,1] op_sel_hi:[1,0]\n ") \
  X(38, "v_swap_b32", "v_swap_b32 v16, v25\n v_swap_b32 v17, v26\n v_swap_b32 v18, v27\n v_swap_b32 v19, v24\n ") \
  X(39, "v_mov_b32 dpp quad", "v_mov_b32_dpp v16, v25 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v17, v26 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v18, v27 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v19, v24 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n ") \
  X(40, "v_mad_u16 op_sel dst hi", "v_mad_u16 v16, v16, v25, v29 op_sel:[0,0,0,1]\n v_mad_u16 v17, v17, v26, v30 op_sel:[0,0,0,1]\n v_mad_u16 v18, v18, v27, v31 op_sel:[0,0,0,1]\n v_mad_u16 v19, v19, v24, v28 op_sel:[0,0,0,1]\n ") \
  X(41, "v_mad_u16 op_sel src hi", "v_mad_u16 v16, v16, v25, v29 op_sel:[1,1,1,0]\n v_mad_u16 v17, v17, v26, v30 op_sel:[1,1,1,0]\n v_mad_u16 v18, v18, v27, v31 op_sel:[1,1,1,0]\n v_mad_u16 v19, v19, v24, v28 op_sel:[1,1,1,0]\n ") \

#define KER(id, name, body) else if (OP == id) { asm volatile(REP32(body) ::: "vcc", "s20", "s21", "s22", "s23", "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31"); }

template <int OP>
__global__ void kern(uint64_t* t, int n)
{
  asm volatile("v_mov_b32 v16, 1\n v_mov_b32 v17, 2\n v_mov_b32 v18, 3\n v_mov_b32 v19, 4\n v_mov_b32 v24, 5\n v_mov_b32 v25, 6\n v_mov_b32 v26, 7\n v_mov_b32 v27, 8\n v_mov_b32 v28, 9\n v_mov_b32 v29, 10\n v_mov_b32 v30, 11\n v_mov_b32 v31, 12\n v_cmp_gt_u32 vcc, v16, v24\n v_cmp_gt_u32 s[20:21], v16, v24" ::: "vcc", "s20", "s21", "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31");
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

/* semantics: what 16-bit ops and d16 LDS loads do to the other half of the destination */
__global__ void sem(uint32_t* o)
{
  __shared__ int8_t lds[64];
  if (threadIdx.x < 64) lds[threadIdx.x] = (int8_t)(threadIdx.x * 7 - 100);
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t r0, r1, r2, r3, r4, r5, r6, r7, r8;
  asm volatile("v_mov_b32 %0, 0xaaaa5555\n v_sub_u16 %0, %0, 1" : "=v"(r0));
  asm volatile("v_mov_b32 %0, 0xaaaa5555\n v_sub_u16_e64 %0, %0, 1" : "=v"(r1));
  asm volatile("v_mov_b32 %0, 0xaaaa5555\n v_mov_b32 %1, 0x00030002\n v_mad_u16 %0, %0, 1, %1 op_sel:[0,0,0,1]" : "=v"(r2), "=v"(r8));
  asm volatile("v_mov_b32 %0, 0xaaaa5555\n v_mov_b32 %1, 0x00030002\n v_mad_u16 %0, %0, 1, %1 op_sel:[1,0,1,0]" : "=v"(r3), "=v"(r8));
  asm volatile("v_mov_b32 %0, 0xaaaa5555\n v_max_i16 %0, %0, 1" : "=v"(r4));
  uint32_t a = 3, b = 5;
  asm volatile("v_mov_b32 %0, 0xaaaa5555\n ds_read_i8_d16 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r5) : "v"(a));
  asm volatile("v_mov_b32 %0, 0xaaaa5555\n ds_read_i8_d16_hi %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r6) : "v"(b));
  asm volatile("v_mov_b32 %0, 0xaaaa5555\n v_add_f16 %0, %0, 1.0" : "=v"(r7));
  o[0] = r0; o[1] = r1; o[2] = r2; o[3] = r3; o[4] = r4; o[5] = r5; o[6] = r6; o[7] = r7;
  o[8] = (uint32_t)(int)lds[3]; o[9] = (uint32_t)(int)lds[5];
}

#define RUN(id, name, body) run<id>(name);
int main()
{
  uint32_t* o;
  (void)hipMalloc(&o, 64 * 4);
  hipLaunchKernelGGL(sem, dim3(1), dim3(64), 0, 0, o);
  uint32_t h[16];
  (void)hipMemcpy(h, o, 16 * 4, hipMemcpyDeviceToHost);
  const char* nm[] = {"v_sub_u16 (VOP2) 0xaaaa5555-1", "v_sub_u16_e64", "v_mad_u16 x*1+0x0002 op_sel dst hi", "v_mad_u16 hi(x)*1+hi(0x00030002) op_sel:[1,0,1,0]",
                      "v_max_i16 (VOP2) 0x5555,1", "ds_read_i8_d16 (lds[3])", "ds_read_i8_d16_hi (lds[5])", "v_add_f16 (VOP2)", "lds[3]", "lds[5]"};
  for (int i = 0; i < 10; ++i) std::printf("SEM %-50s 0x%08x\n", nm[i], h[i]);
  std::printf("%-34s  cycles per wave-instruction per SIMD at 1, 2, 3, 4 waves/SIMD\n", "instruction");
  OPS(RUN)
  return 0;
}
