// Diagnostic microbenchmark: issue cost per wave-instruction per SIMD of the encodings the specialised decoder uses
// (SDWA, VOPC, VOP3, DPP), W = 1..4 waves per SIMD. hipcc -O3 --offload-arch=gfx950 -o valu2 valu2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)

#define OPS(X) \
  X(0, "v_and_b32", "v_and_b32 %0, %0, %1\n v_and_b32 %2, %2, %3\n v_and_b32 %4, %4, %5\n v_and_b32 %6, %6, %7\n ") \
  X(1, "v_or_b32", "v_or_b32 %0, %0, %1\n v_or_b32 %2, %2, %3\n v_or_b32 %4, %4, %5\n v_or_b32 %6, %6, %7\n ") \
  X(2, "v_xor_b32", "v_xor_b32 %0, %0, %1\n v_xor_b32 %2, %2, %3\n v_xor_b32 %4, %4, %5\n v_xor_b32 %6, %6, %7\n ") \
  X(3, "v_lshlrev_b32", "v_lshlrev_b32 %0, 1, %0\n v_lshlrev_b32 %2, 1, %2\n v_lshlrev_b32 %4, 1, %4\n v_lshlrev_b32 %6, 1, %6\n ") \
  X(4, "v_ashrrev_i32", "v_ashrrev_i32 %0, 1, %0\n v_ashrrev_i32 %2, 1, %2\n v_ashrrev_i32 %4, 1, %4\n v_ashrrev_i32 %6, 1, %6\n ") \
  X(5, "v_min_i32", "v_min_i32 %0, %0, %1\n v_min_i32 %2, %2, %3\n v_min_i32 %4, %4, %5\n v_min_i32 %6, %6, %7\n ") \
  X(6, "v_min_i16", "v_min_i16 %0, %0, %1\n v_min_i16 %2, %2, %3\n v_min_i16 %4, %4, %5\n v_min_i16 %6, %6, %7\n ") \
  X(7, "v_max_u16", "v_max_u16 %0, %0, %1\n v_max_u16 %2, %2, %3\n v_max_u16 %4, %4, %5\n v_max_u16 %6, %6, %7\n ") \
  X(8, "v_add_u16", "v_add_u16 %0, %0, %1\n v_add_u16 %2, %2, %3\n v_add_u16 %4, %4, %5\n v_add_u16 %6, %6, %7\n ") \
  X(9, "v_sub_u16", "v_sub_u16 %0, %0, %1\n v_sub_u16 %2, %2, %3\n v_sub_u16 %4, %4, %5\n v_sub_u16 %6, %6, %7\n ") \
  X(10, "v_mul_lo_u16", "v_mul_lo_u16 %0, %0, %1\n v_mul_lo_u16 %2, %2, %3\n v_mul_lo_u16 %4, %4, %5\n v_mul_lo_u16 %6, %6, %7\n ") \
  X(11, "v_mul_u32_u24", "v_mul_u32_u24 %0, %0, %1\n v_mul_u32_u24 %2, %2, %3\n v_mul_u32_u24 %4, %4, %5\n v_mul_u32_u24 %6, %6, %7\n ") \
  X(12, "v_cndmask_b32 vcc", "v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %4, %4, %5, vcc\n v_cndmask_b32 %6, %6, %7, vcc\n ") \
  X(13, "v_cmp_eq_u32 vcc", "v_cmp_eq_u32 vcc, %0, %1\n v_cmp_eq_u32 vcc, %2, %3\n v_cmp_eq_u32 vcc, %4, %5\n v_cmp_eq_u32 vcc, %6, %7\n ") \
  X(14, "v_subrev_u32", "v_subrev_u32 %0, %0, %1\n v_subrev_u32 %2, %2, %3\n v_subrev_u32 %4, %4, %5\n v_subrev_u32 %6, %6, %7\n ") \
  X(15, "v_add_f32", "v_add_f32 %0, %0, %1\n v_add_f32 %2, %2, %3\n v_add_f32 %4, %4, %5\n v_add_f32 %6, %6, %7\n ") \
  X(16, "v_sub_f32", "v_sub_f32 %0, %0, %1\n v_sub_f32 %2, %2, %3\n v_sub_f32 %4, %4, %5\n v_sub_f32 %6, %6, %7\n ") \
  X(17, "v_mul_f32", "v_mul_f32 %0, %0, %1\n v_mul_f32 %2, %2, %3\n v_mul_f32 %4, %4, %5\n v_mul_f32 %6, %6, %7\n ") \
  X(18, "v_min_f32", "v_min_f32 %0, %0, %1\n v_min_f32 %2, %2, %3\n v_min_f32 %4, %4, %5\n v_min_f32 %6, %6, %7\n ") \
  X(19, "v_max_f32", "v_max_f32 %0, %0, %1\n v_max_f32 %2, %2, %3\n v_max_f32 %4, %4, %5\n v_max_f32 %6, %6, %7\n ") \
  X(20, "v_fma_f32", "v_fma_f32 %0, %0, %1, %0\n v_fma_f32 %2, %2, %3, %2\n v_fma_f32 %4, %4, %5, %4\n v_fma_f32 %6, %6, %7, %6\n ") \
  X(21, "v_med3_f32", "v_med3_f32 %0, %0, %1, 1.0\n v_med3_f32 %2, %2, %3, 1.0\n v_med3_f32 %4, %4, %5, 1.0\n v_med3_f32 %6, %6, %7, 1.0\n ") \
  X(22, "v_max_f32 e64 clamp", "v_max_f32_e64 %0, %0, %1 clamp\n v_max_f32_e64 %2, %2, %3 clamp\n v_max_f32_e64 %4, %4, %5 clamp\n v_max_f32_e64 %6, %6, %7 clamp\n ") \
  X(23, "v_add_f32 e64 neg abs", "v_add_f32_e64 %0, -%0, |%1|\n v_add_f32_e64 %2, -%2, |%3|\n v_add_f32_e64 %4, -%4, |%5|\n v_add_f32_e64 %6, -%6, |%7|\n ") \
  X(24, "v_pk_add_f32", "v_pk_add_f32 v[40:41], v[40:41], v[48:49]\n v_pk_add_f32 v[42:43], v[42:43], v[50:51]\n v_pk_add_f32 v[44:45], v[44:45], v[52:53]\n v_pk_add_f32 v[46:47], v[46:47], v[54:55]\n ") \
  X(25, "v_pk_mul_f32", "v_pk_mul_f32 v[40:41], v[40:41], v[48:49]\n v_pk_mul_f32 v[42:43], v[42:43], v[50:51]\n v_pk_mul_f32 v[44:45], v[44:45], v[52:53]\n v_pk_mul_f32 v[46:47], v[46:47], v[54:55]\n ") \
  X(26, "v_pk_fma_f32", "v_pk_fma_f32 v[40:41], v[40:41], v[48:49], v[40:41]\n v_pk_fma_f32 v[42:43], v[42:43], v[50:51], v[42:43]\n v_pk_fma_f32 v[44:45], v[44:45], v[52:53], v[44:45]\n v_pk_fma_f32 v[46:47], v[46:47], v[54:55], v[46:47]\n ") \
  X(27, "v_max_f16", "v_max_f16 %0, %0, %1\n v_max_f16 %2, %2, %3\n v_max_f16 %4, %4, %5\n v_max_f16 %6, %6, %7\n ") \
  X(28, "v_add_f16", "v_add_f16 %0, %0, %1\n v_add_f16 %2, %2, %3\n v_add_f16 %4, %4, %5\n v_add_f16 %6, %6, %7\n ") \
  X(29, "v_pk_max_f16", "v_pk_max_f16 %0, %0, %1\n v_pk_max_f16 %2, %2, %3\n v_pk_max_f16 %4, %4, %5\n v_pk_max_f16 %6, %6, %7\n ") \
  X(30, "v_cvt_f32_i32", "v_cvt_f32_i32 %0, %1\n v_cvt_f32_i32 %2, %3\n v_cvt_f32_i32 %4, %5\n v_cvt_f32_i32 %6, %7\n ") \
  X(31, "v_cvt_f32_ubyte1", "v_cvt_f32_ubyte1 %0, %1\n v_cvt_f32_ubyte1 %2, %3\n v_cvt_f32_ubyte1 %4, %5\n v_cvt_f32_ubyte1 %6, %7\n ") \
  X(32, "v_mov_b32", "v_mov_b32 %0, %1\n v_mov_b32 %2, %3\n v_mov_b32 %4, %5\n v_mov_b32 %6, %7\n ") \
  X(33, "v_bfe_i32", "v_bfe_i32 %0, %0, 8, 8\n v_bfe_i32 %2, %2, 8, 8\n v_bfe_i32 %4, %4, 8, 8\n v_bfe_i32 %6, %6, 8, 8\n ") \
  X(34, "v_and_or_b32", "v_and_or_b32 %0, %0, %1, %0\n v_and_or_b32 %2, %2, %3, %2\n v_and_or_b32 %4, %4, %5, %4\n v_and_or_b32 %6, %6, %7, %6\n ") \
  X(35, "v_xad_u32", "v_xad_u32 %0, %0, %1, %0\n v_xad_u32 %2, %2, %3, %2\n v_xad_u32 %4, %4, %5, %4\n v_xad_u32 %6, %6, %7, %6\n ") \
  X(36, "v_max3_i32", "v_max3_i32 %0, %0, %1, %0\n v_max3_i32 %2, %2, %3, %2\n v_max3_i32 %4, %4, %5, %4\n v_max3_i32 %6, %6, %7, %6\n ") \
  X(37, "v_add_u32 dpp", "v_add_u32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %2, %3, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %4, %5, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %6, %7, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n ") \
  X(38, "v_add_i32 clamp e64", "v_add_i32 %0, %0, %1 clamp\n v_add_i32 %2, %2, %3 clamp\n v_add_i32 %4, %4, %5 clamp\n v_add_i32 %6, %6, %7 clamp\n ") \
  X(39, "v_sub_i16 clamp", "v_sub_i16 %0, %0, %1 clamp\n v_sub_i16 %2, %2, %3 clamp\n v_sub_i16 %4, %4, %5 clamp\n v_sub_i16 %6, %6, %7 clamp\n ") \
  X(40, "v_ldexp_f32", "v_ldexp_f32 %0, %0, %1\n v_ldexp_f32 %2, %2, %3\n v_ldexp_f32 %4, %4, %5\n v_ldexp_f32 %6, %6, %7\n ") \
  X(41, "v_xor_b32 e64 (mod?)", "v_xor_b32_e64 %0, %0, %1\n v_xor_b32_e64 %2, %2, %3\n v_xor_b32_e64 %4, %4, %5\n v_xor_b32_e64 %6, %6, %7\n ") \

#define KER(id, name, body)                                                                                            \
  else if (OP == id) { asm volatile(REP32(body) : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : : "vcc", "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55"); }

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
