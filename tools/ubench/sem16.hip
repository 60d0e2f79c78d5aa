#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void sem(uint32_t* o)
{
  __shared__ int8_t lds[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) lds[i] = (int8_t)(i * 7 - 100);
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t r0 = 0xaaaa5555u, r1 = 0xaaaa5555u, r2 = 0x12345678u, r3 = 0x12345678u, r4 = 0;
  uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int8_t*)lds;
  asm volatile("ds_read_i8_d16 %0, %1 offset:3\n s_waitcnt lgkmcnt(0)" : "+v"(r0) : "v"(a));
  asm volatile("ds_read_i8_d16_hi %0, %1 offset:5\n s_waitcnt lgkmcnt(0)" : "+v"(r1) : "v"(a));
  asm volatile("ds_read_u8_d16_hi %0, %1 offset:5\n s_waitcnt lgkmcnt(0)" : "+v"(r2) : "v"(a));
  asm volatile("ds_read_i8 %0, %1 offset:5\n s_waitcnt lgkmcnt(0)" : "+v"(r4) : "v"(a));
  uint32_t w = 0x00F10017u; /* lo byte 0x17, hi-half byte 0xF1 */
  asm volatile("ds_write_b8_d16_hi %0, %1 offset:10\n ds_write_b8 %0, %1 offset:11\n s_waitcnt lgkmcnt(0)" :: "v"(a), "v"(w) : "memory");
  asm volatile("ds_read_i8 %0, %1 offset:10\n s_waitcnt lgkmcnt(0)" : "=v"(r3) : "v"(a));
  uint32_t r5;
  asm volatile("ds_read_i8 %0, %1 offset:11\n s_waitcnt lgkmcnt(0)" : "=v"(r5) : "v"(a));
  o[0] = r0; o[1] = r1; o[2] = r2; o[3] = r3; o[4] = r4; o[5] = r5; o[6] = (uint32_t)(int)lds[3]; o[7] = (uint32_t)(int)lds[5]; o[8] = a;
  /* packed ops */
  uint32_t p0 = 0x0005FFF0u, p1 = 0x00030004u, q;
  asm volatile("v_pk_sub_i16 %0, %1, %2" : "=v"(q) : "v"(p0), "v"(p1)); o[9] = q;
  asm volatile("v_pk_max_i16 %0, %1, %2" : "=v"(q) : "v"(p0), "v"(p1)); o[10] = q;
  asm volatile("v_pk_mul_lo_u16 %0, %1, %1" : "=v"(q) : "v"(p0)); o[11] = q;
  asm volatile("v_pk_ashrrev_i16 %0, 15, %1" : "=v"(q) : "v"(p0)); o[12] = q;
  uint32_t c2 = 0xfffefffeu; /* -2, -2 */
  asm volatile("v_pk_mad_i16 %0, %1, %2, %3" : "=v"(q) : "v"(p1), "v"(c2), "v"(p0)); o[13] = q;
}
int main()
{
  uint32_t* o;
  (void)hipMalloc(&o, 64 * 4);
  hipLaunchKernelGGL(sem, dim3(1), dim3(64), 0, 0, o);
  uint32_t h[16];
  (void)hipMemcpy(h, o, 16 * 4, hipMemcpyDeviceToHost);
  const char* nm[] = {"ds_read_i8_d16 (0xaaaa5555, lds[3])", "ds_read_i8_d16_hi (0xaaaa5555, lds[5])", "ds_read_u8_d16_hi (0x12345678, lds[5])",
                      "read back lds[10] after ds_write_b8_d16_hi 0x00F10017", "ds_read_i8 lds[5]", "read lds[11] after ds_write_b8 0x..17",
                      "lds[3]", "lds[5]", "lds base", "pk_sub_i16 (5,-16)-(3,4)", "pk_max_i16", "pk_mul_lo_u16 sq", "pk_ashrrev_i16 15", "pk_mad_i16 (3,4)*(-2)+(5,-16)"};
  for (int i = 0; i < 14; ++i) std::printf("%-55s 0x%08x\n", nm[i], h[i]);
  return 0;
}
