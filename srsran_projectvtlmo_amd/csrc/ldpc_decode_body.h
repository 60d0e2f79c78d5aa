/*
 * Device code of the LDPC decoder shared by the translation units that instantiate it: ldpc_hip_kernels.hip (generic
 * kernel, the core specialised kernels and the mixed kernel) and ldpc_spec_kernels_*.hip (further specialised
 * kernels, compiled in parallel). Included once per translation unit.
 */
#pragma once
/*
 * gfx950 (MI355X, CDNA4) decoder kernels of the 5G-NR PUSCH LDPC decode path.
 *
 *  ldpc_decode_kernel          layered normalised min-sum decoder, one workgroup per codeblock with the whole decoder
 *                              state resident in LDS: int8 soft bits (N_full x Z) and one compressed check-to-variable
 *                              record per lifted check node (BG1 Z=384: 26 KiB + 75 KiB). Bit-exact with
 *                              ldpc_decoder_generic (lib/phy/upper/channel_coding/ldpc/ldpc_decoder_impl.cpp:60-308,
 *                              ldpc_decoder_generic.cpp:30-128) including the CRC early stop.
 *  ldpc_rate_dematch_kernel    bit de-interleave + rate dematching + HARQ combining
 *                              (ldpc_rate_dematcher_impl.cpp:46-213), one workgroup per codeblock.
 *
 * Work mapping of the decoder. A base-graph row m lifts to Z independent check nodes t. A 64-lane wave takes 64 (or,
 * with edge splitting, 32) consecutive check nodes of one row, so the row -- degree, edge list, shifts -- is
 * wave-uniform and read through the scalar unit, while the Zc cyclic shift is a per-lane LDS byte gather
 * soft[col][(t + shift) mod Z]. The two-minimum search of a check node runs over the row's edges in the reference's
 * order with its strict '<' (first edge wins). Consecutive rows that share no variable node form one step and are
 * updated concurrently, one barrier per step: they read and write disjoint soft bits, so the result is identical to
 * the layer-serial order of ldpc_decoder_impl.cpp:116-123.
 */
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "ldpc_hip_device.h"
#include "ldpc_spec.h"

namespace ldpc_hip {

namespace {

constexpr int LLR_MAX = 120;
constexpr int LLR_INF = 127;
constexpr int LLR_INTERNAL_INF = LLR_MAX + 1; /* decoder-internal infinity, see "Check-to-variable storage" */

__device__ __forceinline__ bool llr_isinf(int v) { return v > LLR_MAX || v < -LLR_MAX; }

/* Wave-wide XOR reduction (wave64): DPP within each 16-lane row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
 * row_mirror), then the four rows' lanes 0, 16, 32, 48 read out as scalars: no LDS round trips (a ds_bpermute
 * butterfly costs six). Every lane gets the total. */
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
  v ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xb1, 0xf, 0xf, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4e, 0xf, 0xf, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x141, 0xf, 0xf, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x140, 0xf, 0xf, false));
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 0) ^
                               __builtin_amdgcn_readlane(static_cast<int>(v), 16) ^
                               __builtin_amdgcn_readlane(static_cast<int>(v), 32) ^
                               __builtin_amdgcn_readlane(static_cast<int>(v), 48));
}

/* Wave-wide maximum of non-negative ints, the same DPP pattern as wave_xor; every lane gets the result. */
__device__ __forceinline__ int wave_max(int v)
{
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xb1, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4e, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, false));
  return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

/* (a(x) * b(x)) mod G(x) over GF(2); a, b of degree < order; poly includes the x^order term. */
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b, int order, uint32_t poly)
{
  /* a * b mod poly over GF(2) for a, b < x^order (order <= 24; poly includes its x^order term), Horner over the bits
   * of b from the top: 32-bit operations only, the remainder reduced at every step */
  const uint32_t top = 1U << order;
  uint32_t       r   = 0;
  for (int i = order - 1; i >= 0; --i) {
    r <<= 1;
    r ^= (r & top) ? poly : 0U;
    r ^= ((b >> i) & 1U) ? a : 0U;
  }
  return r;
}

__device__ __forceinline__ void crc_params(int poly_id, int& order, uint32_t& poly)
{
  /* hw_dec_cb_crc_type numbering; polynomials of crc_calculator_generic_impl.cpp:28-56 */
  if (poly_id == LDPC_HIP_CRC16) {
    order = 16;
    poly  = 0x11021U;
  } else if (poly_id == LDPC_HIP_CRC24B) {
    order = 24;
    poly  = 0x1800063U;
  } else {
    order = 24;
    poly  = 0x1864cfbU;
  }
}

/* CRC remainder of the first L bits of the packed (MSB-first) message in LDS. Linear decomposition:
 * front-pad to nw 32-bit words (leading zeros do not change a zero-init CRC), remainder =
 * XOR_w [(W_w * x^r mod G) * (x^(32 (nw-1-w)) mod G) mod G]. Block-uniform result. s_table: the poly's LDS copy
 * (CRC_LDS_WORDS: slicing-by-4 tables T_0..T_3, then the powers), so a word's CRC is four independent LDS lookups
 * and its power one more, with no global load on the early-stop path. */
__device__ uint32_t block_crc(const uint8_t* hb, int L, int poly_id, const uint32_t* s_table, uint32_t* s_red,
                              const uint32_t* __restrict__ g_mcol)
{
  const uint32_t* g_pow = s_table + 4 * 256;
  int      order;
  uint32_t poly;
  crc_params(poly_id, order, poly);
  const uint32_t mask = (order == 32) ? 0xffffffffU : ((1U << order) - 1U);
  const int      nw   = (L + 31) / 32;
  const int      p    = nw * 32 - L;
  uint32_t       acc  = 0;
  for (int w = threadIdx.x; w < nw; w += blockDim.x) {
    /* the multiplier's columns first (global, L2-resident; independent of the message, so their latency overlaps the
     * LDS reads below) */
    const uint4* mc = reinterpret_cast<const uint4*>(g_mcol + (nw - 1 - w) * 24);
    uint4        col[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      col[q] = mc[q];
    }
    /* hb is 4-byte aligned (lay.hard): one LDS dword per word, byte-swapped to MSB-first */
    auto be = [&](int i) -> uint32_t {
      if (i < 0) {
        return 0U;
      }
      return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(hb + 4 * i));
    };
    const uint32_t W   = (p == 0) ? be(w) : ((be(w - 1) << (32 - p)) | (be(w) >> p));
    const uint32_t crc = (s_table[3 * 256 + (W >> 24)] ^ s_table[2 * 256 + ((W >> 16) & 0xffU)] ^
                          s_table[256 + ((W >> 8) & 0xffU)] ^ s_table[W & 0xffU]) & mask;
    /* crc * x^(32 (nw - 1 - w)) mod G: the XOR of the columns of crc's set bits (bits >= order are zero) */
    const uint32_t cw[24] = {col[0].x, col[0].y, col[0].z, col[0].w, col[1].x, col[1].y, col[1].z, col[1].w,
                             col[2].x, col[2].y, col[2].z, col[2].w, col[3].x, col[3].y, col[3].z, col[3].w,
                             col[4].x, col[4].y, col[4].z, col[4].w, col[5].x, col[5].y, col[5].z, col[5].w};
    uint32_t       prod[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      prod[i & 3] ^= cw[i] & (0U - ((crc >> i) & 1U));
    }
    acc ^= (prod[0] ^ prod[1]) ^ (prod[2] ^ prod[3]);
    (void)g_pow;
  }
  acc              = wave_xor(acc);
  const int wave   = threadIdx.x >> 6;
  const int nwaves = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_red[wave] = acc;
  }
  __syncthreads();
  /* lane i reads wave i's word (one LDS read, not a chain of nwaves dependent ones), then a wave XOR */
  const int lane = threadIdx.x & 63;
  return wave_xor(lane < nwaves ? s_red[lane] : 0U);
}

/* hard_decision (log_likelihood_ratio.cpp:226-252) of soft[0, K*Z) into LDS packed bytes.
 * Returns true (block-uniform) iff no soft bit is zero. Eight soft bits per thread come in with one 8-byte LDS read
 * (the soft region extends past K*Z, so the last read stays inside it). The block-wide "any zero" goes through the
 * LDS word *s_flag, which holds the token of the last call that found a zero: token must differ between calls, so
 * the flag never needs a reset (and the kernel's LDS stays all dynamic). ZC: Z when it is a compile-time constant
 * (specialised kernel), else 0. */
/* Per byte of four soft bits: t = (w & 0x7f..) + 0x7f.. has a byte's bit 7 set iff its low seven bits are not all
 * zero, so (w | ~t) & 0x80.. marks s <= 0 (the hard bit) and ~(w | t) & 0x80.. marks s == 0. gather4 packs the four
 * marks (bits 7, 15, 23, 31) into a nibble, soft bit 0 first: (m >> 7) * 0x80402010 puts mark j at bit 31 - j and
 * every cross term at a bit of its own below 28 or above 31 (no carries). */
__device__ __forceinline__ uint32_t gather4(uint32_t m) { return ((m >> 7) * 0x80402010U) >> 28; }

template <int ZC = 0>
__device__ __forceinline__ bool block_hard_decision(const int8_t* soft, uint8_t* hb, int KZ, uint32_t* s_flag,
                                                    uint32_t token, int Z = 0, int stride = 0, int read_off = 0)
{
  const int nb   = (KZ + 7) / 8;
  bool      zero = false;
  const int zc = ZC > 0 ? ZC : Z;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    int pos = 8 * b;
    if (stride != 0) {
      /* column-strided copies (specialised kernel, Z % 8 == 0: the 8 bits of a byte share a column) */
      const int col = pos / zc;
      pos           = col * stride + read_off + (pos - col * zc);
    }
    const uint2    w     = *reinterpret_cast<const uint2*>(soft + pos);
    const uint32_t keep  = 0xff00U >> min(8, KZ - 8 * b); /* valid bits of the last byte */
    const uint32_t tx    = (w.x & 0x7f7f7f7fU) + 0x7f7f7f7fU, ty = (w.y & 0x7f7f7f7fU) + 0x7f7f7f7fU;
    const uint32_t hard  = (gather4((w.x | ~tx) & 0x80808080U) << 4) | gather4((w.y | ~ty) & 0x80808080U);
    const uint32_t zeros = (gather4(~(w.x | tx) & 0x80808080U) << 4) | gather4(~(w.y | ty) & 0x80808080U);
    zero                 = zero || (zeros & keep) != 0;
    hb[b]                = static_cast<uint8_t>(hard & keep);
  }
  if (__builtin_amdgcn_ballot_w64(zero) != 0 && (threadIdx.x & 63) == 0) {
    *reinterpret_cast<volatile uint32_t*>(s_flag) = token;
  }
  __syncthreads();
  return *reinterpret_cast<volatile uint32_t*>(s_flag) != token;
}

/* hard_decision of binary16 soft bits (the specialised decoders with ldpc_spec.h SOFT_BYTES = 2), same contract as
 * block_hard_decision: eight soft bits (16 bytes, one LDS read) per output byte. Per 16-bit half, t = (w & 0x7fff) +
 * 0x7fff has bit 15 set iff the magnitude is non-zero, so (w | ~t) & 0x8000 marks s <= 0 (sign set, or zero: the
 * decoder never forms -0, sp::pass2) and ~t & 0x8000 marks s == 0. gather2 puts a word's first soft bit (bit 15) above
 * its second (bit 31), MSB first. */
__device__ __forceinline__ uint32_t gather2(uint32_t m) { return ((m >> 14) & 2U) | (m >> 31); }
__device__ __forceinline__ bool block_hard_decision16(const int8_t* soft, uint8_t* hb, int KZ, uint32_t* s_flag,
                                                      uint32_t token)
{
  const int nb   = (KZ + 7) / 8;
  bool      zero = false;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const uint4    w       = *reinterpret_cast<const uint4*>(soft + 16 * b);
    const uint32_t keep    = 0xff00U >> min(8, KZ - 8 * b); /* valid bits of the last byte */
    const uint32_t q[4]    = {w.x, w.y, w.z, w.w};
    uint32_t       hard    = 0, zeros = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t t = (q[k] & 0x7fff7fffU) + 0x7fff7fffU;
      hard |= gather2((q[k] | ~t) & 0x80008000U) << (6 - 2 * k);
      zeros |= gather2(~t & 0x80008000U) << (6 - 2 * k);
    }
    zero  = zero || (zeros & keep) != 0;
    hb[b] = static_cast<uint8_t>(hard & keep);
  }
  if (__builtin_amdgcn_ballot_w64(zero) != 0 && (threadIdx.x & 63) == 0) {
    *reinterpret_cast<volatile uint32_t*>(s_flag) = token;
  }
  __syncthreads();
  return *reinterpret_cast<volatile uint32_t*>(s_flag) != token;
}

/* Check-to-variable storage. c2v is kept per edge, as the reference keeps it (ldpc_decoder_impl.h:224-226), but
 * only for the edges that exist: int8 c2v[e][t] for graph edge e and lifted check node t (edge-major, stride Z, so
 * a wave's 64 consecutive check nodes read 64 consecutive bytes). BG1 Z=384: 316 * 384 = 121,344 B. An all-zero c2v
 * is the "not yet initialised" state: soft (-) 0 = soft, the first-iteration copy of
 * update_variable_to_check_messages (impl.cpp:196-200).
 *
 * Soft bits inside the decoder hold [-120, 120] for finite LLRs and +-121 for +-infinity (the reference's +-127,
 * llr.h:238): with infinity one step above the finite range, "promotion_sum overflows to infinity" is a single
 * clamp to +-121 and x = s - clamp(s, +-120) is the infinity indicator (+-1 or 0). Only the sign and the zero test of
 * a soft bit ever leave the decoder (hard_decision), and both are unchanged by the encoding. */

/* scale_llr (ldpc_decoder_generic.cpp:70-79) for a finite magnitude m in [0, 120]: round(float(m) * sf), half away
 * from zero. v_mul_f32 is correctly rounded and llvm.round is exact, so this equals the host std::round. */
template <bool SF08>
__device__ __forceinline__ int scale_mag(int m, float sf)
{
  if (SF08) {
    /* sf = 0.8f (the PHY default, ldpc_decoder.h:50): round(0.8 m) = floor((4m + 2) / 5) = (52432 m + 26216) >> 16
     * for m in [0, 120] (checked exhaustively against the float formula) */
    return static_cast<int>((__umul24(static_cast<uint32_t>(m), 52432U) + 26216U) >> 16);
  }
  return static_cast<int>(__builtin_roundf(static_cast<float>(m) * sf));
}

__device__ __forceinline__ int med3i(int x, int lo, int hi) { return min(max(x, lo), hi); } /* v_med3_i32 */

/* binary16 soft bits of four clamped int8 LLRs (the specialised decoders' LDS, ldpc_spec.h SOFT_BYTES = 2):
 * x = b ^ 0x80 is b + 128 as an unsigned byte, so 0x6580 + x = 0x6600 + b is the binary16 pattern of 1536 + b (the
 * [1024, 2048) binade has unit spacing), and (1536 + b) - 1536 = b exactly, +0 for b = 0. Two v_perm, two v_add and
 * two packed subtractions per four LLRs. */
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 soft_f16x4(uint32_t w)
{
  const uint32_t x  = w ^ 0x80808080U;
  const uint32_t lo = __builtin_amdgcn_perm(0U, x, 0x0c010c00U) + 0x65806580U;
  const uint32_t hi = __builtin_amdgcn_perm(0U, x, 0x0c030c02U) + 0x65806580U;
  const f16x2_t  k  = {static_cast<_Float16>(1536.0F), static_cast<_Float16>(1536.0F)};
  return make_uint2(__builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2_t, lo) - k),
                    __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2_t, hi) - k));
}
__device__ __forceinline__ uint16_t soft_f16(int v) { return __builtin_bit_cast(uint16_t, static_cast<_Float16>(v)); }

/* Four int8 LLRs with +-127 (infinity) mapped to the decoder-internal +-121. */
__device__ __forceinline__ uint32_t clamp_inf4(uint32_t w)
{
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int v = med3i(__builtin_amdgcn_sbfe(static_cast<int>(w), 8 * b, 8), -LLR_INTERNAL_INF, LLR_INTERNAL_INF);
    r |= (static_cast<uint32_t>(v) & 0xffU) << (8 * b);
  }
  return r;
}

#if defined(LDPC_HIP_DIAG) || defined(LDPC_HIP_DIAG_PHASE) || defined(LDPC_HIP_DIAG_TBJ) || defined(LDPC_HIP_DIAG_DM)
} // namespace
/* diagnostic build only: s_memtime stamps of block 0 after every step barrier */
static __device__ uint64_t g_diag[4096];
static __device__ uint64_t g_diag2[64 * 16 * 8]; /* last iteration: per step and wave, (start, end of row work) or phases */
namespace {
#endif
#ifdef LDPC_HIP_DIAG /* specialised kernel: per (step, wave) phase stamps of block 0, overwritten every iteration */
#define SPEC_STAMP(S, k)                                                                                               \
  do {                                                                                                                 \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) {                                                                  \
      g_diag2[((S) * 16 + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime();                               \
    }                                                                                                                  \
  } while (0)
#else
#define SPEC_STAMP(S, k) ((void)0)
#endif
#if defined(LDPC_HIP_DIAG) && defined(LDPC_HIP_DIAG_FULL) /* phase stamps inside a step: perturb the schedule */
#define SPEC_STAMP_FULL(S, k) SPEC_STAMP(S, k)
#else
#define SPEC_STAMP_FULL(S, k) ((void)0)
#endif
#ifdef LDPC_HIP_DIAG_PHASE /* diagnostic build: s_memtime at phase boundaries of the row update */
#define PHASE(i) (ph[(i)] = __builtin_amdgcn_s_memtime())
#else
#define PHASE(i) ((void)0)
#endif

/* Partner lane (lane ^ 32) value through v_permlane32_swap. */
__device__ __forceinline__ uint32_t partner32(uint32_t v, int half)
{
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return half ? r[0] : r[1];
}

/* LDS byte at an absolute LDS address. The decode kernel has no static LDS, so its dynamic LDS (smem) starts at LDS
 * address 0 and the soft bits (lay.soft == 0) are addressed by column offset alone -- checked once per launch. */
typedef __attribute__((address_space(3))) int8_t lds_i8;
__device__ __forceinline__ lds_i8* lds_byte(uint32_t addr) { return (lds_i8*)(uintptr_t)addr; }
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ lds_u32* lds_word(uint32_t addr) { return (lds_u32*)(uintptr_t)addr; }

/* ---- per-edge and per-row arithmetic shared by the generic and the specialised row updates (see row_update) ---- */

/* v2c = soft (-) c2v with the infinity push: med3(s - c, +-120) + 512 x, x = s - med3(s, +-120). */
__device__ __forceinline__ int v2c_of(int s, int c)
{
  const int x = s - med3i(s, -LLR_MAX, LLR_MAX); /* infinity indicator: +-1 or 0 */
  return (x << 9) + med3i(s - c, -LLR_MAX, LLR_MAX); /* v_lshl_add_u32 */
}

/* Two-minimum scan step: m2 = min(m2, max(m1, a)) as one v_med3_u32 (the compiler otherwise emits max + min). */
__device__ __forceinline__ void scan_edge(uint32_t& m1, uint32_t& m2, int a)
{
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(m2) : "v"(m1), "v"(a), "v"(m2));
  m1 = min(m1, static_cast<uint32_t>(a));
}

/* End of pass 1: merge a split row's halves (P = 2), then the two scaled magnitudes with the parity sign folded in:
 * p1 for edges with |v2c| != min, p2 for |v2c| == min (see row_update). m1 is returned merged. */
template <int P, bool SF08>
__device__ __forceinline__ void row_scale(uint32_t& m1, uint32_t m2, uint32_t sx, int half, float sf, int& p1, int& p2)
{
  if (P == 2) {
    const uint32_t oth = partner32(m1 | (m2 << 8), half);
    const uint32_t o1 = oth & 0xffU, o2 = oth >> 8;
    m2                = min(min(m2, o2), max(m1, o1));
    m1                = min(m1, o1);
    sx ^= partner32(sx, half);
  }
  const int n1  = scale_mag<SF08>(static_cast<int>(m1), sf);
  const int n2  = scale_mag<SF08>(static_cast<int>(m2), sf);
  const int neg = static_cast<int>(sx) >> 31;
  p1            = (n1 ^ neg) - neg;
  p2            = (n2 ^ neg) - neg;
  /* opaque to the optimiser: otherwise it sinks the scaling into every edge as select + rescale */
  asm volatile("" : "+v"(p1), "+v"(p2));
}

/* Sign mask (0 / -1) and magnitude of v2c. The mask stays opaque, so the magnitude is v_xor + v_sub (not the abs
 * idiom's v_sub + v_max) and pass 2 reuses the mask instead of shifting again. */
__device__ __forceinline__ int sign_mask(int v)
{
  int sv = v >> 31;
  asm("" : "+v"(sv));
  return sv;
}

/* c2v' of an edge with v2c sign mask sv and |v2c| a. */
__device__ __forceinline__ int c2v_new(int sv, int a, uint32_t m1, int p1, int p2)
{
  const int ms = (a == static_cast<int>(m1)) ? p2 : p1;
  return (ms ^ sv) - sv;
}

/* soft' = promotion_sum(c2v', v2c). */
__device__ __forceinline__ int soft_new(int c, int v) { return med3i(c + v, -LLR_INTERNAL_INF, LLR_INTERNAL_INF); }

/* One lifted check node t of a row of degree D -- update_variable_to_check_messages,
 * update_check_to_variable_messages and update_soft_bits (ldpc_decoder_impl.cpp:176-308) restricted to Z-lane t,
 * with the generic kernels' arithmetic (ldpc_decoder_generic.cpp:30-120).
 *
 * P = 1: one lane owns the check node and scans all D edges in order.
 * P = 2: lanes l and l ^ 32 share the check node; the lower half scans edges [0, D0), the upper half [D0, D), and
 *        the partial (min1, min2, sign parity) are merged across the pair: min1 = min(A, B), min2 = min(min2_A,
 *        min2_B, max(min1_A, min1_B)) -- the two smallest of the multiset, as the sequential scan finds them.
 * Edge words (shift | col * Z << 16) come from the LDS edge table; the upper half's slot starts at edge D0.
 *
 * LLR special cases with the internal encoding above (c2v is never infinite: |c2v| <= round(120 sf) <= 120):
 *   v2c   = isinf(s) ? s : clamp(s - c2v, +-120)           (llr.cpp:56-71 operator-)
 *           computed as clamp(s - c2v, +-120) + 512 x: an infinite v2c keeps its sign and a magnitude above 512,
 *           which the two-minimum scan treats exactly like the reference's +-127 (min and min2 start at 120 and
 *           only a magnitude strictly below them is taken; |v2c| == min never holds for it);
 *   soft' = promotion_sum(c2v', v2c) = clamp(c2v' + v2c, +-121)   (llr.cpp:73-86): a finite sum saturates to
 *           infinity past +-120, and an infinite v2c (|v2c| > 512 > 121 + |c2v'|) stays infinite. */
template <int D, int P, bool SF08>
__device__ __forceinline__ void row_update(int t, int half, const uint32_t* s_slot, int8_t* s_soft,
                                           int8_t* s_c2v_row, float sf, int Z, int trash, uint64_t* ph)
{
  PHASE(0);
  constexpr int DP = (P == 1) ? D : (D + 1) / 2; /* edges scanned by this lane */
  constexpr int D0 = DP;                         /* first edge of the upper half (P = 2) */
  const int     kb = (P == 2 && half) ? D0 : 0;
  int8_t*       cq = s_c2v_row + t + kb * Z;     /* this lane's c2v of local edge kk: cq + kk * Z */

  lds_i8* sp[DP]; /* soft bit of edge kk at the cyclic shift */
  int8_t* cp[DP]; /* c2v of edge kk */
  int     vc[DP]; /* v2c */
#pragma unroll
  for (int kk = 0; kk < DP; ++kk) {
    /* edge word shift | col * Z << 16 (wave-uniform, step_task); with splitting the two halves select per lane */
    const bool dummy = (P == 2 && D0 + kk >= D && half); /* upper half of an odd-degree row has one edge less */
    const uint32_t ew   = s_slot[kk];   /* this lane's edge (the upper half's slot starts at edge D0) */
    const uint32_t sh   = ew & 0xffffU;
    const uint32_t colz = ew >> 16;
    const uint32_t j0   = static_cast<uint32_t>(t) + sh;
    const uint32_t j    = min(j0, j0 - static_cast<uint32_t>(Z)); /* (t + shift) mod Z */
    sp[kk]              = lds_byte(colz + j); /* a dummy edge points at the scratch bytes */
    cp[kk]              = dummy ? s_soft + trash : cq;
    cq += Z; /* incremental: keeps the c2v addresses single VOP2 adds */
  }
  PHASE(1);
  int      av[DP];                     /* |v2c| */
  int      sg[DP];                     /* sign mask of v2c */
  uint32_t m1 = LLR_MAX, m2 = LLR_MAX; /* the reference's min and min2 (gen.cpp:46-68) */
  uint32_t sx = 0;                     /* sign parity of all v2c (bit 31) */
#pragma unroll
  for (int kk = 0; kk < DP; ++kk) {
    const bool dummy = (P == 2 && D0 + kk >= D && half);
    const int  v     = v2c_of(*sp[kk], *cp[kk]);
    vc[kk]           = v;
    const int sv     = sign_mask(v);
    sg[kk]           = sv;
    const int a      = dummy ? 0xfff : (v ^ sv) - sv;
    av[kk]           = a;
    scan_edge(m1, m2, a);
    sx ^= dummy ? 0U : static_cast<uint32_t>(v);
  }
  PHASE(2);
  /* c2v' of edge k = sign(v2c_k) * sign(parity) * (k == idx ? n2 : n1) (gen.cpp:93-105). The reference's idx is
   * the first edge with |v2c| == min; any other edge with |v2c| == min makes min2 == min, so "k == idx" can be
   * replaced by "|v2c_k| == min" without changing a single output, and no edge index is tracked. The parity's sign
   * is folded into the two magnitudes once per row. */
  int p1, p2;
  row_scale<P, SF08>(m1, m2, sx, half, sf, p1, p2);
  PHASE(3);
#pragma unroll
  for (int kk = 0; kk < DP; ++kk) {
    const int c = c2v_new(sg[kk], av[kk], m1, p1, p2);
    *cp[kk]     = static_cast<int8_t>(c);
    *sp[kk]     = static_cast<int8_t>(soft_new(c, vc[kk]));
  }
  PHASE(4);
}

/* Dispatch on the (wave-uniform) row degree. BG1 degrees: 3..10, 19; BG2: 3..10 (ldpc_luts_impl.cpp:4383-4519). */
template <int P, bool SF08>
__device__ __forceinline__ void row_dispatch(int deg, int t, int half, const uint32_t* s_slot, int8_t* s_soft,
                                             int8_t* c2v_row, float sf, int Z, int trash, uint64_t* ph)
{
  switch (deg) {
    case 3: row_update<3, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
    case 4: row_update<4, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
    case 5: row_update<5, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
    case 6: row_update<6, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
    case 7: row_update<7, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
    case 8: row_update<8, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
    case 9: row_update<9, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
    case 10: row_update<10, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
    default: row_update<19, P, SF08>(t, half, s_slot, s_soft, c2v_row, sf, Z, trash, ph); break;
  }
}

/* ---- specialised decoder: the whole iteration unrolled at compile time (ldpc_spec.h) ---------------------------
 * The step sequence and every row's degree, columns and shifts are constants, so a row needs no table reads, no
 * degree dispatch and no task fetch: its soft addresses are three VALU ops per edge (t + shift wrapped modulo Z), the
 * column offset being the LDS instruction's immediate. Split rows (P = 2) select the upper half's column and shift
 * per lane with a mask.
 *
 * Check-to-variable messages live in VGPRs, two edges per register (16-bit halves). A lane updates the same (row,
 * check node, edge pairs) in every iteration, so its c2v words never leave it: pair slot q of a row is register q of
 * the lane (srole::q0; the two wave groups' rows take slots independently, BG1 Z=384: 87 registers).
 *
 * A step's work sits inside its wave group's branch (addresses, soft reads, update, writes). Only the early part of a
 * pipelined single-row chain (ldpc_spec.h) crosses a barrier: its registers go through a fresh, undefined carry on
 * every other path, so no path keeps copies of them. */
namespace sp {

using spec::MAX_POS;

template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>)
{
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f)
{
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

/* t, hmask and the address bases pass through opaque asm once per step: every address derived from them is
 * iteration-invariant, and without this the compiler hoists all of them out of the iteration loop (hundreds of live
 * registers, spilled). */
__device__ __forceinline__ uint32_t opaque(uint32_t x)
{
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ uint32_t opaque_s(uint32_t x)
{
  asm volatile("" : "+s"(x));
  return x;
}

/* Two 16-bit lanes per register (v_pk_* instructions: one issue for two edges of a check node). */
typedef short          s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 as_s(uint32_t x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ u16x2 as_u(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t bits(s16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t bits(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ s16x2 splat(int v) { return s16x2{static_cast<short>(v), static_cast<short>(v)}; }
__device__ __forceinline__ u16x2 splatu(unsigned v)
{
  return u16x2{static_cast<unsigned short>(v), static_cast<unsigned short>(v)};
}

/* lane constants of the iteration */
struct lanes {
  uint32_t t1[2];   /* P = 1, wave group g: t = 64 * (wave - g W) + lane, and t + HI */
  uint32_t t1h[2];
  uint32_t t2, t2h; /* P = 2: t = 32 * wave + (lane & 31), and t + HI         */
  uint32_t hmask;   /* P = 2: 0 for lanes 0-31, ~0 for lanes 32-63           */
  int      wave, lane, nof_layers;
  uint32_t one2;    /* SGPR constants (VOP2 with an SGPR source, not a 32-bit literal): int8 0x00010001 (pass1's
                       v_or), binary16 the sign mask 0x80008000 */
  uint32_t onef;    /* binary16: 1.0 in both halves (pass2) */
  uint32_t sa[20];  /* split rows (P = 2, BG1 rows 0-3): the full LDS address of each position, two per word
                       (16 bits each), computed once per decode (dec::fill_split) */
  uint32_t abase;   /* LDS byte address of this lane's first word of the split-address table (lay.c2v + 4 tid) */
  uint32_t act[3];  /* wave-uniform role masks (SGPRs): bit S of act[0] / act[1] / act[2] set when this wave runs the
                       step's first role / second role / the next row's early part (dec::role_masks) */
};

/* Soft bits (spec::SOFT_COPIES). One copy: column c at c * Z; edge k of check node t reads and writes
 * c * Z + (t + shift) mod Z, the modulo as min(t + shift, t + shift - Z) in unsigned arithmetic. Four copies: column c
 * at c * 4Z + {0, Z, 2Z, 3Z}; edge k reads p + Z with p = c * 4Z + t + shift (t + shift < 2Z, so p + Z is inside the
 * copies at Z and 2Z, no modulo) and writes p, p + Z and p + 2Z, which covers both read copies of index
 * (t + shift) mod Z whether or not t + shift wrapped. */
__device__ __forceinline__ int rd8(uint32_t base, uint32_t imm) { return *(lds_byte(base) + imm); }
__device__ __forceinline__ void wr8(uint32_t base, uint32_t imm, uint32_t v)
{
  *(lds_byte(base) + imm) = static_cast<int8_t>(v);
}
/* A soft bit of the specialised decoders (spec::SOFT_BYTES): int8 (ds_read_i8 / ds_write_b8) or binary16
 * (ds_read_u16 / ds_write_b16, its 16 bits in the low half); base + imm is a byte address. */
typedef __attribute__((address_space(3))) uint16_t lds_u16;
constexpr int SB = spec::SOFT_BYTES;
__device__ __forceinline__ int rds(uint32_t base, uint32_t imm)
{
  if constexpr (SB == 2) {
    return *reinterpret_cast<lds_u16*>(lds_byte(base) + imm);
  } else {
    return rd8(base, imm);
  }
}
__device__ __forceinline__ void wrs(uint32_t base, uint32_t imm, uint32_t v)
{
  if constexpr (SB == 2) {
    *reinterpret_cast<lds_u16*>(lds_byte(base) + imm) = static_cast<uint16_t>(v);
  } else {
    wr8(base, imm, v);
  }
}
/* +infinity (the dummy position of an odd row, the scratch column): 121, or 121.0 in binary16 */
constexpr int SOFT_INF = SB == 2 ? 0x5790 : 121;
/* the two-minimum scan's start: 120 (strict <: infinity and +-120 never change it) */
constexpr unsigned MIN_START = SB == 2 ? 0x5780U : 120U;

#if LDPC_SPEC_F16
/* binary16 pairs. Every value is an integer of magnitude <= 337 (exact). min / max run on the bit patterns as 16-bit
 * integers: unsigned for magnitudes (non-negative), signed where one side may be negative (a negative binary16 is a
 * negative int16, and among non-negative values the integer order is the numeric one), so no float min/max (which
 * would canonicalise their inputs first). Constants: 120.0 = 0x5780, 121.0 = 0x5790, 1.0 = 0x3c00. */
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h16x2 as_h(uint32_t x) { return __builtin_bit_cast(h16x2, x); }
__device__ __forceinline__ uint32_t bits(h16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ h16x2 splath(float v) { return h16x2{static_cast<_Float16>(v), static_cast<_Float16>(v)}; }

/* Pass 1 of an edge pair (binary16): d = s - c, its sign bits g (v_and), |d| (v_and), a = |v2c| with +infinity
 * marked by s^2 - 14400 = 241 (fma; <= 0 for a finite s), the per-half two-minimum and the sign parity (v_xor). */
__device__ __forceinline__ void pass1(uint32_t S, uint32_t C, u16x2& M1, u16x2& M2, uint32_t& SX, uint32_t& G,
                                      uint32_t& A, uint32_t smask)
{
  /* smask = 0x80008000 in an SGPR (VOP2 v_and with an SGPR source: no 32-bit literal, 2.1 cycles against 2.6) */
  const h16x2    s  = as_h(S);
  const uint32_t d  = bits(s - as_h(C));
  uint32_t       g  = d & smask;
  /* opaque: otherwise gfx950's v_bitop3_b32 (a half-rate VOP3) fuses g into |d| and into the parity XOR */
  asm("" : "+v"(g));
  const u16x2    af = __builtin_elementwise_min(as_u(d ^ g), splatu(0x5780U)); /* |d|: d without its sign bits */
  const uint32_t iv = bits(__builtin_elementwise_fma(s, s, splath(-14400.0F)));
  const u16x2    a  = as_u(bits(__builtin_elementwise_max(as_s(bits(af)), as_s(iv))));
  M2                = __builtin_elementwise_min(M2, __builtin_elementwise_max(M1, a));
  M1                = __builtin_elementwise_min(M1, a);
  SX ^= g;
  G = g;
  A = bits(a);
}

/* Pass 2 (binary16), with the row's constants from row_consts: N1 = n1, CC = n2 + m1 and PP = the parity's sign
 * bit in both halves. f = max(n1, n2 + m1 - a) (see the int8 note below), P f by a sign flip (v_xor), soft' = sign(v2c)
 * min(a + P f, 121) as fma(u, +-1.0, +0) -- a plain product or sign flip would give -0 for u = 0, and a -0 soft bit
 * would count as negative in the next parity --, c2v' = sign(v2c) P f (v_xor). */
__device__ __forceinline__ void pass2(uint32_t G, uint32_t A, s16x2 N1, s16x2 CC, s16x2 PP, uint32_t& Cnew,
                                      uint32_t& Snew, uint32_t onef)
{
  /* onef = 1.0 in both halves (0x3c003c00) in an SGPR */
  const h16x2    a  = as_h(A);
  const s16x2    f  = __builtin_elementwise_max(N1, as_s(bits(as_h(bits(CC)) - a)));
  const uint32_t pf = bits(f) ^ bits(PP);
  const s16x2    u  = __builtin_elementwise_min(as_s(bits(a + as_h(pf))), splat(0x5790));
  Snew              = bits(__builtin_elementwise_fma(as_h(bits(u)), as_h(G | onef), splath(0.0F)));
  Cnew              = pf ^ G;
}

/* The row's pass-2 constants from its two minima (binary16 bit patterns) and parity word: round(0.8 m) =
 * fma(m, 0.8, 1024) - 1024 (one rounding to the integer grid of [1024, 2048); 0.8 in binary16 is 0.7998, off by
 * < 0.024 for m <= 120, while 0.8 m is never within 0.1 of a half: exact), both minima in one packed fma. */
__device__ __forceinline__ void row_consts(uint32_t m1, uint32_t m2, uint32_t sx, s16x2& N1, s16x2& CC, s16x2& PP)
{
  const h16x2 nn = __builtin_elementwise_fma(as_h(m1 | (m2 << 16)), splath(0.7998046875F), splath(1024.0F)) -
                   splath(1024.0F);
  const s16x2 t  = as_s(bits(nn + as_h(m1 << 16))); /* (n1, n2 + m1) */
  /* swizzled splats: the packed consumers read them through op_sel, no splat instruction */
  N1 = t.xx;
  CC = t.yy;
  PP = splat(static_cast<short>(sx & 0x8000U));
}
#else
/* Pass 1 of an edge pair: v2c = soft (-) c2v per half, its magnitude a (+infinity -> 241) and the per-half
 * two-minimum and parity updates. Arithmetic note at pass2. */
__device__ __forceinline__ void pass1(uint32_t S, uint32_t C, u16x2& M1, u16x2& M2, uint32_t& SX, uint32_t& G,
                                      uint32_t& A, uint32_t one2)
{
  const s16x2 s  = as_s(S);
  const s16x2 d  = s - as_s(C);                               /* s - c                          */
  uint32_t    gb = bits(d >> 15) | one2; /* sign of v2c, +-1 (pass 2 uses it) */
  asm("" : "+v"(gb)); /* keeps |d| = d g: the compiler would rewrite it as max(d, -d), one instruction more */
  const s16x2 g  = as_s(gb);
  const s16x2 af = __builtin_elementwise_min(d * g, splat(120)); /* |clamp(s - c)|  */
  const s16x2 iv = s * s - splat(14400);                      /* 241 iff |s| = 121              */
  const u16x2 a  = as_u(bits(__builtin_elementwise_max(af, iv)));
  M2             = __builtin_elementwise_min(M2, __builtin_elementwise_max(M1, a));
  M1             = __builtin_elementwise_min(M1, a);
  SX ^= bits(g);
  G = bits(g);
  A = bits(a);
}

/* Pass 2 of an edge pair.
 * Arithmetic (int8 LLRs, llr.cpp:39-97; ldpc_decoder_generic.cpp:30-120), with the decoder-internal soft encoding of
 * +-121 for the reference's +-infinity (+-127):
 *   v2c   = isinf(s) ? s : clamp(s - c, +-120): its sign g is the sign of d = s - c in every case (|c| <= 96 < 121),
 *           and a = |v2c| = min(d g, 120) for a finite s, 241 for an infinite one (s^2 - 14400 > 0 only at |s| = 121);
 *           in the two-minimum scan (start 120, strict <) 241 behaves exactly like the reference's 127;
 *   the reference gives min2 to the first edge with |v2c| == min1 and min1 to the others; any other edge with
 *           |v2c| == min1 implies min2 == min1. With n = round(0.8 m) and every a >= m1 (a >= m2 unless a == m1):
 *           f = (a == m1) ? n2 : n1 = max(n1, n2 + m1 - a): for a >= m2 > m1, n2 - n1 <= floor(0.8 (m2 - m1) + 1)
 *           <= m2 - m1 <= a - m1;
 *   c2v'  = sign(v2c) * P * f   (P = +-1, the check node's sign parity);
 *   soft' = promotion_sum(c2v', v2c) = sign(v2c) * min(a + P f, 121): a + P f >= -96, and an infinite v2c (a = 241)
 *           stays at 121. */
__device__ __forceinline__ void pass2(uint32_t G, uint32_t A, s16x2 N1, s16x2 CC, s16x2 PP, uint32_t& Cnew,
                                      uint32_t& Snew, uint32_t onef)
{
  (void)onef;
  const s16x2 a  = as_s(A);
  const s16x2 g  = as_s(G);
  const s16x2 f  = __builtin_elementwise_max(N1, CC - a);
  const s16x2 pf = f * PP;
  const s16x2 u  = __builtin_elementwise_min(a + pf, splat(121));
  Snew           = bits(u * g);
  Cnew           = bits(pf * g);
}

/* the row's pass-2 constants: n = round(0.8 m) = (52432 m + 26216) >> 16 exactly for m in [0, 120] (gen.cpp:70-79
 * with sf = 0.8f), CC = n2 + m1, PP = the check node's sign, +-1 */
__device__ __forceinline__ void row_consts(uint32_t m1, uint32_t m2, uint32_t sx, s16x2& N1, s16x2& CC, s16x2& PP)
{
  const uint32_t n1 = (__umul24(m1, 52432U) + 26216U) >> 16;
  const uint32_t n2 = (__umul24(m2, 52432U) + 26216U) >> 16;
  N1                = splat(static_cast<int>(n1));
  CC                = splat(static_cast<int>(n2 + m1));
  PP                = splat(static_cast<short>(sx | 1U));
}
#endif

/* The check node's two minima and parity from the per-half ones: min1 = min(A, B), min2 = min(min2_A, min2_B,
 * max(min1_A, min1_B)) -- the two smallest of the multiset, as the sequential scan finds them. Parity: each half of SX
 * is the XOR of +-1 values (0x0001 / 0xffff), so bits 1-15 of lo ^ hi all equal the parity of the negative signs and
 * (lo ^ hi) | 1 is the check node's sign, +-1, in the low 16 bits (one shift, XOR and OR per row; the bit-31 form
 * took a shift more). */
__device__ __forceinline__ void fold_halves(u16x2 M1, u16x2 M2, uint32_t SX, uint32_t& m1, uint32_t& m2, uint32_t& sx)
{
  m1 = __builtin_elementwise_min(M1.x, M1.y);
  m2 = __builtin_elementwise_min(__builtin_elementwise_min(M2.x, M2.y), __builtin_elementwise_max(M1.x, M1.y));
  sx = SX ^ (SX >> 16);
}

/* Merge of a split row's halves (lanes l and l ^ 32) through v_permlane32_swap: after the swap each lane holds its
 * own and its partner's values, so the merge is symmetric and needs no select. */
__device__ __forceinline__ void merge_partner(uint32_t& m1, uint32_t& m2, uint32_t& sx)
{
  const uint32_t pk = m1 | (m2 << 16);
  const auto     r  = __builtin_amdgcn_permlane32_swap(pk, pk, false, false);
  const auto     rs = __builtin_amdgcn_permlane32_swap(sx, sx, false, false);
  fold_halves(u16x2{static_cast<unsigned short>(r[0]), static_cast<unsigned short>(r[1])},
              u16x2{static_cast<unsigned short>(r[0] >> 16), static_cast<unsigned short>(r[1] >> 16)}, 0U, m1, m2, sx);
  sx = rs[0] ^ rs[1];
}

template <const spec::sgraph& G>
struct dec {
  static constexpr int      Z       = G.Z;
  static constexpr bool     C1      = spec::SOFT_COPIES == 1; /* one copy: the lane wraps t + shift itself */
  static constexpr uint32_t ZB      = static_cast<uint32_t>(SB) * G.Z; /* bytes per Z soft bits */
  static constexpr uint32_t Z4      = static_cast<uint32_t>(spec::SOFT_COPIES) * ZB; /* column stride (bytes) */
  static constexpr int      NCR     = G.slots;
  static constexpr int      KC      = G.K + 4;                              /* first extension column */
  static constexpr uint32_t SCRATCH = static_cast<uint32_t>(G.N_full) * Z4; /* dummy edges: soft +infinity */
  static constexpr uint32_t HI      = 49152U; /* second address base: every ds immediate fits 16 bits */
  static constexpr int      P2_WAVES = (Z + 31) / 32;
  static_assert(G.valid && 2 * G.W <= 12 && P2_WAVES <= 12, "specialised schedule");

  using cr_t = uint32_t[NCR];

  /* byte offset of edge e of row r in its column's copy at offset 0 (col * 4Z + shift); a dummy edge (e < 0) uses the
   * scratch column */
  static constexpr uint32_t off(int r, int e)
  {
    return e < 0 ? SCRATCH : static_cast<uint32_t>(G.rows[r].col[e]) * Z4 + (C1 ? 0U : shift(r, e));
  }
  static constexpr uint32_t shift(int r, int e) { return e < 0 ? 0U : static_cast<uint32_t>(G.rows[r].sh[e]); }
  static constexpr uint32_t shb(int r, int e) { return static_cast<uint32_t>(SB) * shift(r, e); } /* in bytes */
  /* read/write offset of the copy the decoder uses, relative to off() */
  static constexpr uint32_t RD = C1 ? 0U : static_cast<uint32_t>(G.Z);
  /* extension edge: a degree-1 column (>= K + 4) with shift 0, read and written by this row only -> one copy */
  static constexpr bool     ext(int r, int e) { return e >= 0 && G.rows[r].col[e] >= KC && G.rows[r].sh[e] == 0; }
  static constexpr bool     hi_base(uint32_t o) { return !C1 && o + 3U * Z > 65535U; }
  static_assert(!C1 || SCRATCH + ZB <= 65535U, "one-copy layout: column offsets are ds immediates");


  /* one copy: (t + sh) mod Z = min(t + sh, t + sh - Z) as unsigned (t < Z, sh < Z) */
#if defined(LDPC_SPEC_WRAP32)
  static __device__ __forceinline__ uint32_t wrap(uint32_t x) { return __builtin_elementwise_min(x, x - ZB); }
#else
  /* v_min_u32 is a half-rate instruction; the 16-bit VOP2 v_min_u16 issues at full rate and zeroes the upper half of
   * its result (tools/ubench/README.md), and x, x - Z mod 2^16 order the same way as in 32 bits (x < 2Z <= 2^16) */
  static __device__ __forceinline__ uint32_t wrap(uint32_t x)
  {
    uint32_t r;
    asm("v_min_u16_e32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(x - ZB));
    return r;
  }
#endif
  static constexpr uint32_t imm(uint32_t o) { return hi_base(o) ? o - HI : o; }

  template <int P, int GRP>
  static __device__ __forceinline__ bool lane_active(const lanes& L)
  {
    if constexpr (Z % 64 == 0) {
      return true;
    } else if constexpr (P == 2) {
      return L.t2 < ZB;
    } else {
      return L.t1[GRP] < ZB;
    }
  }

  /* address base and immediate of position j of a role */
  template <const spec::srole& RO, int J>
  static __device__ __forceinline__ uint32_t pos_base(const lanes& L)
  {
    if constexpr (C1) {
      constexpr int e0 = J < RO.npos ? RO.e0[J] : -1;
      if constexpr (RO.p == 1) {
        constexpr uint32_t sh = shb(RO.row, e0);
        return sh == 0 ? L.t1[RO.grp] : wrap(L.t1[RO.grp] + sh);
      } else {
        constexpr int      e1  = J < RO.npos ? RO.e1[J] : -1;
        constexpr uint32_t sh0 = shb(RO.row, e0), sh1 = shb(RO.row, e1);
        uint32_t           x   = L.t2;
        if constexpr (sh0 != 0 || sh1 != 0) {
          x = wrap(x + sh0 + (sh1 != sh0 ? (L.hmask & (sh1 - sh0)) : 0U));
        }
        constexpr uint32_t o0 = off(RO.row, e0), o1 = off(RO.row, e1);
        return o1 == o0 ? x : x + (L.hmask & (o1 - o0)); /* upper half: its own column */
      }
    } else if constexpr (RO.p == 1) {
      constexpr uint32_t o = off(RO.row, J < RO.npos ? RO.e0[J] : -1);
      return hi_base(o) ? L.t1h[RO.grp] : L.t1[RO.grp];
    } else {
      constexpr uint32_t o0 = off(RO.row, J < RO.npos ? RO.e0[J] : -1);
      constexpr uint32_t o1 = off(RO.row, J < RO.npos ? RO.e1[J] : -1);
      return (hi_base(o0) ? L.t2h : L.t2) + (L.hmask & (o1 - o0)); /* upper half: its own edge's offset */
    }
  }
  template <const spec::srole& RO, int J>
  static constexpr uint32_t pos_imm()
  {
    return imm(off(RO.row, J < RO.npos ? RO.e0[J] : -1));
  }
  template <const spec::srole& RO, int J>
  static constexpr bool pos_ext()
  {
    return RO.p == 1 && J < RO.npos && ext(RO.row, RO.e0[J]);
  }

  /* A row's pass-1 state kept in registers across the step barrier (pipelined single-row chains, ldpc_spec.h):
   * addresses, signs and v2c magnitudes of the early pairs, and the partial minima and parity. */
  struct carry {
    uint32_t base[MAX_POS];
    uint32_t gs[MAX_POS / 2], a[MAX_POS / 2];
    u16x2    m1, m2;
    uint32_t sx;
  };

  /* Split rows (P = 2): the upper half's column and shift differ from the lower half's at every position, so an
   * address costs 6-7 VALU ops (per-half deltas, wrap, column) against 3 on an unsplit row. BG1's four split rows have
   * 40 positions per lane whose addresses never change during a decode: they can be computed once (fill_split) and
   * kept as 16-bit halves of registers (every LDS address is below 64 KiB), a position then costing one unpack op. */
#ifndef LDPC_SPEC_SPLIT_ADDR
#define LDPC_SPEC_SPLIT_ADDR 1
#endif
/* Round 2 kept rows 0-1's pairs in 20 registers (the Z=384 kernel was at 168 VGPRs with 8 B/lane of spills; rows 0-1
 * against none: 149.1 -> 147.8 us, profiles/r02/split_addr.txt). Round 3 moved all four rows' pairs to the LDS table
 * below (152 VGPRs, no spill), which is what lets the kernel carry a second iteration loop (iteration_partial) without
 * spilling; the table words are read a step ahead (load_pf), so C2 is unchanged within 0.5%
 * (profiles/r03/partial_ab.txt). */
/* Split rows [LDPC_SPEC_SPLIT_ADDR_ROWS, LDPC_SPEC_SPLIT_LDS_ROWS) keep their precomputed address pairs in LDS instead
 * (one 32-bit word per pair and lane, lane-contiguous: one conflict-free ds_read_b32 and two full-rate unpack ops per
 * pair, against 6-7 VALU ops per position computed in the step, and no registers held across the iteration). The
 * table sits in the specialised layout's c2v region (lay.c2v, unused there: c2v lives in registers); make_lds_layout
 * reserves it (spec::SPLIT_LDS_PAIRS). Each lane writes and reads only its own words, so it needs no barrier. Only BG1
 * graphs have the tables (write_split_tables); split rows of BG2 graphs compute their addresses in the step. */
  static constexpr uint32_t WG = static_cast<uint32_t>(G.waves) * 64U; /* table stride: lanes per workgroup */
  template <bool LDS>
  static constexpr int split_pairs_before_t(int S)
  {
    int n = 0;
    for (int s = 0; s < S; ++s) {
      const spec::srole& r  = G.steps[s].r[0];
      const bool         in = LDS ? (r.row >= LDPC_SPEC_SPLIT_ADDR_ROWS && r.row < LDPC_SPEC_SPLIT_LDS_ROWS)
                                  : r.row < LDPC_SPEC_SPLIT_ADDR_ROWS;
      n += (G.bg == 1 && r.p == 2 && in) ? (r.npos + 1) / 2 : 0;
    }
    return n;
  }
  static constexpr int split_pairs_before(int S) { return split_pairs_before_t<false>(S); }
  static constexpr int lds_pairs_before(int S) { return split_pairs_before_t<true>(S); }
  static_assert(split_pairs_before(G.n_steps) <= 20, "lanes::sa holds the split rows' address pairs");
  static_assert(lds_pairs_before(G.n_steps) <= spec::SPLIT_LDS_PAIRS, "make_lds_layout reserves the table");
  static_assert(static_cast<uint32_t>(spec::SPLIT_LDS_PAIRS) * WG * 4U <= 65536U, "table offsets are ds immediates");
  template <const spec::srole& RO>
  static constexpr bool pre_addr()
  {
    return LDPC_SPEC_SPLIT_ADDR && C1 && G.bg == 1 && RO.p == 2 && RO.row < LDPC_SPEC_SPLIT_ADDR_ROWS;
  }
  template <const spec::srole& RO>
  static constexpr bool pre_lds()
  {
    return LDPC_SPEC_SPLIT_ADDR && C1 && G.bg == 1 && RO.p == 2 && RO.row >= LDPC_SPEC_SPLIT_ADDR_ROWS &&
           RO.row < LDPC_SPEC_SPLIT_LDS_ROWS;
  }
  static_assert(lds_pairs_before(G.n_steps) * static_cast<int>(WG) <= SPLIT_TAB_STRIDE, "global split-table stride");
  static constexpr int LDS_PAIRS = lds_pairs_before(G.n_steps);
  template <int S>
  static __device__ __forceinline__ void fill_split_step(lanes& L, uint32_t* __restrict__ gdst)
  {
    static constexpr spec::srole ro = G.steps[S].r[0];
    if constexpr (pre_addr<ro>() || pre_lds<ro>()) {
      constexpr int K0 = pre_addr<ro>() ? split_pairs_before(S) : lds_pairs_before(S);
      static_for<(ro.npos + 1) / 2>([&](auto ic) __attribute__((always_inline)) {
        constexpr int  i  = decltype(ic)::value;
        const uint32_t lo = pos_base<ro, 2 * i>(L) + pos_imm<ro, 2 * i>();
        const uint32_t hi = (2 * i + 1 < ro.npos) ? pos_base<ro, 2 * i + 1>(L) + pos_imm<ro, 2 * i + 1>() : 0U;
        const uint32_t w  = (lo & 0xffffU) | (hi << 16);
        if constexpr (pre_addr<ro>()) {
          L.sa[K0 + i] = w;
        } else if (L.wave < P2_WAVES) {
          if (gdst != nullptr) { /* the context's global copy (write_split_table) */
            gdst[static_cast<uint32_t>(K0 + i) * WG + static_cast<uint32_t>(L.wave * 64 + L.lane)] = w;
          } else {
            *lds_word(L.abase + static_cast<uint32_t>(K0 + i) * WG * 4U) = w;
          }
        }
      });
    }
  }
  template <int... Ss>
  static __device__ __forceinline__ void fill_split(lanes& L, std::integer_sequence<int, Ss...>, uint32_t* gdst = nullptr)
  {
    (fill_split_step<Ss>(L, gdst), ...);
  }

  /* The LDS-table words of a split step's address pairs, read one step ahead (at the start of the previous step,
   * whose barrier then covers their latency; step 0's at the end of the previous iteration or before the loop). */
  using pf_t = uint32_t[5];
  template <int S>
  static __device__ __forceinline__ void load_pf(pf_t& pf, const lanes& L)
  {
    if constexpr (S >= 0 && S < G.n_steps) {
      static constexpr spec::srole ro = G.steps[S].r[0];
      if constexpr (pre_lds<ro>()) {
        static_assert((ro.npos + 1) / 2 <= 5, "five address pairs per split row");
        constexpr int K0 = lds_pairs_before(S);
        static_for<(ro.npos + 1) / 2>([&](auto ic) __attribute__((always_inline)) {
          constexpr int i = decltype(ic)::value;
          pf[i]           = *lds_word(L.abase + static_cast<uint32_t>(K0 + i) * WG * 4U);
        });
      }
    }
  }

  /* The role's lane words pass through opaque asm once per step: every address is a function of them and
   * iteration-invariant, and is to be computed in the step, not hoisted. */
  template <const spec::srole& RO>
  static __device__ __forceinline__ lanes role_lanes(const lanes& L0)
  {
    lanes L = L0;
    if constexpr (RO.p == 2) {
      /* the upper half's per-position address deltas are iteration-invariant: computed here, not hoisted */
      L.t2    = opaque(L0.t2);
      L.t2h   = opaque(L0.t2h);
      L.hmask = opaque(L0.hmask);
    } else if constexpr (C1) {
      L.t1[RO.grp] = opaque(L0.t1[RO.grp]);
    }
    return L;
  }

  /* The early part of the next step's row (sstep::e): reads and pass 1 of its first nearly positions. */
  template <int S>
  static __device__ __forceinline__ void role_early(cr_t& cr, carry& cy, const lanes& L0)
  {
    static constexpr spec::srole ro = G.steps[S].e;
    constexpr int                Q0 = ro.q0;
    constexpr int                NP = (ro.npos + 1) / 2;
    constexpr int                NE = ro.nearly / 2;
    const lanes                  L  = role_lanes<ro>(L0);
    if (!lane_active<1, ro.grp>(L)) {
      return;
    }
    int lo[NE], hi[NE];
    static_for<NE>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      cy.base[2 * i]     = pos_base<ro, 2 * i>(L);
      cy.base[2 * i + 1] = pos_base<ro, 2 * i + 1>(L);
      lo[i]              = rds(cy.base[2 * i], pos_imm<ro, 2 * i>() + RD);
      hi[i]              = rds(cy.base[2 * i + 1], pos_imm<ro, 2 * i + 1>() + RD);
    });
    /* the late positions' addresses too (no data dependency): off the completing waves' path in the next step */
    static_for<NP - NE>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = NE + decltype(ic)::value;
      cy.base[2 * i]     = pos_base<ro, 2 * i>(L);
      cy.base[2 * i + 1] = pos_base<ro, 2 * i + 1>(L);
    });
    u16x2    M1 = splatu(MIN_START), M2 = splatu(MIN_START);
    uint32_t SX = 0;
    static_for<NE>([&](auto ic) __attribute__((always_inline)) {
      constexpr int  i  = decltype(ic)::value;
      const uint32_t sx = __builtin_amdgcn_perm(static_cast<uint32_t>(hi[i]), static_cast<uint32_t>(lo[i]), 0x05040100U);
      pass1(sx, cr[Q0 + i], M1, M2, SX, cy.gs[i], cy.a[i], L.one2);
    });
    cy.m1 = M1;
    cy.m2 = M2;
    cy.sx = SX;
  }

  /* One role of step S: reads, pass 1 per edge pair (after the early pairs of the previous step, if any), the check
   * node's minima (and the split-row merge), the scaled magnitudes, pass 2 per pair and the soft-bit writes. */
  template <int S, int RI>
  static __device__ __forceinline__ void role(cr_t& cr, carry& cy, const lanes& L0, const pf_t& pf)
  {
    static constexpr spec::srole ro = G.steps[S].r[RI];
    constexpr int                Q0 = ro.q0;
    constexpr int                NP = (ro.npos + 1) / 2; /* pairs */
    constexpr int                NE = ro.nearly / 2;     /* pairs run early */
    constexpr bool               PRE = pre_addr<ro>() || pre_lds<ro>(); /* split row: addresses precomputed */
    constexpr bool               PRL = pre_lds<ro>();                    /* ... and kept in LDS              */
    constexpr int                SK  = PRL ? lds_pairs_before(S) : split_pairs_before(S);
    const lanes                  L  = role_lanes<ro>(L0);
    if (!lane_active<ro.p, ro.grp>(L)) {
      return;
    }
    uint32_t base[2 * NP], Sx[NP], Gs[NP], A[NP];
    int      lo[NP], hi[NP];
    u16x2    M1 = splatu(MIN_START), M2 = splatu(MIN_START);
    uint32_t SX = 0;
    if constexpr (NE > 0) {
      M1 = cy.m1;
      M2 = cy.m2;
      SX = cy.sx;
      static_for<NE>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        base[2 * i]     = cy.base[2 * i];
        base[2 * i + 1] = cy.base[2 * i + 1];
        Gs[i]           = cy.gs[i];
        A[i]            = cy.a[i];
      });
    }
    static_for<NP - NE>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = NE + decltype(ic)::value;
      if constexpr (NE > 0) { /* computed by the early role */
        base[2 * i]     = cy.base[2 * i];
        base[2 * i + 1] = cy.base[2 * i + 1];
      } else
      if constexpr (PRL) { /* full addresses from the LDS table (fill_split), read ahead (load_pf); immediate 0 */
        const uint32_t w = pf[i];
        base[2 * i]      = w & 0xffffU;
        base[2 * i + 1]  = w >> 16;
      } else if constexpr (PRE) { /* full addresses, precomputed (fill_split); immediate 0 */
        base[2 * i]     = L.sa[SK + i] & 0xffffU;
        base[2 * i + 1] = L.sa[SK + i] >> 16;
      } else {
        base[2 * i]     = pos_base<ro, 2 * i>(L);
        base[2 * i + 1] = pos_base<ro, 2 * i + 1>(L);
      }
      lo[i]           = rds(base[2 * i], (PRE ? 0U : pos_imm<ro, 2 * i>()) + RD);
      /* a position past the role's last (both halves dummy): +infinity without a read */
      hi[i] = (2 * i + 1 < ro.npos) ? rds(base[2 * i + 1], (PRE ? 0U : pos_imm<ro, 2 * i + 1>()) + RD) : SOFT_INF;
    });
    static_for<NP - NE>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = NE + decltype(ic)::value;
      /* pack the two sign-extended bytes: [lo.b0, lo.b1, hi.b0, hi.b1] */
      Sx[i] = __builtin_amdgcn_perm(static_cast<uint32_t>(hi[i]), static_cast<uint32_t>(lo[i]), 0x05040100U);
      if constexpr (i == NE) {
        SPEC_STAMP_FULL(S, 1);
      }
      pass1(Sx[i], cr[Q0 + i], M1, M2, SX, Gs[i], A[i], L.one2);
    });
    SPEC_STAMP_FULL(S, 2);
    uint32_t m1, m2, sx;
    fold_halves(M1, M2, SX, m1, m2, sx);
    if constexpr (ro.p == 2) {
      merge_partner(m1, m2, sx);
    }
    s16x2 N1, CC, PP; /* n = round(0.8 m) (gen.cpp:70-79 with sf = 0.8f), n2 + m1, the sign parity */
    row_consts(m1, m2, sx, N1, CC, PP);
    SPEC_STAMP_FULL(S, 3);
    /* Graphs with one wave per row group (Z <= 64): every pair's pass 2 before any of its writes, so the scheduler
     * can interleave the pairs' chains (a packed op reading the previous one's result otherwise waits an s_nop); the
     * step is a latency chain there (BG2 Z=36: 65.8 -> 63.5 us per 128-CB batch). Larger graphs keep pass 2 and the
     * writes pair by pair (batched: BG1 Z=384 +1.5%, profiles/r03/p2_batch_ab.txt). */
    constexpr bool P2B = G.W == 1;
    uint32_t       snv[NP];
    if constexpr (P2B) {
      static_for<NP>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        pass2(Gs[i], A[i], N1, CC, PP, cr[Q0 + i], snv[i], L.onef);
      });
    }
    static_for<NP>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      uint32_t      sn;
      if constexpr (P2B) {
        sn = snv[i];
      } else {
        pass2(Gs[i], A[i], N1, CC, PP, cr[Q0 + i], sn, L.onef);
      }
      constexpr uint32_t i0 = PRE ? 0U : pos_imm<ro, 2 * i>(), i1 = PRE ? 0U : pos_imm<ro, 2 * i + 1>();
      if constexpr (pos_ext<ro, 2 * i>()) {
        wrs(base[2 * i], i0 + RD, sn); /* t + 0 never wraps and only this row reads it: one copy */
      } else {
        if constexpr (C1) {
          wrs(base[2 * i], i0, sn);
        } else {
          wrs(base[2 * i], i0, sn);
          wrs(base[2 * i], i0 + Z, sn);
          wrs(base[2 * i], i0 + 2 * Z, sn);
        }
      }
      const uint32_t sh = sn >> 16;
      if constexpr (2 * i + 1 >= ro.npos) {
        /* dummy: nothing to write */
      } else if constexpr (pos_ext<ro, 2 * i + 1>()) {
        wrs(base[2 * i + 1], i1 + RD, sh);
      } else {
        if constexpr (C1) {
          wrs(base[2 * i + 1], i1, sh);
        } else {
          wrs(base[2 * i + 1], i1, sh);
          wrs(base[2 * i + 1], i1 + Z, sh);
          wrs(base[2 * i + 1], i1 + 2 * Z, sh);
        }
      }
    });
  }

  /* Wave priority (s_setprio) on graphs with W >= 3 waves per group: in a pipelined chain the group completing a row
   * is on the step's critical path and the group running the next row's early part is not, so the arbiter issues the
   * completing waves first when both compete for a SIMD. C2 batch 150.4 -> 148.9 us, BG1 Z = 256 119.2 -> 116.8 us;
   * on BG2 Z = 128 (W = 2) it was 1% slower, so the smaller graphs keep equal priorities
   * (profiles/r02/prio.txt). */
#ifndef LDPC_SPEC_WAVE_PRIO
#define LDPC_SPEC_WAVE_PRIO 1
#endif
  template <int PR>
  static __device__ __forceinline__ void set_prio()
  {
    if constexpr (LDPC_SPEC_WAVE_PRIO && G.W >= 3) {
      __builtin_amdgcn_s_setprio(PR);
    }
  }

  /* cy: the state the early part of this step's row left (read by its role); on return, the state this step's early
   * role leaves for the next step. nx starts undefined, so on every path but the early role's the carried registers
   * are dead across the step (no copies to keep a value no later role on that wave reads). */
  template <int S, bool WRAP>
  static __device__ __forceinline__ void step(cr_t& cr, carry& cy, const lanes& L0, pf_t& pf)
  {
    pf_t cur;
    for (int i = 0; i < 5; ++i) {
      cur[i] = pf[i];
    }
    load_pf<(S + 1 < G.n_steps) ? S + 1 : (WRAP ? 0 : -1)>(pf, L0); /* the next split step's table words */
    SPEC_STAMP(S, 0);
    constexpr spec::sstep st = G.steps[S];
    carry                 nx;
    /* What this wave does in step S: at most one role (a wave belongs to one group; rows beyond the adaptive layer
     * count, impl.cpp:103-114, are skipped). One scalar bit test per role (role_masks). */
    constexpr uint32_t bit = 1U << S;
    /* the masks pass through opaque asm in every step: the tests are loop-invariant, and hoisted out of the iteration
     * loop they would hold one SGPR pair per step and role (spilled) */
    if ((opaque_s(L0.act[0]) & bit) != 0U) {
      set_prio<(st.r[0].p == 1 && (st.r[0].nearly > 0 || st.e.row >= 0)) ? 2 : 1>(); /* a chain row's completion */
      role<S, 0>(cr, cy, L0, cur);
    } else if constexpr (st.r[1].row >= 0) {
      if ((opaque_s(L0.act[1]) & bit) != 0U) {
        set_prio<1>();
        role<S, 1>(cr, cy, L0, cur);
      }
    } else if constexpr (st.e.row >= 0) {
      if ((opaque_s(L0.act[2]) & bit) != 0U) {
        set_prio<0>(); /* the early role has slack until the barrier: the completing group issues first */
        role_early<S>(cr, nx, L0);
      }
    }
    if constexpr (st.e.row >= 0 || st.r[0].nearly > 0) {
      cy = nx;
    }
#ifdef LDPC_HIP_DIAG_FULL
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    SPEC_STAMP(S, 4);
#endif
    __syncthreads();
    SPEC_STAMP(S, 5);
  }

  template <int... S>
  static __device__ __forceinline__ void iteration_impl(cr_t& cr, const lanes& L, pf_t& pf,
                                                        std::integer_sequence<int, S...>)
  {
    carry cy;
    (step<S, true>(cr, cy, L, pf), ...);
  }

  /* one full iteration; pf holds step 0's table words on entry (load_pf<0> before the loop) and on exit */
  static __device__ __forceinline__ void iteration(cr_t& cr, const lanes& L, pf_t& pf)
  {
    iteration_impl(cr, L, pf, std::make_integer_sequence<int, G.n_steps>{});
  }

#ifndef LDPC_SPEC_PARTIAL_LAYERS
#define LDPC_SPEC_PARTIAL_LAYERS 12
#endif
  /* Codeblocks with few layers (high code rate: impl.cpp:103-114 adapts the layer count to the codeblock length, a
   * 6-layer BG1 Z=384 CB in C4's large TB). Steps run in row order, so once a step's first row is beyond the layer
   * count every later step is empty too; an empty step still costs every wave its scalar role checks (about 20 SALU
   * instructions per wave and step on the CU's one scalar unit: a 4-layer BG1 Z=384 iteration spent 6.0 us, 2.2 of
   * them in its 28 empty steps). Codeblocks with at most PARTIAL_LAYERS layers run this iteration instead: the first
   * PARTIAL_STEPS steps, ending at the first empty one. Full-length codeblocks keep the unchecked iteration (the
   * checks in every step cost C2 1-2%, profiles/r03/exit_ab.txt). */
  static constexpr int PARTIAL_LAYERS = LDPC_SPEC_PARTIAL_LAYERS;
  static constexpr int partial_steps()
  {
    int n = 0;
    while (n < G.n_steps && G.steps[n].r[0].row < PARTIAL_LAYERS) {
      ++n;
    }
    return n;
  }
  static constexpr int PARTIAL_STEPS = partial_steps();
  static constexpr bool HAS_PARTIAL  = PARTIAL_LAYERS > 0 && PARTIAL_STEPS < G.n_steps;
  template <int S>
  static __device__ __forceinline__ bool step_more(cr_t& cr, carry& cy, const lanes& L, pf_t& pf)
  {
    step<S, false>(cr, cy, L, pf);
    if constexpr (S + 1 < PARTIAL_STEPS) {
      return G.steps[S + 1].r[0].row < L.nof_layers;
    } else {
      return false;
    }
  }
  template <int... S>
  static __device__ __forceinline__ void partial_impl(cr_t& cr, const lanes& L, pf_t& pf,
                                                      std::integer_sequence<int, S...>)
  {
    carry cy;
    (void)(step_more<S>(cr, cy, L, pf) && ...);
  }
  static __device__ __forceinline__ void iteration_partial(cr_t& cr, const lanes& L)
  {
    pf_t pf;
    load_pf<0>(pf, L);
    partial_impl(cr, L, pf, std::make_integer_sequence<int, PARTIAL_STEPS>{});
  }

  /* Per-wave role masks, computed once per decode from the wave's group and the layer count. Deciding a step's role
   * from the wave index and the rows' layer tests in every step cost each wave about 20 scalar instructions per step,
   * and a CU has one scalar unit for its 12 waves. */
  static_assert(G.n_steps <= 32, "one mask bit per step");
  /* The masks from a few constexpr step masks and the layer count: rows are in step order, so the steps whose
   * first row is below nl are a prefix [0, n0(nl)) (n0 a constexpr table read with one scalar load); a step's
   * second row r + 1 is below nl iff r < nl - 1, and an early role runs the next step's first row. */
  struct mask_tab {
    uint32_t r0g[2], r1g[2], eg[2], p2;
    uint8_t  n0[64];
  };
  static constexpr mask_tab make_mask_tab()
  {
    mask_tab t{};
    for (int S = 0; S < G.n_steps; ++S) {
      const spec::sstep& st = G.steps[S];
      if (st.r[0].p == 2) {
        t.p2 |= 1U << S;
      } else {
        t.r0g[st.r[0].grp] |= 1U << S;
        if (st.r[1].row >= 0) {
          t.r1g[st.r[1].grp] |= 1U << S;
        }
        if (st.e.row >= 0) {
          t.eg[st.e.grp] |= 1U << S;
        }
      }
    }
    for (int nl = 0; nl < 64; ++nl) {
      int n = 0;
      while (n < G.n_steps && G.steps[n].r[0].row < nl) {
        ++n;
      }
      t.n0[nl] = static_cast<uint8_t>(n);
    }
    return t;
  }
  static constexpr mask_tab MT = make_mask_tab();
  static __device__ __forceinline__ uint32_t prefix(int n) { return n >= 32 ? ~0U : ((1U << n) - 1U); }
  static __device__ __forceinline__ void role_masks(lanes& L)
  {
    const mask_tab&           t   = MT;
    const int                 nl  = L.nof_layers < 63 ? L.nof_layers : 63;
    const int                 n0  = t.n0[nl];
    const int                 n0m = t.n0[nl > 0 ? nl - 1 : 0];
    const uint32_t            pre0 = prefix(n0), pre1 = prefix(n0m), pree = prefix(n0 > 0 ? n0 - 1 : 0);
    uint32_t                  a0 = (L.wave < P2_WAVES) ? (t.p2 & pre0) : 0U, a1 = 0, ae = 0;
    if (L.wave < 2 * G.W) {
      const int grp = L.wave < G.W ? 0 : 1;
      a0 |= t.r0g[grp] & pre0;
      a1 = t.r1g[grp] & pre1;
      ae = t.eg[grp] & pree;
    }
    L.act[0] = opaque_s(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a0))));
    L.act[1] = opaque_s(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a1))));
    L.act[2] = opaque_s(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(ae))));
  }

  template <bool FILL>
  static __device__ __forceinline__ lanes make_lanes(int wave, int lane, int nof_layers, uint32_t abase)
  {
    lanes L{};
    L.abase      = abase;
    L.wave       = wave;
    L.lane       = lane;
    L.nof_layers = nof_layers;
    L.one2       = opaque_s(SB == 2 ? 0x80008000U : 0x00010001U);
    L.onef       = opaque_s(0x3c003c00U);
    for (int i = 0; i < 2; ++i) { /* byte offsets of the lane's check node */
      L.t1[i]  = static_cast<uint32_t>(SB * ((wave - i * G.W) * 64 + lane));
      L.t1h[i] = L.t1[i] + HI;
    }
    L.t2    = static_cast<uint32_t>(SB * (wave * 32 + (lane & 31)));
    L.t2h   = L.t2 + HI;
    L.hmask = (lane >= 32) ? 0xffffffffU : 0U;
    for (auto& w : L.sa) {
      w = 0;
    }
    if constexpr (FILL && !LDPC_SPEC_SPLIT_COPY) {
      fill_split(L, std::make_integer_sequence<int, G.n_steps>{});
    }
    role_masks(L);
    return L;
  }

  /* The split-row address table of this graph into global memory (ldpc_split_table_kernel, once per context): the
   * words fill_split would write into LDS, at the same word index, so a codeblock's prologue copies them instead of
   * computing them (about 300 VALU instructions per lane, 1.1 us per codeblock at Z = 384). */
  static __device__ __forceinline__ void write_split_table(uint32_t* gdst, int wave, int lane)
  {
    lanes L = make_lanes<false>(wave, lane, 64, 0U);
    fill_split(L, std::make_integer_sequence<int, G.n_steps>{}, gdst);
  }
};

/* ---- lane-split decoder of the one-wave graphs (spec::qgraph, ldpc_spec.h) ----------------------------------------
 * Step S: a two-row step runs row r[0] on waves [0, WH) and row r[1] on waves [WH, 2 WH), P2 lanes per check node
 * (lane i of a group: check node i / P2, edges i % P2 + P2 j); a single-row step runs its row on every wave, 2 P2
 * lanes per check node. Per lane and step: its address pairs and c2v pairs sit in the step's register slots [q0, q0 + nq)
 * (the same slots for both roles of a step: each lane runs one role), the reads, pass 1 of each edge pair, the merge of
 * the check node's partial minima and parity across its lanes (DPP), the scaled magnitudes, pass 2 and the writes,
 * then the step barrier. Positions without an edge address the scratch column held at +infinity. */
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v)
{
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, 0xf, 0xf, false));
}

/* merge of two lanes' (min1, min2, parity): the two smallest of the multiset and the XOR of the parities */
template <int CTRL>
__device__ __forceinline__ void merge_lanes(uint32_t& m1, uint32_t& m2, uint32_t& sx)
{
  const uint32_t o1 = dpp_mov<CTRL>(m1), o2 = dpp_mov<CTRL>(m2), os = dpp_mov<CTRL>(sx);
  m2 = min(min(m2, o2), max(m1, o1));
  m1 = min(m1, o1);
  sx ^= os;
}

template <const spec::sgraph& G, const spec::qgraph& Q>
struct qdec {
  static constexpr int      Z       = G.Z;
  static constexpr int      NS      = Q.slots;
  static constexpr uint32_t WG      = static_cast<uint32_t>(Q.waves) * 64U; /* table stride: lanes per workgroup */
  static constexpr uint32_t SCRATCH = static_cast<uint32_t>(SB * G.N_full) * static_cast<uint32_t>(Z);
  static_assert(Q.valid && SCRATCH + SB * Z <= 65535U, "lane-split schedule: 16-bit LDS addresses");
  using cr_t = uint32_t[NS];

  struct qlanes {
    uint32_t one2, onef;
    int      nof_layers, grp;
    bool     act2, act1; /* this lane's check node exists (t < Z) in a two-row / a single-row step */
  };
  static __device__ __forceinline__ qlanes make_lanes(int wave, int lane, int nof_layers)
  {
    qlanes L{};
    L.one2       = opaque_s(SB == 2 ? 0x80008000U : 0x00010001U);
    L.onef       = opaque_s(0x3c003c00U);
    L.nof_layers = nof_layers;
    L.grp        = wave < Q.WH ? 0 : 1;
    L.act2       = ((wave - L.grp * Q.WH) * 64 + lane) / Q.P2 < Z;
    L.act1       = (wave * 64 + lane) / (2 * Q.P2) < Z;
    return L;
  }

  /* The address table (ldpc_split_table_kernel, once per context): word (q0 + i) * WG + tid holds the LDS addresses
   * of the lane's positions 2 i and 2 i + 1 in the step's role, soft[col][(t + shift) mod Z] (scratch: no edge). */
  template <int S>
  static __device__ __forceinline__ void write_table_step(uint32_t* dst, int wave, int lane)
  {
    constexpr spec::qstep st   = Q.steps[S];
    constexpr bool        pair = st.r[1].row >= 0;
    const int             ri   = (pair && wave >= Q.WH) ? 1 : 0;
    const int             P    = pair ? Q.P2 : 2 * Q.P2;
    const int             i    = pair ? (wave - ri * Q.WH) * 64 + lane : wave * 64 + lane;
    const int             t = i / P, k = i % P;
    int                   col[spec::MAX_DEG], sh[spec::MAX_DEG], deg = 0, npos = 0;
    static_for<2>([&](auto rc) __attribute__((always_inline)) {
      constexpr int R = decltype(rc)::value;
      if constexpr (R == 0 || pair) {
        constexpr spec::srow row = G.rows[st.r[R].row];
        if (ri == R) {
          deg  = row.deg;
          npos = st.r[R].npos;
          static_for<spec::MAX_DEG>([&](auto ec) __attribute__((always_inline)) {
            constexpr int e = decltype(ec)::value;
            col[e]          = row.col[e];
            sh[e]           = row.sh[e];
          });
        }
      }
    });
    for (int q = 0; q < st.nq; ++q) {
      uint32_t a[2];
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * q + h, e = k + P * j;
        a[h]        = SCRATCH;
        if (t < Z && j < npos && e < deg) {
          a[h] = static_cast<uint32_t>(SB * (col[e] * Z + (t + sh[e]) % Z));
        }
      }
      dst[static_cast<uint32_t>(st.q0 + q) * WG + static_cast<uint32_t>(wave * 64 + lane)] = a[0] | (a[1] << 16);
    }
  }
  template <int... Ss>
  static __device__ __forceinline__ void write_table(uint32_t* dst, int wave, int lane, std::integer_sequence<int, Ss...>)
  {
    (write_table_step<Ss>(dst, wave, lane), ...);
  }

  template <int S, int RI>
  static __device__ __forceinline__ void role(cr_t& cr, const cr_t& tab, const qlanes& L)
  {
    constexpr spec::qstep st = Q.steps[S];
    constexpr spec::qrole ro = st.r[RI];
    constexpr int         NP = (ro.npos + 1) / 2;
    constexpr int         Q0 = st.q0;
    if (!(ro.P == Q.P2 ? L.act2 : L.act1)) {
      return;
    }
    uint32_t base[2 * NP], Gs[NP], A[NP];
    int      lo[NP], hi[NP];
    static_for<NP>([&](auto ic) __attribute__((always_inline)) {
      constexpr int  i = decltype(ic)::value;
      const uint32_t w = opaque(tab[Q0 + i]); /* read in the step: not hoisted out of the iteration loop */
      base[2 * i]      = w & 0xffffU;
      base[2 * i + 1]  = w >> 16;
      lo[i]            = rds(base[2 * i], 0);
      hi[i]            = (2 * i + 1 < ro.npos) ? rds(base[2 * i + 1], 0) : SOFT_INF;
    });
    SPEC_STAMP_FULL(S, 1);
    u16x2    M1 = splatu(MIN_START), M2 = splatu(MIN_START);
    uint32_t SX = 0;
    static_for<NP>([&](auto ic) __attribute__((always_inline)) {
      constexpr int  i  = decltype(ic)::value;
      const uint32_t sx = __builtin_amdgcn_perm(static_cast<uint32_t>(hi[i]), static_cast<uint32_t>(lo[i]), 0x05040100U);
      pass1(sx, cr[Q0 + i], M1, M2, SX, Gs[i], A[i], L.one2);
    });
    uint32_t m1, m2, sx;
    fold_halves(M1, M2, SX, m1, m2, sx);
    merge_lanes<0xb1>(m1, m2, sx); /* quad_perm [1, 0, 3, 2]: the lane pair */
    if constexpr (ro.P >= 4) {
      merge_lanes<0x4e>(m1, m2, sx); /* quad_perm [2, 3, 0, 1]: the other pair of the quad */
    }
    if constexpr (ro.P >= 8) {
      merge_lanes<0x141>(m1, m2, sx); /* row_half_mirror: the other quad of the eight lanes */
    }
    static_assert(ro.P == 2 || ro.P == 4 || ro.P == 8, "lanes per check node");
    SPEC_STAMP_FULL(S, 2);
    s16x2 N1, CC, PP; /* round(0.8 m), gen.cpp:70-79; n2 + m1; the sign parity */
    row_consts(m1, m2, sx, N1, CC, PP);
    SPEC_STAMP_FULL(S, 3);
    uint32_t snv[NP];
    static_for<NP>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      pass2(Gs[i], A[i], N1, CC, PP, cr[Q0 + i], snv[i], L.onef);
    });
    static_for<NP>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      wrs(base[2 * i], 0, snv[i]);
      if constexpr (2 * i + 1 < ro.npos) {
        wrs(base[2 * i + 1], 0, snv[i] >> 16);
      }
    });
  }

  /* false when the step's first row is beyond the codeblock's layers (impl.cpp:103-114): rows go in step order, so
   * this and every later step of the iteration are empty */
  template <int S>
  static __device__ __forceinline__ bool step(cr_t& cr, const cr_t& tab, const qlanes& L)
  {
    constexpr spec::qstep st = Q.steps[S];
    if (st.r[0].row >= L.nof_layers) {
      return false;
    }
    SPEC_STAMP(S, 0);
    if constexpr (st.r[1].row >= 0) {
      if (L.grp == 0) {
        role<S, 0>(cr, tab, L);
      } else if (st.r[1].row < L.nof_layers) {
        role<S, 1>(cr, tab, L);
      }
    } else {
      role<S, 0>(cr, tab, L);
    }
#ifdef LDPC_HIP_DIAG_FULL
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    SPEC_STAMP(S, 4);
#endif
    __syncthreads();
    SPEC_STAMP(S, 5);
    return true;
  }
  template <int... S>
  static __device__ __forceinline__ void iteration_impl(cr_t& cr, const cr_t& tab, const qlanes& L,
                                                        std::integer_sequence<int, S...>)
  {
    (void)(step<S>(cr, tab, L) && ...);
  }
  static __device__ __forceinline__ void iteration(cr_t& cr, const cr_t& tab, const qlanes& L)
  {
    iteration_impl(cr, tab, L, std::make_integer_sequence<int, Q.n_steps>{});
  }
};

/* ---- register-resident decoder of the one-wave graphs (spec::rgraph, ldpc_spec.h) ---------------------------------
 * One wave per codeblock, lane t = check node t of the row being updated (lanes t >= Z: duplicates when Z divides 64,
 * don't-cares otherwise). sv[c]: column c's register (rotation and half per the compile-time state); cr: the c2v
 * pairs of every row (pair i of row r at cr[q0 + i]). A read at rotation k is one ds_bpermute_b32 from lane
 * (t + k) mod Z: when Z divides 64 the address 4 t + 4 k wraps by itself (ds_bpermute uses address bits [7:2]) and the
 * constant goes into the instruction offset; otherwise the address is byte k % 4 of the lane's rotation table word
 * rt[k / 4] (4 ((t + k) mod Z) for each k, built once per codeblock), at most one shift. */
#ifndef LDPC_SPEC_REG_SCHED_BARRIER
#define LDPC_SPEC_REG_SCHED_BARRIER 1
#endif
template <const spec::sgraph& G, const spec::rgraph& R>
struct rdec {
  static constexpr int  Z    = G.Z;
  static constexpr int  NC   = G.N_full;
  static constexpr int  NP   = R.n_pairs;
  static constexpr bool POW2 = (64 % Z) == 0;
  static constexpr int  NRT  = POW2 ? 1 : (Z + 3) / 4;
  static_assert(R.valid && NP > 0, "register-resident schedule");
  static_assert(SB == 1, "register-resident decoder: int8 soft bits (build with -DLDPC_SPEC_F16=0)");
  using sv_t = uint32_t[NC];
  using cr_t = uint32_t[NP];

  struct rlanes {
    uint32_t t4;      /* 4 * lane */
    uint32_t rt[NRT]; /* byte j of rt[q]: 4 ((lane + 4 q + j) mod Z) (Z not dividing 64) */
    uint32_t one2, c121;
    int      nl; /* the codeblock's layer count (uniform) */
  };
  static __device__ __forceinline__ rlanes make_lanes(int lane, int nl)
  {
    rlanes L{};
    L.t4 = 4U * static_cast<uint32_t>(lane);
    if constexpr (!POW2) {
      for (int q = 0; q < NRT; ++q) {
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) {
          w |= (4U * static_cast<uint32_t>((lane + 4 * q + j) % Z)) << (8 * j);
        }
        L.rt[q] = w;
      }
    } else {
      L.rt[0] = 0;
    }
    L.one2 = opaque_s(0x00010001U);
    L.c121 = opaque_s(121U);
    L.nl   = nl;
    return L;
  }

  template <int K>
  static __device__ __forceinline__ uint32_t rot(uint32_t v, const rlanes& L)
  {
    if constexpr (K == 0) {
      return v;
    } else if constexpr (POW2) {
      return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(L.t4 + 4U * K), static_cast<int>(v)));
    } else {
      constexpr int  q = K / 4, j = K % 4;
      const uint32_t a = j == 0 ? L.rt[q] : (L.rt[q] >> (8 * j));
      return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(a), static_cast<int>(v)));
    }
  }
  /* v_perm selector: the low half from byte pair h0 of src1, the high half from byte pair h1 of src0 */
  static constexpr uint32_t psel(int h0, int h1)
  {
    return static_cast<uint32_t>((2 * h0) | ((2 * h0 + 1) << 8) | ((4 + 2 * h1) << 16) | ((5 + 2 * h1) << 24));
  }

  /* the lane words pass through opaque asm once per row, in place (a copy would cost a v_mov per word and row):
   * every rotation address derived from them is iteration-invariant, and hoisted out of the iteration loop they
   * would hold a register per rotation */
  static __device__ __forceinline__ void opaque_lanes(rlanes& L)
  {
    asm volatile("" : "+v"(L.t4));
    for (int q = 0; q < NRT; ++q) {
      asm volatile("" : "+v"(L.rt[q]));
    }
  }

  template <int RI, bool MASK>
  static __device__ __forceinline__ void row(sv_t& sv, cr_t& cr, rlanes& L)
  {
    opaque_lanes(L);
    static constexpr spec::rrow rw  = R.rows[RI];
    constexpr int               NPR = (rw.deg + 1) / 2;
    uint32_t                    Gs[NPR], A[NPR];
    u16x2                       M1 = splatu(MIN_START), M2 = splatu(MIN_START);
    uint32_t                    SX = 0;
    static_for<NPR>([&](auto ic) __attribute__((always_inline)) {
      constexpr int  i   = decltype(ic)::value;
      constexpr bool two = 2 * i + 1 < rw.deg;
      constexpr int  j1  = two ? 2 * i + 1 : 2 * i;
      constexpr int  c0 = rw.e[2 * i].col, k0 = rw.e[2 * i].k, h0 = rw.e[2 * i].half, g0 = rw.e[2 * i].reg;
      constexpr int  c1 = rw.e[j1].col, k1 = rw.e[j1].k, h1 = two ? rw.e[j1].half : 0, g1 = rw.e[j1].reg;
      uint32_t       S;
      if constexpr (two && g0 == g1 && k0 == k1 && h0 == 0 && h1 == 1) {
        S = rot<k0>(sv[c0], L); /* both edges' columns in one register, same rotation: already the pair */
      } else {
        const uint32_t v0 = rot<k0>(sv[c0], L);
        uint32_t       v1 = L.c121; /* no second edge: +infinity */
        if constexpr (two) {
          v1 = rot<k1>(sv[c1], L);
        }
        S = __builtin_amdgcn_perm(v1, v0, psel(h0, h1));
      }
      pass1(S, cr[rw.q0 + i], M1, M2, SX, Gs[i], A[i], L.one2);
    });
    uint32_t m1, m2, sx;
    fold_halves(M1, M2, SX, m1, m2, sx);
    uint32_t n1 = (__umul24(m1, 52432U) + 26216U) >> 16; /* round(0.8 m), gen.cpp:70-79 */
    uint32_t cc = ((__umul24(m2, 52432U) + 26216U) >> 16) + m1;
    if constexpr (MASK && RI >= 4) { /* a row beyond the layer count (nl >= 4 always) updates to the identity */
      /* opaque: hoisted out of the iteration loop, the 38 row tests became spilled 64-bit masks and v_cndmask */
      const uint32_t act = RI < static_cast<int>(opaque_s(static_cast<uint32_t>(L.nl))) ? ~0U : 0U;
      n1 &= act;
      cc &= act;
    }
    const s16x2 N1 = splat(static_cast<int>(n1));
    const s16x2 CC = splat(static_cast<int>(cc));
    const s16x2 PP = splat(static_cast<short>(sx | 1U));
    static_for<NPR>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      uint32_t      sn;
      pass2(Gs[i], A[i], N1, CC, PP, cr[rw.q0 + i], sn, 0U);
      sv[rw.e[2 * i].col] = sn;
      if constexpr (2 * i + 1 < rw.deg) {
        sv[rw.e[2 * i + 1].col] = sn;
      }
    });
#if LDPC_SPEC_REG_SCHED_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
  }

  static constexpr int chunk_begin(int x) { return x == 0 ? 0 : R.exit_row[x - 1]; }
  static constexpr int chunk_end(int x) { return x < R.n_exits ? R.exit_row[x] : G.M; }

  /* leaving the iteration before row exit_row[XI]: every column the rest of the iteration would have written goes
   * to its boundary state (rotation, half, and the register it shares with its boundary partner) */
  template <int XI>
  static __device__ __forceinline__ void fixup(sv_t& sv, rlanes& L)
  {
    opaque_lanes(L);
    static_for<NC>([&](auto ccn) __attribute__((always_inline)) {
      constexpr int c    = decltype(ccn)::value;
      constexpr int p    = R.partner[c];
      constexpr int pp   = p < 0 ? c : p;
      constexpr int k    = (R.end[c].rho - R.at_exit[XI][c].rho + Z) % Z;
      constexpr int kp   = (R.end[pp].rho - R.at_exit[XI][pp].rho + Z) % Z;
      constexpr int ch   = R.at_exit[XI][c].half, eh = R.end[c].half, chp = R.at_exit[XI][pp].half;
      if constexpr (R.at_exit[XI][c].reg != R.end[c].reg && (p < 0 || eh == 0)) {
        const uint32_t v = rot<k>(sv[c], L);
        if constexpr (p < 0) {
          sv[c] = ch == eh ? v : (eh != 0 ? (v << 16) : (v >> 16));
        } else {
          const uint32_t vp = rot<kp>(sv[p], L);
          const uint32_t w  = __builtin_amdgcn_perm(vp, v, psel(ch, chp));
          sv[c]                     = w;
          sv[p]                     = w;
        }
      }
    });
  }

  template <int B, bool MASK, int... I>
  static __device__ __forceinline__ void rows_impl(sv_t& sv, cr_t& cr, rlanes& L, std::integer_sequence<int, I...>)
  {
    (row<B + I, MASK>(sv, cr, L), ...);
  }
  template <int X>
  static __device__ __forceinline__ bool chunk(sv_t& sv, cr_t& cr, rlanes& L)
  {
    if constexpr (X > 0) {
      if (chunk_begin(X) >= static_cast<int>(opaque_s(static_cast<uint32_t>(L.nl)))) {
        fixup<X - 1>(sv, L);
        return false;
      }
    }
    rows_impl<chunk_begin(X), true>(sv, cr, L, std::make_integer_sequence<int, chunk_end(X) - chunk_begin(X)>{});
    return true;
  }
  template <int... X>
  static __device__ __forceinline__ void iteration_impl(sv_t& sv, cr_t& cr, rlanes& L,
                                                        std::integer_sequence<int, X...>)
  {
    (void)(chunk<X>(sv, cr, L) && ...);
  }
  /* a codeblock with fewer layers than rows: chunks, exits and identity rows */
  static __device__ __forceinline__ void iteration_partial(sv_t& sv, cr_t& cr, rlanes& L)
  {
    iteration_impl(sv, cr, L, std::make_integer_sequence<int, R.n_exits + 1>{});
  }
  /* every row a layer (nl == M): one straight-line block, no exits, no masks */
  static __device__ __forceinline__ void iteration(sv_t& sv, cr_t& cr, rlanes& L)
  {
    rows_impl<0, false>(sv, cr, L, std::make_integer_sequence<int, G.M>{});
  }

  /* the registers in their boundary state from the soft bits in LDS (column c at c Z) */
  static __device__ __forceinline__ void load(sv_t& sv, int lane)
  {
    const int tz = POW2 ? (lane & (Z - 1)) : lane;
    static_for<NC>([&](auto ccn) __attribute__((always_inline)) {
      constexpr int c    = decltype(ccn)::value;
      constexpr int rho  = R.end[c].rho, half = R.end[c].half;
      constexpr int p    = R.partner[c];
      constexpr int rhop = p < 0 ? 0 : R.end[p < 0 ? 0 : p].rho;
      if constexpr (p < 0 || half == 0) {
        const uint32_t va = static_cast<uint32_t>(rd8(static_cast<uint32_t>((tz + rho) % Z), c * Z));
        if constexpr (p < 0) {
          sv[c] = half != 0 ? (va << 16) : va;
        } else {
          const uint32_t vb = static_cast<uint32_t>(rd8(static_cast<uint32_t>((tz + rhop) % Z), p * Z));
          const uint32_t w  = __builtin_amdgcn_perm(vb, va, 0x05040100U);
          sv[c]             = w;
          sv[p]             = w;
        }
      }
    });
  }
  /* Early stop from the registers (the check of impl.cpp:126-134 without the LDS hard-decision and CRC passes, whose
   * registers on top of the decoder's spilled it): hard bit = soft <= 0 (llr.cpp:226-252), any zero soft bit of the
   * K Z systematic ones fails, and the CRC of the first Lsig hard bits (zero-init, MSB first) is linear in them: lane t
   * keeps, per systematic column c, the remainder x^(Lsig - 1 - i + order) mod G of its bit i = c Z + (t + rho_c) mod Z
   * (zero for i >= Lsig and for lanes t >= Z), and the check XORs the ones of its set bits over the wave. */
  using ec_t = uint32_t[G.K];
  static __device__ __forceinline__ void et_setup(ec_t& ec, int lane, int Lsig, int order, const uint32_t* xpow)
  {
    static_for<G.K>([&](auto ccn) __attribute__((always_inline)) {
      constexpr int c = decltype(ccn)::value;
      constexpr int rho = R.end[c].rho;
      const int     i   = c * Z + (lane + rho) % Z;
      ec[c]             = (lane < Z && i < Lsig) ? xpow[Lsig - 1 - i + order] : 0U;
    });
  }
  static __device__ __forceinline__ bool et_check(const sv_t& sv, const ec_t& ec, int lane)
  {
    uint32_t acc = 0, zero = 0;
    static_for<G.K>([&](auto ccn) __attribute__((always_inline)) {
      constexpr int c    = decltype(ccn)::value;
      constexpr int half = R.end[c].half;
      const int     v    = half != 0 ? (static_cast<int>(sv[c]) >> 16) : static_cast<int>(static_cast<short>(sv[c]));
      acc ^= v <= 0 ? ec[c] : 0U;
      zero |= v == 0 ? 1U : 0U;
    });
    /* uniform (readfirstlane, ballot): a per-lane condition would make the loop exit divergent, and the compiler
     * then keeps every loop-carried register twice (spilled) */
    acc = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(wave_xor(acc))));
    return __builtin_amdgcn_ballot_w64(zero != 0U && lane < Z) == 0 && acc == 0U;
  }

  /* the systematic columns' soft bits back into LDS (the hard decision reads [0, K Z)) */
  static __device__ __forceinline__ void store_systematic(const sv_t& sv, int lane)
  {
    if (lane < Z) {
      static_for<G.K>([&](auto ccn) __attribute__((always_inline)) {
        constexpr int c = decltype(ccn)::value;
        constexpr int rho = R.end[c].rho, half = R.end[c].half;
        wr8(static_cast<uint32_t>((lane + rho) % Z), c * Z, half != 0 ? (sv[c] >> 16) : sv[c]);
      });
    }
  }
};

} // namespace sp

} // namespace

/* Lifted graphs of every (BG, Z), indexed by slot = (BG - 1) * 51 + lifting position; slot 102 + s holds graph s
 * with the narrow step schedule (ldpc_graph.h NARROW_SLOT_BASE). Constant memory: all row, step and edge words are
 * read with scalar loads (the row a wave works on is uniform). One copy per translation unit (static): the one
 * ldpc_hip_kernels.hip uploads serves the generic and mixed kernels; the specialised kernels compiled elsewhere
 * (ldpc_spec_kernels_*.hip) take every graph field from their compile-time schedule and never read it. */
static __constant__ graph_desc c_graphs[204];

} // namespace ldpc_hip
#include "ldpc_dematch_body.h" /* dematch_body: the decode kernels' fused first phase */
namespace ldpc_hip {

/* Graph fields of the generic body (this unit's c_graphs). */
__device__ __forceinline__ int graph_field_Z(int slot) { return c_graphs[slot].Z; }
__device__ __forceinline__ int graph_field_K(int slot) { return c_graphs[slot].K; }
__device__ __forceinline__ int graph_field_N(int slot) { return c_graphs[slot].N_full; }
__device__ __forceinline__ int graph_field_task_waves(int slot) { return c_graphs[slot].task_waves; }

/* One codeblock per workgroup (the body of ldpc_decode_kernel and ldpc_decode_mixed_kernel). The generic body also
 * runs in workgroups wider than its schedule (mixed launches): waves at or beyond graph->task_waves only take part in
 * the block-wide phases and the step barriers. */
template <bool SF08, int SPEC_ID>
__device__ __forceinline__ void decode_cb(const dec_cb& d, int graph_slot, const step_task* __restrict__ tasks,
                                          const lds_layout& lay, const int8_t* llr_base,
                                          uint8_t* __restrict__ out_base, ldpc_hip_cb_result* __restrict__ res_base,
                                          const uint32_t* __restrict__ crc_tables, const dematch_cb* dm_cbs,
                                          const dematch_cb& dm_one)
{
#define graph (&c_graphs[graph_slot])
  constexpr bool SPEC = SPEC_ID >= 0; /* specialised body: spec::k_specs[SPEC_ID] */
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  int8_t*   s_soft = reinterpret_cast<int8_t*>(smem); /* lay.soft == 0: column offsets are LDS addresses */
  if (static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_i8*)s_soft)) != 0U || lay.soft != 0U) {
    __builtin_trap(); /* lds_byte() would address the wrong bytes */
  }
  uint16_t* s_soft16 = reinterpret_cast<uint16_t*>(smem); /* binary16 soft bits (specialised kernels, SOFT_BYTES = 2) */
  constexpr bool F16 = SPEC_ID >= 0 && spec::SOFT_BYTES == 2;
  int8_t*   s_c2v  = reinterpret_cast<int8_t*>(smem + lay.c2v);
  uint8_t*  s_hb   = smem + lay.hard;
  uint32_t* s_red  = reinterpret_cast<uint32_t*>(smem + lay.red);
  uint32_t* s_crct = reinterpret_cast<uint32_t*>(smem + lay.crct);

#ifdef LDPC_HIP_DIAG_CB /* diagnostic build: stamp 6, the body's entry (before a fused dematcher) */
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    reinterpret_cast<uint64_t*>(const_cast<uint32_t*>(crc_tables) + DIAG_CB_OFFSET)[blockIdx.x * 8 + 6] =
        __builtin_amdgcn_s_memrealtime();
  }
#endif
  if (dm_cbs != nullptr || dm_one.soft != nullptr) {
    /* fused rate dematching (ldpc_hip_dematch_decode_launch, the HAL batch): this CB's dematcher runs first, into the
     * soft buffer the prologue then loads (llr_base + d.llr_offset); its LDS staging and table copy sit in the
     * decoder's dynamic LDS (the launch reserves DM_FUSED_LDS), free again after the barrier. A workgroup's own
     * global stores are visible to its loads after the barrier. */
    dematch_body(dm_cbs != nullptr ? dm_cbs[blockIdx.x] : dm_one,
                 *reinterpret_cast<const demod_tables*>(crc_tables + DTAB_OFFSET), reinterpret_cast<int8_t*>(smem),
                 *reinterpret_cast<demod_tables*>(smem + DM_STAGE));
    __syncthreads();
  }
  if (d.keep_passed != 0 && res_base != nullptr && res_base[d.result_index].crc_pass != 0) {
    return; /* HARQ: CRC passed in an earlier transmission; message and result stay (pusch_decoder_impl.cpp:336-346) */
  }
  const int     tid    = threadIdx.x;
  const int     nthr   = blockDim.x;
  const int     lane   = tid & 63;
  const int     wave   = __builtin_amdgcn_readfirstlane(tid >> 6);
  /* the specialised bodies take every graph field from their compile-time schedule: they may be compiled in a unit
   * whose c_graphs copy is never uploaded (ldpc_spec_kernels_*.hip) */
  using SG             = spec::spec_graph<SPEC ? SPEC_ID : 0>;
  const int     Z      = SPEC ? SG::g.Z : graph_field_Z(graph_slot);
  const int     K      = SPEC ? SG::g.K : graph_field_K(graph_slot);
  const int     N_full = SPEC ? SG::g.N_full : graph_field_N(graph_slot);
  const int     KZ     = K * Z;
  const int     L      = static_cast<int>(d.llr_length);
  const int8_t* llr    = llr_base + d.llr_offset;
  uint8_t*      out    = out_base + d.out_offset;
  const float   sf     = d.scaling_factor;

#ifdef LDPC_HIP_DIAG_CB_DM
#define LDPC_DIAG_CB_DM_ON 1
#else
#define LDPC_DIAG_CB_DM_ON 0
#endif
#ifdef LDPC_HIP_DIAG_CB /* diagnostic build: device-wide 100 MHz stamps per workgroup, in the context's table buffer
                          * (every translation unit's kernels reach it; ldpc_hip_diag_cb_read); with
                          * LDPC_HIP_DIAG_CB_DM slots 1-3 hold the fused dematcher's stamps instead */
#define CB_STAMP(k)                                                                                                    \
  if (tid == 0 && blockIdx.x < 1024 && !(LDPC_DIAG_CB_DM_ON && (k) >= 1 && (k) <= 3)) {                              \
    reinterpret_cast<uint64_t*>(const_cast<uint32_t*>(crc_tables) + DIAG_CB_OFFSET)[blockIdx.x * 8 + (k)] =         \
        __builtin_amdgcn_s_memrealtime();                                                                              \
  }
#else
#define CB_STAMP(k)
#endif
  CB_STAMP(0);
  /* ---- prologue: soft bits (load_soft_bits, impl.cpp:149-174), CRC tables, zeroed c2v records ----
   * Every global load a thread needs is issued before any of them is used (the LLRs, up to PRO_U 16-byte loads per
   * thread and pass, then the CRC tables), so their latencies overlap instead of adding up loop trip by loop trip;
   * the last non-zero LLR index is reduced per wave (DPP) into s_red[wave], so no barrier is needed before it. */
  int       last_local = 0;
  const int total      = N_full * Z;
  const bool vec16     = (reinterpret_cast<uintptr_t>(llr) & 15U) == 0 && ((2 * Z) & 15) == 0 && (L & 15) == 0;
  constexpr int PRO_U  = 4;
  const int z4 = (2 * Z) / 16, l4 = L / 16, t4 = (total + 15) / 16;
  const uint4* g4 = reinterpret_cast<const uint4*>(llr);
  uint4        pv[PRO_U];
  int          base4 = 0;
  if (vec16) { /* first pass's loads: [0, 2Z) zero, [2Z, 2Z + L) LLRs, rest zero */
#pragma unroll
    for (int u = 0; u < PRO_U; ++u) {
      const int i = tid + u * nthr;
      pv[u]       = (i >= z4 && i < z4 + l4 && i < t4) ? g4[i - z4] : make_uint4(0, 0, 0, 0);
    }
  }
  /* BG1 split-row address table (specialised kernel): the context's global copy, 16 bytes per load, its loads in
   * flight with the LLRs'; stored into the c2v region before the prologue barrier (a thread writes other lanes' words) */
  using SD                = sp::dec<SG::g>;
  /* one-wave graphs: the lane-split decoder (sp::qdec); its address table comes into registers here, its loads in
   * flight with the LLRs' (the same words for every codeblock of a launch: L2-resident after the first) */
  /* one-wave graphs on the register-resident decoder (sp::rdec): soft bits and c2v in registers, no tables */
  constexpr bool REG      = SPEC && spec::is_reg(SG::g);
  constexpr bool QUAD     = SPEC && !REG && spec::is_quad(SG::g);
  constexpr int  QN       = QUAD ? SG::q.slots : 1;
  using QD                = sp::qdec<SG::g, SG::q>;
  uint32_t      qtab[QN];
  if constexpr (QUAD) {
    const uint32_t* gq = crc_tables + lay.split_tab;
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      qtab[q] = gq[static_cast<uint32_t>(q) * QD::WG + static_cast<uint32_t>(tid)];
    }
  }
  constexpr int SPLIT_U4  = (SPEC && !QUAD && !REG && LDPC_SPEC_SPLIT_COPY) ? SD::LDS_PAIRS * static_cast<int>(SD::WG) / 4 : 0;
  constexpr int SPLIT_PER = 5; /* loads per thread: LDS_PAIRS / 4 at the decoder's own width */
  uint4         stv[SPLIT_PER];
  if constexpr (SPLIT_U4 > 0) {
    const uint4* gs = reinterpret_cast<const uint4*>(crc_tables + lay.split_tab);
#pragma unroll
    for (int u = 0; u < SPLIT_PER; ++u) {
      const int i = tid + u * nthr;
      stv[u]      = i < SPLIT_U4 ? gs[i] : make_uint4(0, 0, 0, 0);
    }
  }
  /* CRC tables for the LDS copy (T_0, T_1..T_3, x^(32 e) mod G: 324 16-byte chunks, every source 16-byte aligned):
   * issued here with the LLRs' and the split table's loads, stored after the LLRs. Round 4 had a loop of two 4-byte
   * loads per trip before the LLR loads: five dependent trips in a 128-thread workgroup (BG2 Z=36), most of its
   * 5 us prologue on the work-queue path. */
  constexpr int   CRC_U4  = CRC_LDS_WORDS / 4;
  constexpr int   CRC_PER = 3; /* loads per thread in flight: every chunk at 108 threads or more */
  static_assert(CRC_LDS_WORDS % 4 == 0 && 256 % 4 == 0 && CRC_TABLE_SIZE % 4 == 0 && CRC_SLICE_OFFSET % 4 == 0 &&
                    CRC_SLICE_WORDS % 4 == 0,
                "CRC tables copied in 16-byte chunks");
  const bool      crc_on = d.crc_mode != LDPC_HIP_CRC_MODE_NONE;
  const uint4*    tab4   = reinterpret_cast<const uint4*>(crc_tables + static_cast<int>(d.crc_poly) * CRC_TABLE_SIZE);
  const uint4*    slc4 =
      reinterpret_cast<const uint4*>(crc_tables + CRC_SLICE_OFFSET + static_cast<int>(d.crc_poly) * CRC_SLICE_WORDS);
  auto crc_chunk = [&](int j) { return j < 64 ? tab4[j] : (j < 256 ? slc4[j - 64] : tab4[j - 192]); };
  uint4 crcv[CRC_PER];
  if (crc_on) {
#pragma unroll
    for (int u = 0; u < CRC_PER; ++u) {
      const int j = tid + u * nthr;
      crcv[u]     = j < CRC_U4 ? crc_chunk(j) : make_uint4(0, 0, 0, 0);
    }
  }
  {
    uint4*    c2v4 = reinterpret_cast<uint4*>(s_c2v);
    int       n16  = 0; /* specialised: c2v in registers */
    if constexpr (!SPEC) {
      n16 = (static_cast<int>(graph->c2v_bytes) + 15) / 16;
    }
    for (int i = tid; i < n16; i += nthr) {
      c2v4[i] = make_uint4(0, 0, 0, 0);
    }
    const int nhb = static_cast<int>(lay.red - lay.hard) / 4;
    for (int i = tid; i < nhb; i += nthr) {
      reinterpret_cast<uint32_t*>(s_hb)[i] = 0;
    }
  }
  if constexpr (SPEC) {
    /* dummy edges of odd split rows read and write a scratch column held at +infinity (+121): never a minimum, no
     * sign, and promotion_sum keeps it there (namespace sp) */
    const int n4 = (static_cast<int>(lay.soft_stride) + 3) / 4; /* whole column (the layout leaves 64 bytes of slack) */
    int*      sc = reinterpret_cast<int*>(s_soft + static_cast<int>(lay.soft_stride) * N_full);
    for (int i = tid; i < n4; i += nthr) {
      sc[i] = F16 ? 0x57905790 : 0x79797979; /* 121.0 in binary16 / 121 = 0x79 in every byte */
    }
  } else {
    /* edge table: per row EDGE_SLOT words, padded with dummy edges at the scratch bytes after the soft columns.
     * Generic: shift | (col * Z) << 16. Specialised: col * 4Z + shift (byte offset of the copy at column offset 0). */
    uint32_t*      s_edges = reinterpret_cast<uint32_t*>(smem + lay.edges);
    constexpr bool copies4 = false;
    const uint32_t dummy   = static_cast<uint32_t>(graph->N_full) * graph->Z << 16;
    for (int i = tid; i < graph->M * EDGE_SLOT; i += nthr) {
      const int      r   = i / EDGE_SLOT, k = i - r * EDGE_SLOT;
      const uint32_t rw  = graph->rows[r];
      uint32_t       w   = dummy;
      if (k < static_cast<int>(rw >> 16)) {
        const uint32_t ew = graph->edges[(rw & 0xffffU) + k];
        w = copies4 ? (ew & 0xffffU) * 4U + (ew >> 16) : (ew >> 16) | ((ew & 0xffffU) << 16);
      }
      s_edges[i] = w;
    }
  }
  if (tid == 0) {
    s_red[30] = 0; /* block_hard_decision's flag */
  }
  if constexpr (SPLIT_U4 > 0) {
    uint4*       st = reinterpret_cast<uint4*>(smem + lay.c2v);
    const uint4* gs = reinterpret_cast<const uint4*>(crc_tables + lay.split_tab);
#pragma unroll
    for (int u = 0; u < SPLIT_PER; ++u) {
      const int i = tid + u * nthr;
      if (i < SPLIT_U4) {
        st[i] = stv[u];
      }
    }
    for (int i = tid + SPLIT_PER * nthr; i < SPLIT_U4; i += nthr) { /* narrower workgroups only */
      st[i] = gs[i];
    }
  }
  if (vec16) {
    uint4* s4 = reinterpret_cast<uint4*>(s_soft);
    while (true) {
#pragma unroll
      for (int u = 0; u < PRO_U; ++u) {
        const int i = base4 + tid + u * nthr;
        if (i >= t4) {
          continue;
        }
        uint4 v = pv[u];
        if (i >= z4 && i < z4 + l4) {
          const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 3; q >= 0; --q) {
            if (wv[q] != 0) {
              const int hi = 31 - __builtin_clz(wv[q]); /* highest set bit -> byte index */
              last_local   = max(last_local, (i - z4) * 16 + q * 4 + hi / 8 + 1);
              break;
            }
          }
          v = make_uint4(clamp_inf4(v.x), clamp_inf4(v.y), clamp_inf4(v.z), clamp_inf4(v.w));
        }
        if constexpr (F16) { /* 16 LLRs -> 32 bytes */
          const uint2 a = soft_f16x4(v.x), b = soft_f16x4(v.y), c = soft_f16x4(v.z), e = soft_f16x4(v.w);
          s4[2 * i]     = make_uint4(a.x, a.y, b.x, b.y);
          s4[2 * i + 1] = make_uint4(c.x, c.y, e.x, e.y);
        } else if constexpr (SPEC && spec::SOFT_COPIES == 4) {
          /* the two copies the specialised decoder reads (column offsets Z and 2Z); Z % 16 == 0 */
          const int col = (16 * i) / Z, o = 16 * i - col * Z;
          uint4*    c4  = reinterpret_cast<uint4*>(s_soft + col * static_cast<int>(lay.soft_stride) + Z + o);
          c4[0]         = v;
          c4[Z / 16]    = v;
        } else {
          s4[i] = v;
        }
      }
      base4 += PRO_U * nthr;
      if (base4 >= t4) {
        break;
      }
#pragma unroll
      for (int u = 0; u < PRO_U; ++u) { /* the next pass's loads (blocks narrower than t4 / PRO_U threads) */
        const int i = base4 + tid + u * nthr;
        pv[u]       = (i >= z4 && i < z4 + l4 && i < t4) ? g4[i - z4] : make_uint4(0, 0, 0, 0);
      }
    }
  } else if (!(SPEC && spec::SOFT_COPIES == 4) && (reinterpret_cast<uintptr_t>(llr) & 15U) == 0) {
    /* 16-byte loads whatever the alignment of 2Z and L (Z % 8 != 0, e.g. BG2 Z=36, or shortened lengths): the chunks
     * land at soft + 2Z + 16 k through 4-byte (Z even) or 2-byte LDS writes, the last L % 16 LLRs by byte loads, and
     * a thread issues all its loads of a pass (and the tail's) before storing any. A loop of byte loads instead paid
     * one memory round trip per trip (BG2 Z=36, 128 threads: 15 trips, a 22 us prologue from pinned host memory). */
    const int lc = L >> 4, lt = L & 15;
    int8_t    tv = 0;
    if (tid < lt) {
      tv = llr[16 * lc + tid];
    }
    for (int i = tid; i < 2 * Z; i += nthr) {
      if constexpr (F16) {
        s_soft16[i] = 0;
      } else {
        s_soft[i] = 0;
      }
    }
    for (int i = 2 * Z + L + tid; i < total; i += nthr) {
      if constexpr (F16) {
        s_soft16[i] = 0;
      } else {
        s_soft[i] = 0;
      }
    }
    for (int c0 = 0; c0 < lc; c0 += PRO_U * nthr) {
      uint4 w[PRO_U];
#pragma unroll
      for (int u = 0; u < PRO_U; ++u) {
        const int k = c0 + tid + u * nthr;
        w[u]        = k < lc ? g4[k] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < PRO_U; ++u) {
        const int k = c0 + tid + u * nthr;
        if (k >= lc) {
          continue;
        }
        const uint32_t wv[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
        for (int q = 3; q >= 0; --q) {
          if (wv[q] != 0) {
            const int hi = 31 - __builtin_clz(wv[q]);
            last_local   = max(last_local, k * 16 + q * 4 + hi / 8 + 1);
            break;
          }
        }
        int8_t* dst = s_soft + 2 * Z + 16 * k;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t c = clamp_inf4(wv[q]);
          if constexpr (F16) { /* element 2Z + 16 k + 4 q: byte 4 Z + 32 k + 8 q, 4-byte aligned */
            const uint2 h                                      = soft_f16x4(c);
            reinterpret_cast<uint32_t*>(s_soft16 + 2 * Z + 16 * k)[2 * q]     = h.x;
            reinterpret_cast<uint32_t*>(s_soft16 + 2 * Z + 16 * k)[2 * q + 1] = h.y;
          } else if ((Z & 1) == 0) {
            reinterpret_cast<uint32_t*>(dst)[q] = c;
          } else {
            reinterpret_cast<uint16_t*>(dst)[2 * q]     = static_cast<uint16_t>(c);
            reinterpret_cast<uint16_t*>(dst)[2 * q + 1] = static_cast<uint16_t>(c >> 16);
          }
        }
      }
    }
    if (tid < lt) {
      const int li = 16 * lc + tid;
      if (tv != 0) {
        last_local = max(last_local, li + 1);
      }
      if constexpr (F16) {
        s_soft16[2 * Z + li] = soft_f16(med3i(tv, -LLR_INTERNAL_INF, LLR_INTERNAL_INF));
      } else {
        s_soft[2 * Z + li] = static_cast<int8_t>(med3i(tv, -LLR_INTERNAL_INF, LLR_INTERNAL_INF));
      }
    }
  } else {
    for (int i = tid; i < total; i += nthr) {
      int8_t    v  = 0;
      const int li = i - 2 * Z;
      if (li >= 0 && li < L) {
        v = llr[li];
        if (v != 0) {
          last_local = max(last_local, li + 1);
        }
        v = static_cast<int8_t>(med3i(v, -LLR_INTERNAL_INF, LLR_INTERNAL_INF));
      }
      if constexpr (F16) {
        s_soft16[i] = soft_f16(v);
      } else if constexpr (SPEC && spec::SOFT_COPIES == 4) {
        const int col = i / Z, o = i - col * Z;
        s_soft[col * static_cast<int>(lay.soft_stride) + Z + o]     = v;
        s_soft[col * static_cast<int>(lay.soft_stride) + 2 * Z + o] = v;
      } else {
        s_soft[i] = v;
      }
    }
  }
  CB_STAMP(7); /* diagnostic build: the soft bits' loads have returned and are stored */
  if (crc_on) {
    uint4* s4 = reinterpret_cast<uint4*>(s_crct);
#pragma unroll
    for (int u = 0; u < CRC_PER; ++u) {
      const int j = tid + u * nthr;
      if (j < CRC_U4) {
        s4[j] = crcv[u];
      }
    }
    for (int j = tid + CRC_PER * nthr; j < CRC_U4; j += nthr) { /* workgroups of fewer than 108 threads */
      s4[j] = crc_chunk(j);
    }
  }
  {
    const int wl = wave_max(last_local);
    if (lane == 0) {
      s_red[wave] = static_cast<uint32_t>(wl);
    }
  }
  __syncthreads();
  CB_STAMP(1);
  /* lane i reads wave i's maximum (one LDS read per lane), then a wave maximum: uniform */
  const int last = wave_max(lane < (nthr + 63) / 64 ? static_cast<int>(s_red[lane]) : 0);
  const int nb   = (KZ + 7) / 8;
  const int Lsig = KZ - static_cast<int>(d.nof_filler_bits);

  int  has_value  = 0;
  int  iterations = d.max_iterations;
  bool write_out  = true;

  if (last == 0) {
    /* All-zero LLRs (impl.cpp:86-94): no CRC -> message of ones; with a CRC -> untouched, nullopt. */
    if (d.crc_mode == LDPC_HIP_CRC_MODE_EARLY_STOP) {
      write_out = false;
    } else {
      for (int b = tid; b < nb; b += nthr) {
        const int nbits = min(8, KZ - 8 * b);
        s_hb[b]         = static_cast<uint8_t>((0xff00U >> nbits) & 0xffU);
      }
      __syncthreads();
      if (d.crc_mode == LDPC_HIP_CRC_MODE_CHECK_AFTER) {
        has_value = (block_crc(s_hb, Lsig, d.crc_poly, s_crct,
                               s_red, crc_tables + CRC_MCOL_OFFSET + d.crc_poly * CRC_MCOL_WORDS) == 0);
      }
    }
  } else {
    /* Codeblock length and number of layers (impl.cpp:103-114). */
    int cb_len = max(last + 2 * Z, (K + 4) * Z);
    cb_len     = ((cb_len + Z - 1) / Z) * Z;
    const int nof_layers = cb_len / Z - K;
    const int half  = lane >> 5;
    const int trash = N_full * Z; /* scratch bytes after the soft bits take the dummy-edge stores */
    /* steps whose first row is a layer beyond nof_layers are skipped; a step's own rows are checked per task */
    int n_steps = 0; /* generic body only */
    if constexpr (!SPEC) {
      n_steps = graph->n_steps;
      for (int s = 0; s < n_steps; ++s) {
        if (graph->step_row0[s] >= nof_layers) {
          n_steps = s;
          break;
        }
      }
    }
    /* This wave's task of step s is the step_task at tasks[s * tw + wave]. It is fetched one step ahead, lane i
     * loading word i (a vector load, so the step barrier does not wait for it), and read out with v_readlane. */
    const int        tw   = SPEC ? 1 : graph_field_task_waves(graph_slot);
    const bool       idle = wave >= tw; /* wider workgroup than the schedule (mixed launch): barriers only */
    const step_task* tk   = tasks + (idle ? 0 : wave); /* this wave's task of step s: tk[s * tw] (scalar loads) */

    bool     hb_current = false;
#ifdef LDPC_HIP_DIAG
    int diag_n = 1;
    if (blockIdx.x == 0 && tid == 0) {
      g_diag[0] = __builtin_amdgcn_s_memtime();
    }
#endif
    step_task nxt = tk[0]; /* fetched one step ahead: the scalar load overlaps the previous step's row update */
    typename SD::cr_t cr; /* specialised kernel: this lane's c2v bytes, all zero = not yet initialised */
    for (auto& q : cr) {
      q = 0;
    }
    sp::lanes sl{};
    if constexpr (!QUAD && !REG) {
      sl = SD::template make_lanes<SPEC>(wave, lane, __builtin_amdgcn_readfirstlane(nof_layers),
                                        lay.c2v + 4U * static_cast<uint32_t>(tid));
    }
    typename SD::pf_t pf = {0, 0, 0, 0, 0};
    if constexpr (SPEC && !QUAD && !REG) {
      SD::template load_pf<0>(pf, sl);
    }
    using RD = sp::rdec<SG::g, SG::r>;
    uint32_t rsv[REG ? SG::g.N_full : 1]; /* register-resident decoder: the columns' registers */
    uint32_t rcr[REG ? SG::r.n_pairs : 1]; /* ... and the c2v pairs */
    for (auto& q : rcr) {
      q = 0;
    }
    auto rl = [&] {
      if constexpr (REG) {
        return RD::make_lanes(lane, __builtin_amdgcn_readfirstlane(nof_layers));
      } else {
        return 0;
      }
    }();
    uint32_t rec[REG ? SG::g.K : 1]; /* register-resident decoder: the early-stop CRC terms (RD::et_setup) */
    if constexpr (REG) {
      RD::load(rsv, lane);
      if (d.crc_mode == LDPC_HIP_CRC_MODE_EARLY_STOP) {
        RD::et_setup(rec, lane, Lsig, d.crc_poly == LDPC_HIP_CRC16 ? 16 : 24,
                     crc_tables + CRC_XPOW_OFFSET + d.crc_poly * CRC_XPOW_WORDS);
      }
    }
    uint32_t qcr[QN]; /* lane-split decoder: this lane's c2v pairs */
    for (auto& q : qcr) {
      q = 0;
    }
    const auto ql = [&] {
      if constexpr (QUAD) {
        return QD::make_lanes(wave, lane, __builtin_amdgcn_readfirstlane(nof_layers));
      } else {
        return 0;
      }
    }();
    /* the iteration loop; with a partial form (few-layer codeblocks: dec::iteration_partial) in two copies, the
     * branch between them taken once per codeblock, outside the loop */
    CB_STAMP(2);
    auto run_iterations = [&](auto partial) __attribute__((always_inline)) {
    for (int it = 0; it < d.max_iterations; ++it) {
      if constexpr (QUAD) {
        QD::iteration(qcr, qtab, ql);
      } else if constexpr (SPEC) {
        if constexpr (decltype(partial)::value) {
          SD::iteration_partial(cr, sl);
        } else {
          SD::iteration(cr, sl, pf);
        }
      }
      for (int g = 0; g < (SPEC ? 0 : n_steps); ++g) {
#ifdef LDPC_HIP_DIAG
        if (blockIdx.x == 0 && lane == 0 && it == d.max_iterations - 1) {
          g_diag2[(g * 16 + wave) * 2] = __builtin_amdgcn_s_memtime();
        }
#endif
        uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        PHASE(7);
        const step_task cur = nxt;
        nxt                 = tk[(g + 1 < n_steps ? g + 1 : 0) * tw];
        const uint32_t  h   = cur.w[0];
        const int      row = static_cast<int>((h >> 8) & 0xffU);
        if ((h & 64U) != 0U && row < nof_layers && !idle) {
          const int deg     = static_cast<int>(h & 31U);
          const int t0      = static_cast<int>(h >> 16);
          int8_t*         c2v_row = s_c2v + cur.w[1];
          const uint32_t* s_slot  = reinterpret_cast<const uint32_t*>(smem + cur.w[2]);
          if ((h & 32U) != 0U) {
            const int t = t0 + (lane & 31);
            if (t < Z) {
#ifndef LDPC_HIP_DIAG_SKIP
              row_dispatch<2, SF08>(deg, t, half, s_slot + (half ? (deg + 1) / 2 : 0), s_soft, c2v_row, sf, Z,
                                   trash, ph);
#endif
            }
          } else {
            const int t = t0 + lane;
            if (t < Z) {
#ifndef LDPC_HIP_DIAG_SKIP
              row_dispatch<1, SF08>(deg, t, 0, s_slot, s_soft, c2v_row, sf, Z, trash, ph);
#endif
            }
          }
        }
#ifdef LDPC_HIP_DIAG_PHASE
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PHASE(5);
        __syncthreads();
        PHASE(6);
        if (blockIdx.x == 0 && lane == 0 && it == d.max_iterations - 1) {
          for (int q = 0; q < 8; ++q) {
            g_diag2[(g * 16 + wave) * 8 + q] = ph[q];
          }
        }
#endif
#ifdef LDPC_HIP_DIAG
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (blockIdx.x == 0 && lane == 0 && it == d.max_iterations - 1) {
          g_diag2[(g * 16 + wave) * 2 + 1] = __builtin_amdgcn_s_memtime();
        }
#endif
        __syncthreads();
#ifdef LDPC_HIP_DIAG
        if (blockIdx.x == 0 && tid == 0 && diag_n < 4000) {
          g_diag[diag_n++] = __builtin_amdgcn_s_memtime();
        }
#endif
      }
      hb_current = false;
      if (d.crc_mode == LDPC_HIP_CRC_MODE_EARLY_STOP) {
        bool ok;
        if constexpr (F16) {
          ok = block_hard_decision16(s_soft, s_hb, KZ, &s_red[30], static_cast<uint32_t>(it) + 1U);
        } else {
          ok = block_hard_decision<SPEC ? SG::g.Z : 0>(s_soft, s_hb, KZ, &s_red[30], static_cast<uint32_t>(it) + 1U, Z,
                                                       SPEC ? static_cast<int>(lay.soft_stride) : 0,
                                                       static_cast<int>(lay.soft_read));
        }
        hb_current    = true;
        if (ok && block_crc(s_hb, Lsig, d.crc_poly, s_crct,
                            s_red, crc_tables + CRC_MCOL_OFFSET + d.crc_poly * CRC_MCOL_WORDS) == 0) {
          has_value  = 1;
          iterations = it + 1;
          break;
        }
      }
    }
    };
    /* The register-resident decoder's loop: two copies, full-length codeblocks without the layer checks. The early
     * stop ends it through the loop condition */
    auto reg_loop = [&](auto partial) __attribute__((always_inline)) {
      /* uniform by construction (the descriptor may come through vector loads): a divergent loop exit makes the
       * compiler keep every loop-carried register twice */
      int        n  = __builtin_amdgcn_readfirstlane(static_cast<int>(d.max_iterations));
      const bool et = __builtin_amdgcn_readfirstlane(static_cast<int>(d.crc_mode)) == LDPC_HIP_CRC_MODE_EARLY_STOP;
      for (int it = 0; it < n && REG; ++it) {
        if constexpr (REG) {
          if constexpr (decltype(partial)::value) {
            RD::iteration_partial(rsv, rcr, rl);
          } else {
            RD::iteration(rsv, rcr, rl);
          }
          if (et && RD::et_check(rsv, rec, lane)) {
            has_value  = 1;
            iterations = it + 1;
            n          = it + 1;
          }
        }
      }
    };
    if constexpr (REG) {
      if (nof_layers < SG::g.M) {
        reg_loop(std::true_type{});
      } else {
        reg_loop(std::false_type{});
      }
    } else if constexpr (SPEC && !QUAD && !REG && SD::HAS_PARTIAL) {
      if (__builtin_expect(nof_layers <= SD::PARTIAL_LAYERS, 0)) {
        run_iterations(std::true_type{});
      } else {
        run_iterations(std::false_type{});
      }
    } else {
      run_iterations(std::false_type{});
    }
    CB_STAMP(3);
    if (!hb_current) {
      if constexpr (REG) {
        RD::store_systematic(rsv, lane);
        __syncthreads();
      }
      if constexpr (F16) {
        block_hard_decision16(s_soft, s_hb, KZ, &s_red[30], 0xffffffffU);
      } else {
        block_hard_decision<SPEC ? SG::g.Z : 0>(s_soft, s_hb, KZ, &s_red[30], 0xffffffffU, Z,
                                                SPEC ? static_cast<int>(lay.soft_stride) : 0,
                                                static_cast<int>(lay.soft_read));
      }
    }
    if (d.crc_mode == LDPC_HIP_CRC_MODE_CHECK_AFTER) {
      has_value = (block_crc(s_hb, Lsig, d.crc_poly, s_crct,
                             s_red, crc_tables + CRC_MCOL_OFFSET + d.crc_poly * CRC_MCOL_WORDS) == 0);
    }
  }

  CB_STAMP(4);
  if (write_out) {
    for (int b = tid; b < nb; b += nthr) {
      out[b] = s_hb[b];
    }
  }
  if (tid == 0 && res_base != nullptr) {
    ldpc_hip_cb_result r;
    r.crc_pass               = static_cast<uint8_t>(has_value);
    r.nof_iterations         = static_cast<uint8_t>(iterations);
    r.status                 = write_out ? LDPC_HIP_STATUS_OUTPUT_WRITTEN : 0;
    res_base[d.result_index] = r;
  }
  CB_STAMP(5);
#undef CB_STAMP
#undef graph
}

/* threads per workgroup at most: the generic body 16 waves, a specialised one 12 (up to 168 VGPRs), the
 * register-resident decoder one wave (up to 256 VGPRs) */
template <int SPEC_ID>
constexpr int decode_max_threads()
{
  if constexpr (SPEC_ID < 0) {
    return 1024;
  } else {
    return spec::is_reg(spec::spec_graph<SPEC_ID>::g) ? 64 : 768;
  }
}

template <bool SF08, int SPEC_ID>
__global__ void __launch_bounds__(decode_max_threads<SPEC_ID>())
    ldpc_decode_kernel(const dec_cb* __restrict__ cbs, dec_cb one, int graph_slot, const step_task* __restrict__ tasks,
                       lds_layout lay, const int8_t* llr_base, uint8_t* __restrict__ out_base,
                       ldpc_hip_cb_result* __restrict__ res_base, const uint32_t* __restrict__ crc_tables,
                       const dematch_cb* dm_cbs, dematch_cb dm_one)
{
  /* cbs == nullptr: a one-CB launch whose descriptor came by value in the kernel arguments (no dependent load from
   * the descriptor table before the first LLR load; the HAL's zero-copy tables are in host memory).
   * llr_base is not __restrict__: with the fused dematcher (dm_cbs / dm_one) the workgroup first writes the soft
   * buffer it then reads through llr_base, through the dematch descriptor's pointer. */
  decode_cb<SF08, SPEC_ID>(cbs != nullptr ? cbs[blockIdx.x] : one, graph_slot, tasks, lay, llr_base, out_base, res_base,
                           crc_tables, dm_cbs, dm_one);
}

/* ---- device work queue: the persistent loop of a unit's grid (ldpc_hip_dwq.cpp) ------------------------------------
 * Wave 0 of a workgroup polls the ring slot of the next ticket, `next` (its view of the device claim counter): one
 * round trip reads the slot's 48 words (lanes 0-47) and the host's stop word (lane 48) from pinned memory. A slot whose
 * three sequence words equal next + 1 holds a published item; lane 0 claims it with a device-scope CAS of the claim
 * counter (next -> next + 1), and the item, already in registers, goes to LDS. A failed CAS returns the counter's
 * value, which becomes `next` (another workgroup claimed it). Only published items are ever claimed, so a workgroup
 * that leaves never strands one. Idle workgroups poll in turns (workgroup b in the 0.25 us slots where
 * (t / slot) mod grid = b: one slot read per 0.25 us for the grid); a workgroup that has just finished an item polls
 * twice at once, and one that lost a claim polls again at once, so back-to-back work does not wait for a turn
 * (polling freely for 20 us after seeing work, measured in round 4, cost more PCIe and host-cache traffic than it
 * saved, profiles/r04/route_ab_eager_v1.json). The body runs (fused
 * dematch + specialised decode, or a dematch alone), every wave drains its stores, and after a barrier lane 0 makes the
 * workgroup's writes visible system-wide (release fence: the HARQ soft bits in HBM for the next transmission's
 * workgroup on any XCD, the results in pinned host memory) and stores the done flag. Every wave leaves the loop
 * together: after idle_ticks without work, after life_ticks in all, or on stop; the host relaunches a grid when it
 * finds work unclaimed and the grid gone (ldpc_hip_dwq.cpp). Every spin is bounded. */
constexpr uint32_t DWQ_NONE = 0xffffffffU;
template <class BODY>
__device__ __forceinline__ void dwq_loop(const dwq_args& a, BODY&& body)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  /* control words: [0] claimed ticket, [1] stop, [2] ticks from t0 to the claim, [3] / [4] t0; the item from [8] */
  uint32_t* s_ctl  = reinterpret_cast<uint32_t*>(smem + a.ctl_lds);
  uint32_t* s_item = s_ctl + 8;
  const int tid    = threadIdx.x;
  const int lane   = tid & 63;
  uint64_t  t0     = __builtin_amdgcn_s_memrealtime();
  uint64_t  last   = t0;
  uint32_t  next   = 0; /* wave 0: the next ticket to poll */
  uint32_t  quick  = 0; /* wave 0: polls left outside the turns (the first ones after an item) */
  if (tid == 0) {
    s_ctl[3] = static_cast<uint32_t>(t0);
    s_ctl[4] = static_cast<uint32_t>(t0 >> 32);
  }
  if (tid < 64) {
    next = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(
        __hip_atomic_load(a.dev_ctl + DWQ_D_CLAIMED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))));
  }
#ifdef LDPC_HIP_DIAG_DWQ /* diagnostic build: lane 0's 100 MHz stamps of each item, into dead words of its slot */
  uint64_t t_claim = 0;
#endif
  while (true) {
    if (tid < 64) {
      uint32_t       claim = DWQ_NONE, stop = 0;
      const uint64_t tin   = __builtin_amdgcn_s_memrealtime();
      while (claim == DWQ_NONE && stop == 0U) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (now - tin > 1000U) { /* 10 us: back to the idle / lifetime checks */
          break;
        }
        if (quick == 0U) {
          const uint32_t slot = static_cast<uint32_t>(now / a.slot_ticks);
          const uint32_t ahead = (blockIdx.x + gridDim.x - slot % gridDim.x) % gridDim.x; /* slots to this turn */
          if (ahead != 0U) {
            if ((a.poll_flags & DWQ_POLL_LONG_SLEEP) != 0U && ahead * a.slot_ticks > 100U) {
              __builtin_amdgcn_s_sleep(32); /* ~2,048 cycles, ~0.85 us at 2.4 GHz */
            } else {
              __builtin_amdgcn_s_sleep(2);
            }
            continue;
          }
        }
        quick = quick != 0U ? quick - 1U : 0U;
        const uint32_t* sw = a.ring + (next & a.ring_mask) * DWQ_WIRE_WORDS;
        uint32_t        w  = 0;
        if (lane < static_cast<int>(DWQ_WIRE_WORDS)) {
          w = __hip_atomic_load(sw + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else if (lane == static_cast<int>(DWQ_WIRE_WORDS)) {
          w = __hip_atomic_load(a.host_ctl + DWQ_H_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        auto lane_word = [&](int l) {
          return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(w), l));
        };
        stop                = lane_word(DWQ_WIRE_WORDS);
        if (stop != 0U || (a.poll_flags & DWQ_POLL_TEST_NO_CLAIM) != 0U) {
          /* a stopped grid claims nothing more (a timed-out wait on the host stops it and then takes its exit as the
           * point after which no item of the queue can touch the caller's buffers, dwq_wait) */
          continue;
        }
        const uint32_t want = next + 1U;
        /* the checksum of payload words 0-43 (lane l carries payload word l - l / 16) against word 44 (lane 46) */
        const int      pw   = lane - (lane >> 4);
        const uint32_t mx   = (lane < static_cast<int>(DWQ_WIRE_WORDS) && (lane & 15) != 15 && pw < 44)
                                  ? dwq_mix(w, static_cast<uint32_t>(pw)) : 0U;
        const uint32_t sum  = wave_xor(mx);
        if (lane_word(15) == want && lane_word(31) == want && lane_word(47) == want && sum == lane_word(46)) {
          uint32_t exp = next;
          uint32_t ok  = 0;
          if (lane == 0) {
            /* relaxed: the item is already in registers (validated by its sequence words), the previous item's
             * writes were released with its done flag, and the acquire for the HARQ memory follows the claim; an
             * acq_rel CAS wrote back and invalidated the L2 around it on every claim */
            ok = __hip_atomic_compare_exchange_strong(a.dev_ctl + DWQ_D_CLAIMED, &exp, next + 1U, __ATOMIC_RELAXED,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     ? 1U
                     : 0U;
          }
          ok  = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(ok)));
          exp = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(exp)));
          if (ok != 0U) {
            claim = next;
            next  = next + 1U;
            if (lane < static_cast<int>(DWQ_WIRE_WORDS) && (lane & 15) != 15) {
              s_item[lane - (lane >> 4)] = w;
            } else if (lane >= 61) {
              s_item[DWQ_WIRE_PAYLOAD + (lane - 61)] = 0; /* pad[1..3] */
            }
          } else {
            next  = exp; /* another workgroup claimed it: poll the counter's next ticket at once */
            quick = quick != 0U ? quick : 1U;
          }
          continue;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (claim != DWQ_NONE) {
        /* the HARQ soft bits an earlier item left in HBM, possibly from another XCD's L2, and the host's new inputs
         * in pinned staging this CU's vector cache may hold from an earlier item (a timing variant without this
         * acquire decoded stale LLRs) */
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
#ifdef LDPC_HIP_DIAG_DWQ
      t_claim = now;
#endif
      if (lane == 0) {
        s_ctl[0] = claim;
        s_ctl[1] = stop;
        s_ctl[2] = static_cast<uint32_t>(now - t0);
      }
    }
    __syncthreads();
    const uint32_t claim   = s_ctl[0];
    const uint32_t stop    = s_ctl[1];
    const uint64_t elapsed = s_ctl[2];
    if (claim == DWQ_NONE) {
      __syncthreads(); /* every wave has read the control words before wave 0 writes them again */
      if (stop != 0U || elapsed - (last - t0) > a.idle_ticks || elapsed > a.life_ticks) {
        break;
      }
      continue;
    }
    /* The item's words go to scalar registers (the launched kernel's descriptor comes from the kernel arguments into
     * SGPRs as well): a vector-register copy lived across the body and made the BG1 bodies spill. Nothing of the loop
     * lives in registers across the body: its state is rebuilt from the control words after it. */
    uint32_t words[DWQ_ITEM_WORDS];
    for (uint32_t k = 0; k != DWQ_ITEM_WORDS; ++k) {
      words[k] = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(s_item[k])));
    }
    /* memcpy, not stores through a uint32_t* into the struct: its 64-, 16- and 8-bit fields read back after such
     * stores are not ordered after them under type-based alias analysis (a loop-carried `it` then handed the body some
     * fields of the workgroup's previous item: wrong decodes of successive calls with different lengths) */
    dwq_item it;
    __builtin_memcpy(&it, words, sizeof(it));
#ifdef LDPC_HIP_DIAG_DWQ
    const uint64_t t_item = __builtin_amdgcn_s_memrealtime();
#endif
    if (it.spec != DWQ_SPEC_NOOP) {
      body(it);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t done_claim = s_ctl[0];
    t0    = (static_cast<uint64_t>(s_ctl[4]) << 32) | s_ctl[3];
    last  = t0 + s_ctl[2];
    next  = done_claim + 1U;
    quick = 2U; /* a workgroup done with an item looks at the next ticket at once (back-to-back work), twice */
    if (tid == 0) {
#ifdef LDPC_HIP_DIAG_DWQ
      uint32_t* pw = const_cast<uint32_t*>(a.ring + (claim & a.ring_mask) * DWQ_WIRE_WORDS);
      pw[44]       = static_cast<uint32_t>(t_claim);
      pw[45]       = static_cast<uint32_t>(t_item - t_claim);
      pw[46]       = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime() - t_claim);
      pw[14]       = blockIdx.x;
#endif
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(a.done + (done_claim & a.ring_mask), done_claim + 1U, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  /* the grid's last workgroup to leave tells the host (ldpc_hip_dwq.cpp ensure_running: no runtime query per submit) */
  if (tid == 0) {
    const uint32_t n = __hip_atomic_fetch_add(a.dev_ctl + DWQ_D_EXITS, 1U, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n + 1U == a.exit_target) {
      __hip_atomic_store(a.host_exit, a.exit_target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

/* The work-queue kernels: one per specialised graph (its fused dematch + decode body only) and one for dematch-only
 * items, so each has the register allocation of its own body. Round 4 first had one kernel per translation unit that
 * dispatched on it.spec among the unit's 4-10 bodies: the union spilled 24-137 VGPRs to scratch and 189-518 SGPRs
 * (the launched kernels of the same bodies spill none), and its bodies ran up to 1.5x slower than launched ones. */
template <int SPEC_ID>
__global__ void __launch_bounds__(decode_max_threads<SPEC_ID>()) ldpc_dwq_decode_kernel(dwq_args a)
{
  dwq_loop(a, [&](const dwq_item& it) __attribute__((always_inline)) {
    decode_cb<true, SPEC_ID>(it.cb, 0, nullptr, it.lay, it.llr_base, it.out_base, it.res_base, it.crc_tables, nullptr,
                             it.dm);
  });
}

/* Diagnostic build (LDPC_HIP_DIAG): each specialised-kernel unit has its own static g_diag2 (the stamps of its
 * kernels), read by ldpc_hip_diag2_read_<unit> (tools/diag_timeline.py); nothing in other builds. */
#if defined(LDPC_HIP_DIAG)
#define LDPC_DIAG_UNIT_READER(u)                                                                                       \
  extern "C" int ldpc_hip_diag2_read_##u(uint64_t* out, uint32_t n)                                                  \
  {                                                                                                                    \
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag2), n * sizeof(uint64_t)) == hipSuccess ? 0 : -2;               \
  }
#else
#define LDPC_DIAG_UNIT_READER(u)
#endif

/* dwq_kernel_<unit>(id): the work-queue kernel of specialised graph id of the unit's list, nullptr for other ids */
#define LDPC_DWQ_KERNEL_CASE(id, bg, z, ils)                                                                           \
  case id: return reinterpret_cast<const void*>(&ldpc_dwq_decode_kernel<id>);
#define LDPC_DWQ_KERNELS(NAME, LIST)                                                                                   \
  const void* NAME(int id)                                                                                             \
  {                                                                                                                    \
    switch (id) {                                                                                                      \
      LIST(LDPC_DWQ_KERNEL_CASE)                                                                                       \
    default: return nullptr;                                                                                           \
    }                                                                                                                  \
  }

/* The split-row address table of specialised graph SPEC_ID into dst (dec::write_split_table), or for a one-wave graph
 * its lane-split decoder's address table (qdec::write_table): one workgroup of the decoder's width, launched once per
 * context (ldpc_hip_api.cpp write_split_tables). */
template <int SPEC_ID>
__global__ void __launch_bounds__(768) ldpc_split_table_kernel(uint32_t* __restrict__ dst)
{
  using SG = spec::spec_graph<SPEC_ID>;
  using SD = sp::dec<SG::g>;
  if constexpr (spec::is_reg(SG::g)) { /* the register-resident decoder has no table */
  } else if constexpr (spec::is_quad(SG::g)) { /* the lane-split decoder's address table (sp::qdec) */
    sp::qdec<SG::g, SG::q>::write_table(dst, static_cast<int>(threadIdx.x >> 6), static_cast<int>(threadIdx.x & 63),
                                        std::make_integer_sequence<int, SG::q.n_steps>{});
  } else if constexpr (SD::LDS_PAIRS > 0) {
    SD::write_split_table(dst, static_cast<int>(threadIdx.x >> 6), static_cast<int>(threadIdx.x & 63));
  }
}


} // namespace ldpc_hip
