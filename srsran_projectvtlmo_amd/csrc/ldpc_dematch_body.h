/*
 * Rate dematching (ldpc_rate_dematcher_impl.cpp:46-213) and the soft demodulation it can fuse
 * (demodulation_mapper_impl.cpp:78-106), as device functions: ldpc_rate_dematch_kernel and ldpc_demodulate_kernel
 * (ldpc_hip_kernels.hip) run them standalone, the decode kernels (ldpc_decode_body.h) as a fused first phase.
 * Included by ldpc_decode_body.h after its LLR helpers (llr_isinf, LLR_MAX, LLR_INF), in the same namespaces.
 */
#pragma once

namespace ldpc_hip {
namespace {

__device__ __forceinline__ int8_t dm_quantize(float v, float range)
{
#pragma clang fp contract(off)
  float c = v;
  if (fabsf(v) > range) {
    c = copysignf(range, v);
  }
  return static_cast<int8_t>(roundf(c / range * 120.0F));
}

__device__ __forceinline__ float dm_interval(float x, float rn, float width, int nof, const float* sl, const float* ic)
{
#pragma clang fp contract(off)
  /* static_cast<int>(std::floor(.)) as the reference's x86-64 build executes it: NaN / out of range -> INT_MIN
   * (cvttss2si), i.e. the first interval; a GPU conversion would saturate instead */
  const float q   = floorf(x / width);
  int         idx = (q >= -2147483648.0F && q < 2147483648.0F) ? static_cast<int>(q) : INT_MIN;
  idx             = max(idx, -nof) + nof / 2;
  idx             = min(max(idx, 0), nof - 1);
  float l = sl[idx] * x + ic[idx];
  l *= rn;
  return l;
}

__device__ __forceinline__ int8_t dm_bpsk(float re, float im, float nv)
{
#pragma clang fp contract(off)
  if (!(nv > 0)) {
    return 0;
  }
  const float gain = 2.0F * 1.41421356237309504880F;
  return dm_quantize(gain * (re + im) / nv, 24.0F);
}

__device__ __forceinline__ int8_t dm_qpsk(float x, float nv)
{
#pragma clang fp contract(off)
  if (!(nv > 0)) {
    return 0;
  }
  const float gain = 2.0F * 1.41421356237309504880F;
  return dm_quantize(gain * x / nv, 24.0F);
}

/* All Qm LLRs of one symbol, modulation known at compile time; the tables are in LDS (dynamic interval indices). */
template <int MOD>
__device__ __forceinline__ void dm_symbol(float2 z, float nv, uint32_t i, const demod_tables& tab, int8_t (&o)[8])
{
#pragma clang fp contract(off)
  if constexpr (MOD == 1) {
    o[0] = dm_bpsk(z.x, z.y, nv);
  } else if constexpr (MOD == 0) { /* odd-indexed symbols rotated: (im, -re) */
    o[0] = (i & 1U) ? dm_bpsk(z.y, -z.x, nv) : dm_bpsk(z.x, z.y, nv);
  } else if constexpr (MOD == 2) {
    o[0] = dm_qpsk(z.x, nv);
    o[1] = dm_qpsk(z.y, nv);
  } else {
    if (z.x * z.x + z.y * z.y < 1e-9F) { /* is_near_zero (math_utils.h:85-94) */
#pragma unroll
      for (int b = 0; b < MOD; ++b) {
        o[b] = 0;
      }
      return;
    }
    if constexpr (MOD == 4) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float x = c == 0 ? z.x : z.y;
        if (!(nv > 0)) {
          o[c]     = 0;
          o[2 + c] = 0;
          continue;
        }
        float l01 = 4 * tab.s10 * x;
        if (fabsf(x) > 2 * tab.s10) {
          l01 = 2 * l01 - copysignf(0.8F, x);
        }
        l01 /= nv;
        o[c]      = dm_quantize(l01, 24.0F);
        float l23 = 0.8F - 4 * tab.s10 * fabsf(x);
        l23 /= nv;
        o[2 + c] = dm_quantize(l23, 24.0F);
      }
    } else {
      const float rn = (nv > 0) ? 1 / nv : 0.0F;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float x = c == 0 ? z.x : z.y;
        if constexpr (MOD == 6) {
          o[c]     = dm_quantize(dm_interval(x, rn, tab.w64a, 8, tab.sl64[0], tab.ic64[0]), 20.0F);
          o[2 + c] = dm_quantize(dm_interval(x, rn, tab.w64a, 8, tab.sl64[1], tab.ic64[1]), 20.0F);
          o[4 + c] = dm_quantize(dm_interval(x, rn, tab.w64c, 4, tab.sl64[2], tab.ic64[2]), 20.0F);
        } else {
          o[c]     = dm_quantize(dm_interval(x, rn, tab.w256a, 16, tab.sl256[0], tab.ic256[0]), 20.0F);
          o[2 + c] = dm_quantize(dm_interval(x, rn, tab.w256a, 16, tab.sl256[1], tab.ic256[1]), 20.0F);
          o[4 + c] = dm_quantize(dm_interval(x, rn, tab.w256a, 16, tab.sl256[2], tab.ic256[2]), 20.0F);
          o[6 + c] = dm_quantize(dm_interval(x, rn, tab.w256c, 8, tab.sl256[3], tab.ic256[3]), 20.0F);
        }
      }
    }
  }
}

/* ldpc_rate_dematcher_impl::rate_dematch (ldpc_rate_dematcher_impl.cpp:46-213), one workgroup per codeblock.
 * The sequential allot loop (:128-201) is kept; each contiguous copy/combine/zero/fill range inside it runs across the
 * workgroup, with a barrier between passes over the circular buffer (a later pass combines into positions an earlier
 * pass wrote, and saturated sums do not associate). De-interleaving (:203-213) is fused as a gather: the CB's E LLRs
 * are first staged in LDS by 16-byte loads (E <= DM_STAGE; longer inputs are gathered from global memory), and each
 * thread steps its de-interleave index (e mod E/Qm) * Qm + e div E/Qm incrementally, one division per contiguous
 * range instead of one per LLR. */
/* Fused soft demodulation (ldpc_hip_demod_dematch_launch): symbol i of the CB gives LLRs [i * QM, (i + 1) * QM) */
template <int MOD>
__device__ __forceinline__ void dm_stage(const dematch_cb& d, unsigned nsym, const demod_tables& tab, int8_t* s_in,
                                         float2 z0, float nv0)
{
  constexpr int QM = (MOD <= 1) ? 1 : MOD;
  for (unsigned i = threadIdx.x; i < nsym; i += blockDim.x) {
    int8_t o[8];
    const bool first = i == threadIdx.x; /* the first symbol was loaded before the table barrier */
    dm_symbol<MOD>(first ? z0 : reinterpret_cast<const float2*>(d.sym)[i], first ? nv0 : d.nv[i], i, tab, o);
#pragma unroll
    for (int k = 0; k < QM; ++k) {
      s_in[i * QM + k] = o[k];
    }
  }
}

/* The dematcher's work for codeblock d: ldpc_rate_dematch_kernel's body, and the decode kernels' fused first phase
 * (ldpc_decode_body.h decode_cb, before the decoder prologue). s_in: DM_STAGE bytes of LDS staging; s_dtab: an LDS copy
 * of the demodulation tables (soft-demodulating form only). Uses the whole workgroup (any width); leaves the LDS and
 * the soft buffer written but issues no final barrier. */
__device__ __forceinline__ void dematch_body(const dematch_cb& d, const demod_tables& tab, int8_t* s_in,
                                             demod_tables& s_dtab)
{
#if defined(LDPC_HIP_DIAG_CB_DM) /* diagnostic build: the decoder's per-workgroup stamp slots 1-3 (decode_cb then skips
                                    * its own stamps 1-3), at the context's table buffer (tab sits at DTAB_OFFSET) */
#define DM_STAMP(k)                                                                                                    \
  if (threadIdx.x == 0 && blockIdx.x < 1024) {                                                                         \
    reinterpret_cast<uint64_t*>(const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(&tab) - DTAB_OFFSET) +       \
                                DIAG_CB_OFFSET)[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();             \
  }
#elif defined(LDPC_HIP_DIAG_DM) /* diagnostic build: device-wide 100 MHz stamps per workgroup (g_diag2[block * 8 + k]) */
#define DM_STAMP(k)                                                                                                    \
  if (threadIdx.x == 0 && blockIdx.x < 1024) {                                                                         \
    g_diag2[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                                                  \
  }
#else
#define DM_STAMP(k)
#endif
  const int        tid = threadIdx.x;
  const int        nth = blockDim.x;

  const unsigned N      = d.cb_length;
  const unsigned Ncb    = (d.Nref > 0) ? min(d.Nref, N) : N;
  const bool     is_bg1 = (N % 66U) == 0;
  const unsigned Z      = is_bg1 ? N / 66U : N / 50U;
  const unsigned bg_k   = is_bg1 ? 22U : 10U;
  const unsigned nsys   = (bg_k - 2U) * Z;
  const unsigned ninfo  = nsys - d.nof_filler_bits;
  const unsigned F      = d.nof_filler_bits;
  const unsigned E      = d.rm_length;
  const unsigned Qm     = d.modulation_order;
  const unsigned EQ     = E / Qm;
  /* k0 = floor(sf * Ncb / N) * Z (:104-105); sf * Ncb <= 56 * 25344 fits 32 bits exactly */
  const unsigned sfac   = is_bg1 ? (d.rv == 0 ? 0U : d.rv == 1 ? 17U : d.rv == 2 ? 33U : 56U)
                                 : (d.rv == 0 ? 0U : d.rv == 1 ? 13U : d.rv == 2 ? 25U : 43U);
  const unsigned k0     = ((sfac * Ncb) / N) * Z;

  int8_t*       out = d.soft;
  const int8_t* in  = d.llr;
  const bool    staged = E <= (d.stage_bytes != 0 ? d.stage_bytes : DM_STAGE);
  if (d.sym != nullptr) {
    /* demodulate straight into the staging buffer (the host guarantees E <= DM_STAGE); tables in LDS */
    constexpr int NW = static_cast<int>(sizeof(demod_tables) / 4);
    /* this thread's first symbol and noise variance, loaded before the table barrier (one memory round trip for both) */
    float2 z0  = make_float2(0.F, 0.F);
    float  nv0 = 0.F;
    if (static_cast<unsigned>(tid) < EQ) {
      z0  = reinterpret_cast<const float2*>(d.sym)[tid];
      nv0 = d.nv[tid];
    }
    for (int i = tid; i < NW; i += nth) {
      reinterpret_cast<uint32_t*>(&s_dtab)[i] = reinterpret_cast<const uint32_t*>(&tab)[i];
    }
    __syncthreads();
    switch (d.demod) { /* block-uniform */
      case 0: dm_stage<0>(d, EQ, s_dtab, s_in, z0, nv0); break;
      case 1: dm_stage<1>(d, EQ, s_dtab, s_in, z0, nv0); break;
      case 2: dm_stage<2>(d, EQ, s_dtab, s_in, z0, nv0); break;
      case 4: dm_stage<4>(d, EQ, s_dtab, s_in, z0, nv0); break;
      case 6: dm_stage<6>(d, EQ, s_dtab, s_in, z0, nv0); break;
      default: dm_stage<8>(d, EQ, s_dtab, s_in, z0, nv0); break;
    }
    __syncthreads();
    DM_STAMP(1);
  } else if (staged) {
    if ((reinterpret_cast<uintptr_t>(in) & 15U) == 0) {
      /* 16-byte loads, up to four in flight per thread, and the last E % 16 LLRs' byte loads issued with the first
       * pass: one memory round trip for a codeblock of up to 64 x nth bytes (the input may be pinned host memory) */
      const unsigned n16 = E / 16U, et = E - 16U * n16;
      const unsigned ut = static_cast<unsigned>(tid), un = static_cast<unsigned>(nth);
      int8_t         tb  = 0;
      if (ut < et) {
        tb = in[16U * n16 + ut];
      }
      for (unsigned i0 = ut; i0 < n16; i0 += 4U * un) {
        uint4 w[4];
#pragma unroll
        for (unsigned u = 0; u < 4; ++u) {
          const unsigned i = i0 + u * un;
          w[u]             = i < n16 ? reinterpret_cast<const uint4*>(in)[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (unsigned u = 0; u < 4; ++u) {
          const unsigned i = i0 + u * un;
          if (i < n16) {
            reinterpret_cast<uint4*>(s_in)[i] = w[u];
          }
        }
      }
      if (ut < et) {
        s_in[16U * n16 + ut] = tb;
      }
    } else {
      for (unsigned i = static_cast<unsigned>(tid); i < E; i += static_cast<unsigned>(nth)) {
        s_in[i] = in[i];
      }
    }
    __syncthreads();
    DM_STAMP(1);
  }
  const int8_t* src = (staged || d.sym != nullptr) ? static_cast<const int8_t*>(s_in) : in;
  auto sat_add = [](int a, int b) -> int8_t { /* log_likelihood_ratio::operator+ (llr.cpp:56-71) */
    if (a == -b) {
      return 0;
    }
    if (llr_isinf(a)) {
      return static_cast<int8_t>(a);
    }
    if (llr_isinf(b)) {
      return static_cast<int8_t>(b);
    }
    return static_cast<int8_t>(min(max(a + b, -LLR_MAX), LLR_MAX));
  };
  /* out[dst + i] = (or +=) the de-interleaved LLR e0 + i, i < n (deinterleave_bits_Qm, :203-213: LLR e of the
   * rate-matched order is input (e mod EQ) * Qm + e div EQ); q = e div EQ and r = e mod EQ advance by nth per step */
  /* DM_UNROLL elements per trip: every source read of the trip is issued before its stores, so a thread waits for
   * the LDS once per trip, not once per element */
  constexpr unsigned DM_UNROLL = 8;
  auto range = [&](unsigned dst, unsigned e0, unsigned n, bool combine) {
    if (static_cast<unsigned>(tid) >= n) {
      return;
    }
    const unsigned e  = e0 + static_cast<unsigned>(tid);
    unsigned       q  = e / EQ;
    unsigned       r  = e - q * EQ;
    const unsigned un = static_cast<unsigned>(nth);
    const unsigned dq = un / EQ;
    const unsigned dr = un - dq * EQ;
    auto next = [&]() {
      r += dr;
      q += dq;
      const bool wrap = r >= EQ;
      r               = wrap ? r - EQ : r;
      q += wrap ? 1U : 0U;
    };
    /* whole trips (every lane's DM_UNROLL elements in range, a uniform count): no per-element guards, so the trip is
     * straight-line code; a guarded element costs an exec-mask branch around its load and its store (round 6: a
     * one-codeblock HAL TB's de-interleave, two waves, was 2.1 us of mostly such branches) */
    const unsigned trips = n / (DM_UNROLL * un);
    unsigned       i     = static_cast<unsigned>(tid);
    for (unsigned t = 0; t < trips; ++t, i += DM_UNROLL * un) {
      int v[DM_UNROLL];
#pragma unroll
      for (unsigned k = 0; k < DM_UNROLL; ++k) {
        v[k] = src[r * Qm + q];
        next();
      }
      /* combining: the trip's old soft values are all loaded before any store (each position is written once per
       * range), so a trip waits for the soft buffer once, not once per element */
      if (combine) {
        int o[DM_UNROLL];
#pragma unroll
        for (unsigned k = 0; k < DM_UNROLL; ++k) {
          o[k] = out[dst + i + k * un];
        }
#pragma unroll
        for (unsigned k = 0; k < DM_UNROLL; ++k) {
          out[dst + i + k * un] = sat_add(o[k], v[k]);
        }
      } else {
#pragma unroll
        for (unsigned k = 0; k < DM_UNROLL; ++k) {
          out[dst + i + k * un] = static_cast<int8_t>(v[k]);
        }
      }
    }
    /* the rest (fewer than DM_UNROLL * nth elements): one element per loop trip */
    for (; i < n; i += un) {
      const int v = src[r * Qm + q];
      next();
      out[dst + i] = combine ? sat_add(out[dst + i], v) : static_cast<int8_t>(v);
    }
  };

  /* out[b, e) = 0: byte-wise up to a 16-byte boundary of the address, then 16-byte stores, then the tail */
  auto zero_fill = [&](unsigned b, unsigned e) {
    if (b >= e) {
      return;
    }
    const unsigned mis  = static_cast<unsigned>(reinterpret_cast<uintptr_t>(out + b) & 15U);
    const unsigned head = min(e - b, mis == 0 ? 0U : 16U - mis);
    const unsigned nv   = (e - b - head) / 16U;
    for (unsigned i = tid; i < head; i += nth) {
      out[b + i] = 0;
    }
    uint4* o4 = reinterpret_cast<uint4*>(out + b + head);
    for (unsigned i = tid; i < nv; i += nth) {
      o4[i] = make_uint4(0, 0, 0, 0);
    }
    for (unsigned i = b + head + 16U * nv + tid; i < e; i += nth) {
      out[i] = 0;
    }
  };

  bool     copy     = d.new_data != 0;
  unsigned tmp_idx  = k0;
  unsigned consumed = 0;
  unsigned left     = E;
  while (left != 0) {
    if (tmp_idx < ninfo) {
      const unsigned n = min(ninfo - tmp_idx, left);
      if (copy) {
        zero_fill(0, tmp_idx);
      }
      range(tmp_idx, consumed, n, !copy);
      tmp_idx += n;
      consumed += n;
      left -= n;
    } else if (copy) {
      zero_fill(0, ninfo);
    }
    if (copy) {
      for (unsigned i = tid; i < F; i += nth) {
        out[ninfo + i] = static_cast<int8_t>(LLR_INF);
      }
    }
    if (tmp_idx < nsys) {
      tmp_idx = nsys;
    }
    const unsigned np = min(Ncb - tmp_idx, left);
    range(tmp_idx, consumed, np, !copy);
    tmp_idx = (tmp_idx + np) % Ncb;
    consumed += np;
    left -= np;
    if (left != 0) {
      copy = false;
    }
    __syncthreads();
    DM_STAMP(2);
  }
  if (copy && tmp_idx != 0) {
    const unsigned cnt = Ncb - tmp_idx; /* out.last(buffer_length - tmp_idx) over the N-sized output (:197-200) */
    zero_fill(N - cnt, N);
  }
#if defined(LDPC_HIP_DIAG_DM) || defined(LDPC_HIP_DIAG_CB_DM)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  DM_STAMP(3);
#endif
#undef DM_STAMP
}

} // namespace
} // namespace ldpc_hip
