/*
 * gfx950 (MI355X, CDNA4) kernels of the 5G-NR PUSCH LDPC decode path.
 *
 *  ldpc_decode_kernel<MAXDEG>  layered normalised min-sum decoder, one workgroup per codeblock, the whole decoder
 *                              state resident in LDS (int8 soft bits + int8 check-to-variable messages; BG1 Z=384
 *                              uses 147 KiB of the 160 KiB). Bit-exact with ldpc_decoder_generic
 *                              (lib/phy/upper/channel_coding/ldpc/ldpc_decoder_impl.cpp:60-308,
 *                              ldpc_decoder_generic.cpp:30-128) including the CRC early stop.
 *  ldpc_rate_dematch_kernel    bit de-interleave + rate dematching + HARQ combining
 *                              (ldpc_rate_dematcher_impl.cpp:46-213), one workgroup per codeblock.
 *
 * Work mapping of the decoder. A base-graph row m lifts to Z independent check nodes t; one thread owns check node
 * (m, t) for the whole layer update, so the Zc cyclic shift is an LDS byte gather soft[col][(t + shift) mod Z] and
 * the two-minimum search runs over the row's edges in order inside one thread (strict '<', first edge wins, exactly
 * as the reference's sequential scan). check-to-variable messages are stored per (edge, t), i.e. in check-node
 * order; the value stored for (edge k, t) is the reference's c2v[m][slot][j] with j = (t + shift_k) mod Z, so the
 * relabelling changes no value. Consecutive rows that share no variable node are updated concurrently (one barrier
 * per row group): they read and write disjoint soft bits, so the result is identical to the layer-serial order.
 */
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ldpc_hip_device.h"

namespace ldpc_hip {

namespace {

constexpr int LLR_MAX = 120;
constexpr int LLR_INF = 127;

__device__ __forceinline__ bool llr_isinf(int v) { return v > LLR_MAX || v < -LLR_MAX; }

/* Wave-wide XOR reduction (wave64). */
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v ^= __shfl_xor(v, o, 64);
  }
  return v;
}

/* (a(x) * b(x)) mod G(x) over GF(2); a, b of degree < order; poly includes the x^order term. */
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b, int order, uint32_t poly)
{
  uint64_t prod = 0;
  for (int i = 0; i < order; ++i) {
    prod ^= ((b >> i) & 1U) ? (static_cast<uint64_t>(a) << i) : 0ULL;
  }
  for (int i = 2 * order - 2; i >= order; --i) {
    prod ^= ((prod >> i) & 1ULL) ? (static_cast<uint64_t>(poly) << (i - order)) : 0ULL;
  }
  return static_cast<uint32_t>(prod);
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
 * XOR_w [(W_w * x^r mod G) * (x^(32 (nw-1-w)) mod G) mod G]. Block-uniform result. */
__device__ uint32_t block_crc(const uint8_t* hb, int L, int poly_id, const uint32_t* s_table,
                              const uint32_t* __restrict__ g_pow, uint32_t* s_red)
{
  int      order;
  uint32_t poly;
  crc_params(poly_id, order, poly);
  const uint32_t mask = (order == 32) ? 0xffffffffU : ((1U << order) - 1U);
  const int      nw   = (L + 31) / 32;
  const int      p    = nw * 32 - L;
  uint32_t       acc  = 0;
  for (int w = threadIdx.x; w < nw; w += blockDim.x) {
    auto be = [&](int i) -> uint32_t {
      if (i < 0) {
        return 0U;
      }
      return (static_cast<uint32_t>(hb[4 * i]) << 24) | (static_cast<uint32_t>(hb[4 * i + 1]) << 16) |
             (static_cast<uint32_t>(hb[4 * i + 2]) << 8) | static_cast<uint32_t>(hb[4 * i + 3]);
    };
    const uint32_t W   = (p == 0) ? be(w) : ((be(w - 1) << (32 - p)) | (be(w) >> p));
    uint32_t       crc = 0;
#pragma unroll
    for (int b = 3; b >= 0; --b) {
      const uint32_t byte = (W >> (8 * b)) & 0xffU;
      crc                 = ((crc << 8) ^ s_table[((crc >> (order - 8)) ^ byte) & 0xffU]) & mask;
    }
    acc ^= gf2_mulmod(crc, g_pow[nw - 1 - w], order, poly);
  }
  acc              = wave_xor(acc);
  const int wave   = threadIdx.x >> 6;
  const int nwaves = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_red[wave] = acc;
  }
  __syncthreads();
  uint32_t r = 0;
  for (int i = 0; i < nwaves; ++i) {
    r ^= s_red[i];
  }
  return r;
}

/* hard_decision (log_likelihood_ratio.cpp:226-252) of soft[0, K*Z) into LDS packed bytes.
 * Returns true (block-uniform) iff no soft bit is zero. */
__device__ bool block_hard_decision(const int8_t* soft, uint8_t* hb, int KZ)
{
  const int nb   = (KZ + 7) / 8;
  int       zero = 0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    uint32_t  byte = 0;
    const int base = 8 * b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (base + i < KZ) {
        const int s = soft[base + i];
        byte |= static_cast<uint32_t>(s <= 0) << (7 - i);
        zero |= (s == 0);
      }
    }
    hb[b] = static_cast<uint8_t>(byte);
  }
  return __syncthreads_or(zero) == 0;
}

/* One lifted check node (row word rw, index t): variable-to-check update, two-minimum search and check-to-variable /
 * soft-bit update -- update_variable_to_check_messages, update_check_to_variable_messages and update_soft_bits
 * (ldpc_decoder_impl.cpp:176-308) restricted to the Z-lane t, with the generic kernels' arithmetic
 * (ldpc_decoder_generic.cpp:30-120). c2v is never infinite (|c2v| <= round(120 sf) <= 120), which reduces the LLR
 * special cases to: v2c = isinf(soft) ? soft : clamp(soft - c2v); soft' = isinf(v2c) ? v2c : promote(c2v + v2c). */
template <int MAXDEG>
__device__ __forceinline__ void check_node_update(int t, uint32_t rw, const uint32_t* s_edges, int8_t* s_soft,
                                                  int8_t* s_c2v, const int8_t* s_lut, int Z)
{
  const int e0  = static_cast<int>(rw & 0xffffU);
  const int deg = static_cast<int>(rw >> 16);
  int       v[MAXDEG];
  int       addr[MAXDEG];
  int       m1 = LLR_MAX, m2 = LLR_MAX, idx = 0, sg = 0;
#pragma unroll
  for (int k = 0; k < MAXDEG; ++k) {
    if (k < deg) {
      const uint32_t ew = s_edges[e0 + k];
      int            j  = t + static_cast<int>(ew >> 16);
      j                 = (j >= Z) ? j - Z : j;
      const int a_s     = static_cast<int>(ew & 0xffffU) + j;
      addr[k]           = a_s;
      const int s       = s_soft[a_s];
      const int c       = s_c2v[(e0 + k) * Z + t];
      int       vv      = min(max(s - c, -LLR_MAX), LLR_MAX);
      vv                = llr_isinf(s) ? s : vv;
      v[k]              = vv;
      const int a       = abs(vv);
      idx               = (a < m1) ? k : idx;
      m2                = min(m2, max(m1, a));
      m1                = min(m1, a);
      sg ^= (vv < 0);
    }
  }
  const int s1 = s_lut[m1];
  const int s2 = s_lut[m2];
#pragma unroll
  for (int k = 0; k < MAXDEG; ++k) {
    if (k < deg) {
      const int mag = (k == idx) ? s2 : s1;
      const int c   = (sg ^ (v[k] < 0)) ? -mag : mag;
      s_c2v[(e0 + k) * Z + t] = static_cast<int8_t>(c);
      int sum = c + v[k];
      sum     = (sum > LLR_MAX) ? LLR_INF : ((sum < -LLR_MAX) ? -LLR_INF : sum);
      s_soft[addr[k]] = static_cast<int8_t>(llr_isinf(v[k]) ? v[k] : sum);
    }
  }
}

} // namespace

template <int MAXDEG>
__global__ void __launch_bounds__(1024)
    ldpc_decode_kernel(const dec_cb* __restrict__ cbs, const graph_desc* __restrict__ graph, lds_layout lay,
                       const int8_t* __restrict__ llr_base, uint8_t* __restrict__ out_base,
                       ldpc_hip_cb_result* __restrict__ res_base, const uint32_t* __restrict__ crc_tables)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  int8_t*   s_soft   = reinterpret_cast<int8_t*>(smem + lay.soft);
  int8_t*   s_c2v    = reinterpret_cast<int8_t*>(smem + lay.c2v);
  uint32_t* s_edges  = reinterpret_cast<uint32_t*>(smem + lay.edges);
  uint32_t* s_rows   = reinterpret_cast<uint32_t*>(smem + lay.rows);
  uint32_t* s_groups = reinterpret_cast<uint32_t*>(smem + lay.groups);
  int8_t*   s_lut    = reinterpret_cast<int8_t*>(smem + lay.lut);
  uint8_t*  s_hb     = smem + lay.hard;
  uint32_t* s_red    = reinterpret_cast<uint32_t*>(smem + lay.red);
  uint32_t* s_crct   = reinterpret_cast<uint32_t*>(smem + lay.crct);

  const dec_cb d       = cbs[blockIdx.x];
  const int    tid     = threadIdx.x;
  const int    nthr    = blockDim.x;
  const int    Z       = graph->Z;
  const int    K       = graph->K;
  const int    N_full  = graph->N_full;
  const int    n_edges = graph->n_edges;
  const int    M       = graph->M;
  const int    KZ      = K * Z;
  const int    L       = static_cast<int>(d.llr_length);
  const int8_t* llr    = llr_base + d.llr_offset;
  uint8_t*      out    = out_base + d.out_offset;

  /* ---- prologue: schedule, LUT, CRC table, zeroed c2v, soft bits (load_soft_bits, impl.cpp:149-174) ---- */
  for (int i = tid; i < n_edges; i += nthr) {
    s_edges[i] = graph->edges[i];
  }
  for (int i = tid; i < M; i += nthr) {
    s_rows[i]   = graph->rows[i];
    s_groups[i] = graph->groups[i];
  }
  const float sf = d.scaling_factor;
  for (int i = tid; i <= LLR_MAX; i += nthr) {
    s_lut[i] = static_cast<int8_t>(__builtin_roundf(static_cast<float>(i) * sf)); /* scale_llr, gen.cpp:70-79 */
  }
  if (d.crc_mode != LDPC_HIP_CRC_MODE_NONE) {
    const uint32_t* tab = crc_tables + static_cast<int>(d.crc_poly) * CRC_TABLE_SIZE;
    for (int i = tid; i < 256; i += nthr) {
      s_crct[i] = tab[i];
    }
  }
  {
    uint4*    c2v4 = reinterpret_cast<uint4*>(s_c2v);
    const int n16  = (n_edges * Z + 15) / 16;
    for (int i = tid; i < n16; i += nthr) {
      c2v4[i] = make_uint4(0, 0, 0, 0);
    }
    const int nhb = (lay.red - lay.hard) / 4;
    for (int i = tid; i < nhb; i += nthr) {
      reinterpret_cast<uint32_t*>(s_hb)[i] = 0;
    }
  }
  if (tid == 0) {
    s_red[31] = 0;
  }
  __syncthreads();
  int last_local = 0;
  const int total = N_full * Z;
  for (int i = tid; i < total; i += nthr) {
    int8_t v = 0;
    const int li = i - 2 * Z;
    if (li >= 0 && li < L) {
      v = llr[li];
      if (v != 0) {
        last_local = max(last_local, li + 1);
      }
    }
    s_soft[i] = v;
  }
  if (last_local > 0) {
    atomicMax(reinterpret_cast<int*>(&s_red[31]), last_local);
  }
  __syncthreads();
  const int last = static_cast<int>(s_red[31]);
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
        has_value = (block_crc(s_hb, Lsig, d.crc_poly, s_crct, crc_tables + d.crc_poly * CRC_TABLE_SIZE + 256,
                               s_red) == 0);
      }
    }
  } else {
    /* Codeblock length and number of layers (impl.cpp:103-114). */
    int cb_len = max(last + 2 * Z, (K + 4) * Z);
    cb_len     = ((cb_len + Z - 1) / Z) * Z;
    const int nof_layers = cb_len / Z - K;
    const int n_groups   = graph->n_groups;

    bool hb_current = false;
    for (int it = 0; it < d.max_iterations; ++it) {
      for (int g = 0; g < n_groups; ++g) {
        const uint32_t gw = s_groups[g];
        const int      r0 = static_cast<int>(gw & 0xffU);
        if (r0 >= nof_layers) {
          break;
        }
        const int nr    = min(static_cast<int>(gw >> 8), nof_layers - r0);
        const int items = nr * Z;
        for (int item = tid; item < items; item += nthr) {
          int r = 0, t = item;
          while (t >= Z) {
            t -= Z;
            ++r;
          }
          check_node_update<MAXDEG>(t, s_rows[r0 + r], s_edges, s_soft, s_c2v, s_lut, Z);
        }
        __syncthreads();
      }
      hb_current = false;
      if (d.crc_mode == LDPC_HIP_CRC_MODE_EARLY_STOP) {
        const bool ok = block_hard_decision(s_soft, s_hb, KZ);
        hb_current    = true;
        if (ok && block_crc(s_hb, Lsig, d.crc_poly, s_crct, crc_tables + d.crc_poly * CRC_TABLE_SIZE + 256,
                            s_red) == 0) {
          has_value  = 1;
          iterations = it + 1;
          break;
        }
      }
    }
    if (!hb_current) {
      block_hard_decision(s_soft, s_hb, KZ);
    }
    if (d.crc_mode == LDPC_HIP_CRC_MODE_CHECK_AFTER) {
      has_value = (block_crc(s_hb, Lsig, d.crc_poly, s_crct, crc_tables + d.crc_poly * CRC_TABLE_SIZE + 256,
                             s_red) == 0);
    }
  }

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
}

/* ldpc_rate_dematcher_impl::rate_dematch (ldpc_rate_dematcher_impl.cpp:46-213), one workgroup per codeblock.
 * The sequential allot loop (:128-201) is kept; each contiguous copy/combine/zero/fill range inside it runs across the
 * workgroup, with a barrier between passes over the circular buffer (a later pass combines into positions an earlier
 * pass wrote, and saturated sums do not associate). De-interleaving (:203-213) is fused as a gather. */
__global__ void __launch_bounds__(256) ldpc_rate_dematch_kernel(const dematch_cb* __restrict__ cbs)
{
  const dematch_cb d   = cbs[blockIdx.x];
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
  auto aux = [&](unsigned e) -> int {
    return (Qm == 1U) ? in[e] : in[(e % EQ) * Qm + e / EQ]; /* deinterleave_bits_Qm */
  };
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

  bool     copy     = d.new_data != 0;
  unsigned tmp_idx  = k0;
  unsigned consumed = 0;
  unsigned left     = E;
  while (left != 0) {
    if (tmp_idx < ninfo) {
      const unsigned n = min(ninfo - tmp_idx, left);
      if (copy) {
        for (unsigned i = tid; i < tmp_idx; i += nth) {
          out[i] = 0;
        }
        for (unsigned i = tid; i < n; i += nth) {
          out[tmp_idx + i] = static_cast<int8_t>(aux(consumed + i));
        }
      } else {
        for (unsigned i = tid; i < n; i += nth) {
          out[tmp_idx + i] = sat_add(out[tmp_idx + i], aux(consumed + i));
        }
      }
      tmp_idx += n;
      consumed += n;
      left -= n;
    } else if (copy) {
      for (unsigned i = tid; i < ninfo; i += nth) {
        out[i] = 0;
      }
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
    if (copy) {
      for (unsigned i = tid; i < np; i += nth) {
        out[tmp_idx + i] = static_cast<int8_t>(aux(consumed + i));
      }
    } else {
      for (unsigned i = tid; i < np; i += nth) {
        out[tmp_idx + i] = sat_add(out[tmp_idx + i], aux(consumed + i));
      }
    }
    tmp_idx = (tmp_idx + np) % Ncb;
    consumed += np;
    left -= np;
    if (left != 0) {
      copy = false;
    }
    __syncthreads();
  }
  if (copy && tmp_idx != 0) {
    const unsigned cnt = Ncb - tmp_idx; /* out.last(buffer_length - tmp_idx) over the N-sized output (:197-200) */
    for (unsigned i = tid; i < cnt; i += nth) {
      out[N - cnt + i] = 0;
    }
  }
}

/* ---- host-side launch helpers (called from ldpc_hip_api.cpp) ---- */

hipError_t launch_decode(int maxdeg, const dec_cb* d_cbs, uint32_t n, const graph_desc* d_graph,
                         const lds_layout& lay, int block, const int8_t* llr, uint8_t* out,
                         ldpc_hip_cb_result* res, const uint32_t* d_crc, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  if (maxdeg > BG2_MAXDEG) {
    hipLaunchKernelGGL(ldpc_decode_kernel<BG1_MAXDEG>, dim3(n), dim3(block), lay.total, stream, d_cbs, d_graph, lay,
                       llr, out, res, d_crc);
  } else {
    hipLaunchKernelGGL(ldpc_decode_kernel<BG2_MAXDEG>, dim3(n), dim3(block), lay.total, stream, d_cbs, d_graph, lay,
                       llr, out, res, d_crc);
  }
  return hipGetLastError();
}

hipError_t launch_dematch(const dematch_cb* d_cbs, uint32_t n, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ldpc_rate_dematch_kernel, dim3(n), dim3(256), 0, stream, d_cbs);
  return hipGetLastError();
}

hipError_t configure_kernels(uint32_t max_lds)
{
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ldpc_decode_kernel<BG1_MAXDEG>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(max_lds));
  if (e != hipSuccess) {
    return e;
  }
  return hipFuncSetAttribute(reinterpret_cast<const void*>(&ldpc_decode_kernel<BG2_MAXDEG>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(max_lds));
}

} // namespace ldpc_hip
