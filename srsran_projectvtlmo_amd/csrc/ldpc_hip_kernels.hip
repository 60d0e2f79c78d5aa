/*
 * gfx950 (MI355X, CDNA4) kernels of the 5G-NR PUSCH LDPC path besides the decoder body (ldpc_decode_body.h): the mixed
 * decode kernel, rate dematching, TB join, encoder, rate matcher, soft demodulation, and the host-side launchers.
 */
/* this unit instantiates the core specialised kernels (the mixed kernel's bodies); ldpc_spec_kernels_*.hip the rest */
#include <algorithm>
#include <vector>

#define LDPC_SPEC_TU_GRAPHS LDPC_SPEC_GRAPHS_CORE
#include "ldpc_decode_body.h"

namespace ldpc_hip {

/* Several (BG, Z) groups of one plan in ONE launch of 768-thread workgroups (a mixed slot: the large TB's BG1 Z=384
 * CBs on the specialised body beside the small TBs' BG2 CBs on the generic one). Workgroup b decodes CB b of the
 * plan's group-sorted order; its group is the last one with first_block <= b. Used when the whole plan fits the
 * device at once, so one launch replaces a fork/join of per-group launches and their event waits. */
template <bool SF08>
__global__ void __launch_bounds__(768)
    ldpc_decode_mixed_kernel(const dec_cb* __restrict__ cbs, const mixed_group* __restrict__ groups, uint32_t ngroups,
                             const step_task* __restrict__ tasks, const int8_t* llr_base, /* see ldpc_decode_kernel */
                             uint8_t* __restrict__ out_base, ldpc_hip_cb_result* __restrict__ res_base,
                             const uint32_t* __restrict__ crc_tables, const dematch_cb* __restrict__ dm_cbs)
{
  const dematch_cb dm_none{}; /* fused dematcher: dm_cbs[block], or none */
  uint32_t lo = 0, hi = ngroups;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (groups[mid].first_block <= blockIdx.x) {
      lo = mid;
    } else {
      hi = mid;
    }
  }
  const mixed_group g = groups[lo];
  if constexpr (SF08) {
    bool done = false; /* g.spec: specialised kernel id + 1 (a workgroup-uniform branch) */
    sp::static_for<spec::NOF_CORE_SPECS>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      if (g.spec == static_cast<uint32_t>(i + 1)) {
        decode_cb<true, i>(cbs[blockIdx.x], g.graph_slot, tasks + g.task_offset, g.lay, llr_base, out_base, res_base,
                           crc_tables, dm_cbs, dm_none);
        done = true;
      }
    });
    if (done) {
      return;
    }
  }
  decode_cb<SF08, -1>(cbs[blockIdx.x], g.graph_slot, tasks + g.task_offset, g.lay, llr_base, out_base, res_base,
                      crc_tables, dm_cbs, dm_none);
}

/* the persistent work-queue kernels (ldpc_hip_dwq.cpp) of the core graphs, and the one of the dematch-only items */
LDPC_DWQ_KERNELS(dwq_kernel_core, LDPC_SPEC_GRAPHS_CORE)
__global__ void __launch_bounds__(DM_THREADS) ldpc_dwq_dematch_kernel(dwq_args a)
{
  dwq_loop(a, [&](const dwq_item& it) __attribute__((always_inline)) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    dematch_body(it.dm, *reinterpret_cast<const demod_tables*>(it.crc_tables + DTAB_OFFSET),
                 reinterpret_cast<int8_t*>(smem), *reinterpret_cast<demod_tables*>(smem + DM_STAGE));
  });
}
const void* dwq_kernel_dematch() { return reinterpret_cast<const void*>(&ldpc_dwq_dematch_kernel); }

/* ldpc_rate_dematcher_impl::rate_dematch, one workgroup per codeblock (ldpc_dematch_body.h dematch_body). */
__global__ void __launch_bounds__(DM_THREADS) ldpc_rate_dematch_kernel(const dematch_cb* __restrict__ cbs,
                                                                       dematch_cb one, demod_tables tab)
{
  __shared__ __attribute__((aligned(16))) int8_t s_in[DM_STAGE];
  __shared__ demod_tables                        s_dtab;
  dematch_body(cbs != nullptr ? cbs[blockIdx.x] : one, tab, s_in, s_dtab); /* nullptr: one CB, descriptor by value */
}


/* ---- transport-block join: pusch_decoder_impl::join_and_notify / concatenate_codeblocks (pusch_decoder_impl.cpp:
 * 384-497), one workgroup per TB. Each thread owns a contiguous run of TB bytes: it gathers them bit-exactly from the
 * CB messages (data bits only: K*Z - CRC - filler per CB) and folds their CRC24A remainder into the TB CRC with
 * CRC(A || B) = CRC(A) x^(8|B|) + CRC(B) mod G. ---- */
namespace {

/* bit i of a packed MSB-first message, as the low bit */
__device__ __forceinline__ uint32_t msg_bit(const uint8_t* m, uint32_t i) { return (m[i >> 3] >> (7 - (i & 7))) & 1U; }

/* 8 message bits starting at bit q (q + 8 <= message length + 8; the byte after the message is never consumed) */
__device__ __forceinline__ uint32_t msg_byte_at(const uint8_t* m, uint32_t q)
{
  const uint32_t b = q >> 3, sh = q & 7U;
  if (sh == 0) {
    return m[b];
  }
  return ((static_cast<uint32_t>(m[b]) << sh) | (static_cast<uint32_t>(m[b + 1]) >> (8 - sh))) & 0xffU;
}

} // namespace

/* Multi-workgroup TB join. The TB is front-padded with zero bytes to a whole number of 4 KiB chunks (leading zeros do
 * not change a zero-initialised CRC); workgroup (TB, chunk c) gathers its 4 KiB, each thread 16 bytes, computes the
 * chunk's CRC24A remainder as XOR_t crc_t * x^(8*16*(255-t)) mod G, and stores it. The last workgroup of the TB to
 * arrive (device-scope counter) combines the chunks as XOR_c crc_c * x^(8*4096*(n-1-c)) mod G, checks the checksum
 * carried by the last CB, writes the result and resets the TB's CB flags on a TB CRC failure (:423-428). The powers
 * of x come from the host (build_crc_tables). work: per TB TBJ_WORK_WORDS words (chunk CRCs, arrival counter; the
 * counter is zero between launches). blocks[b]: workgroup b's TB descriptor, TB index and chunk (one load, no search).
 * The kernel is a chain of dependent memory round trips, so every load that does not depend on another load's value
 * is issued as early as possible: the power of x for this thread, the checksum bits, and the chunk's message bytes
 * (gathered before the CB CRC flags are known; discarded when a CB failed). */
__global__ void __launch_bounds__(TBJ_THREADS)
    ldpc_tb_join_kernel(const tbj_block* __restrict__ blocks, const uint8_t* __restrict__ msgs,
                        ldpc_hip_cb_result* __restrict__ cb_res,
                        uint8_t* __restrict__ tb_base, ldpc_hip_tb_result* __restrict__ tb_res,
                        const uint32_t* __restrict__ crc_tables, uint32_t* __restrict__ work)
{
  __shared__ uint32_t s_tab[256];
  __shared__ uint32_t s_acc[4];
  __shared__ uint32_t s_wok[TBJ_THREADS / 64];
  const int              tid   = threadIdx.x;
#ifdef LDPC_HIP_DIAG_TBJ /* diagnostic build: device-wide 100 MHz stamps per workgroup (g_diag2[block * 8 + k]) */
#define TBJ_STAMP(k)                                                                                                   \
  if (tid == 0 && blockIdx.x < 64) {                                                                                   \
    g_diag2[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                                                  \
  }
#else
#define TBJ_STAMP(k)
#endif
  TBJ_STAMP(0);
  const uint32_t*        pw    = crc_tables + TBJ_POW_OFFSET;
  const uint32_t         pw_t  = pw[TBJ_THREADS - 1 - tid]; /* x^(8*16*(255-tid)) mod G */
  const tbj_block&       blk   = blocks[blockIdx.x];
  const uint32_t         t     = blk.tb;
  const uint32_t         chunk = blk.chunk;
  const ldpc_hip_tb_desc d     = blk.d;
  const uint32_t         C     = d.nof_cbs;
  const uint8_t*         m0    = msgs + d.msg_offset;
  uint8_t*               tb    = tb_base + d.tb_offset;
  const uint32_t         nb    = d.tbs / 8U;
  const uint32_t         nch   = (nb + TBJ_CHUNK - 1) / TBJ_CHUNK;
  const uint32_t         pad   = nch * TBJ_CHUNK - nb; /* leading zero bytes */
  constexpr uint32_t     G     = 0x1864cfbU;
  const uint32_t         kd    = d.cb_msg_bits - d.cb_crc_bits - d.nof_filler_bits; /* data bits per CB (:62-64) */
  /* the checksum: the 24 bits after the last CB's share of the TB (:486-490), loaded now, used by the last workgroup */
  uint32_t chksum = 0;
  if (tid == 0 && C > 1) {
    const uint32_t last = d.tbs - (C - 1U) * kd;
    const uint8_t* ml   = m0 + static_cast<size_t>(C - 1U) * d.msg_stride;
    for (uint32_t i = 0; i < 24U; ++i) {
      chksum = (chksum << 1) | msg_bit(ml, last + i);
    }
  }

  if (tid == 0) {
    s_acc[1] = 0;
  }
  const uint32_t* tab = crc_tables + LDPC_HIP_CRC24A * CRC_TABLE_SIZE;
  s_tab[tid]          = tab[tid];
  /* this thread's TB bytes: virtual positions v0 .. v0 + 15 of the padded TB, real byte = v - pad */
  const uint32_t v0 = chunk * TBJ_CHUNK + static_cast<uint32_t>(tid) * TBJ_BYTES;
  /* gather (C > 1): all loads first, then the CRC chain over registers; issued before the CB flags are known */
  uint32_t val[TBJ_BYTES] = {};
  if (C > 1 && (kd & 7U) == 0) {
    /* whole data bytes per CB (every TB the segmenter makes: TBS, CRC and filler bits are multiples of 8): byte
     * loads, the CB index and offset stepped without divisions, no branches around the loads */
    const uint32_t kdb   = kd >> 3;
    const uint32_t first = (v0 >= pad) ? v0 - pad : 0;
    uint32_t       r     = first / kdb;
    uint32_t       o     = first - r * kdb;
#pragma unroll
    for (int k = 0; k < TBJ_BYTES; ++k) {
      const bool real = v0 + k >= pad;
      const uint8_t x = m0[static_cast<size_t>(r) * d.msg_stride + o];
      val[k]          = real ? x : 0U;
      const bool step = real && o + 1U == kdb;
      o               = step ? 0U : o + (real ? 1U : 0U);
      r += step ? 1U : 0U;
    }
  } else if (C > 1) {
    const uint32_t first = (v0 >= pad) ? v0 - pad : 0;
    uint32_t       p     = 8U * first;
    uint32_t       r     = p / kd;
    uint32_t       q     = p - r * kd;
#pragma unroll
    for (int k = 0; k < TBJ_BYTES; ++k) {
      const uint32_t v = v0 + k;
      uint32_t       x = 0;
      if (v >= pad) {
        if (q + 8U <= kd) {
          x = msg_byte_at(m0 + static_cast<size_t>(r) * d.msg_stride, q);
        } else { /* straddles into the next CB */
          for (uint32_t i = 0; i < 8U; ++i) {
            const uint32_t qi = q + i;
            x = (x << 1) | ((qi < kd) ? msg_bit(m0 + static_cast<size_t>(r) * d.msg_stride, qi)
                                      : msg_bit(m0 + static_cast<size_t>(r + 1) * d.msg_stride, qi - kd));
          }
        }
        q += 8U;
        if (q >= kd) {
          q -= kd;
          ++r;
        }
      }
      val[k] = x;
    }
  }
  /* CBs whose CRC passed: per-thread count, wave sum by shuffles, one LDS word per wave (no zeroing barrier) */
  uint32_t myok = 0;
  for (uint32_t r = tid; r < C; r += TBJ_THREADS) {
    myok += (cb_res[d.result_index + r].crc_pass != 0) ? 1U : 0U;
  }
  for (int o = 32; o > 0; o >>= 1) {
    myok += __shfl_xor(myok, o);
  }
  if ((tid & 63) == 0) {
    s_wok[tid >> 6] = myok;
  }
  __syncthreads();
  TBJ_STAMP(1);
  uint32_t nok = 0;
  for (int w = 0; w < TBJ_THREADS / 64; ++w) {
    nok += s_wok[w];
  }

  if (C == 1) {
    /* the CB CRC is the TB CRC; copy the TB bytes only when it passed (:409-417) */
    if (nok == 1) {
      for (uint32_t k = 0; k < TBJ_BYTES; ++k) {
        const uint32_t v = v0 + k;
        if (v >= pad) {
          tb[v - pad] = m0[v - pad];
        }
      }
    }
    if (chunk == 0 && tid == 0) {
      tb_res[t] = ldpc_hip_tb_result{static_cast<uint8_t>(nok), static_cast<uint8_t>(nok), static_cast<uint16_t>(nok)};
    }
    return;
  }
  if (nok != C) { /* :418-420, nothing written */
    if (chunk == 0 && tid == 0) {
      tb_res[t] = ldpc_hip_tb_result{0, 0, static_cast<uint16_t>(nok)};
    }
    return;
  }
  uint32_t crc = 0;
#pragma unroll
  for (int k = 0; k < TBJ_BYTES; ++k) {
    crc = ((crc << 8) ^ s_tab[((crc >> 16) ^ val[k]) & 0xffU]) & 0xffffffU; /* crc_calculator_generic_impl.cpp */
  }
  crc = gf2_mulmod(crc, pw_t, 24, G);
  for (int o = 32; o > 0; o >>= 1) { /* wave XOR, then one LDS atomic per wave (same-address atomics serialise) */
    crc ^= __shfl_xor(crc, o);
  }
  if ((tid & 63) == 0) {
    atomicXor(&s_acc[1], crc);
  }
  __syncthreads();
  TBJ_STAMP(2);
  /* Hand-off to the TB's last workgroup without cache-wide fences (cdna_hip_programming.md Guideline 16, R1): the chunk
   * CRC is stored write-through (agent-scope atomic store), drained, then the arrival counter is bumped; the last
   * arriver reads the chunk CRCs with agent-scope (sc1) loads, which bypass the stale caches. */
  typedef __attribute__((address_space(1))) uint32_t gu32;
  gu32* wk = (gu32*)(uintptr_t)(work + static_cast<size_t>(t) * TBJ_WORK_WORDS); /* global, not flat */
  if (tid == 0) {
    __hip_atomic_store(&wk[chunk], s_acc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_acc[2] = __hip_atomic_fetch_add(&wk[TBJ_MAX_CHUNKS], 1U, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  TBJ_STAMP(3);
  /* the TB bytes, stored after the hand-off: no barrier or counter waits for their completion (vmcnt counts stores
   * too); the kernel's end makes them visible */
#pragma unroll
  for (int k = 0; k < TBJ_BYTES; ++k) {
    const uint32_t v = v0 + k;
    if (v >= pad) {
      tb[v - pad] = static_cast<uint8_t>(val[k]);
    }
  }
  if (s_acc[2] != nch - 1) {
    return; /* not the last workgroup of this TB */
  }
  if (tid == 0) {
    s_acc[3] = 0;
  }
  __syncthreads();
  if (static_cast<uint32_t>(tid) < ((nch + 63U) & ~63U)) { /* the waves holding chunks, whole */
    uint32_t x = 0;
    if (static_cast<uint32_t>(tid) < nch) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); /* keeps the sc1 loads below the counter read */
      const uint32_t c = __hip_atomic_load(&wk[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x                = gf2_mulmod(c, pw[TBJ_THREADS + nch - 1 - tid], 24, G);
    }
    for (int o = 32; o > 0; o >>= 1) {
      x ^= __shfl_xor(x, o);
    }
    if ((tid & 63) == 0) {
      atomicXor(&s_acc[3], x);
    }
  }
  __syncthreads();
  if (tid == 0) {
    wk[TBJ_MAX_CHUNKS] = 0; /* counter back to zero for the next launch */
    s_acc[0]           = (s_acc[3] == chksum) ? 1U : 0U;
    tb_res[t] = ldpc_hip_tb_result{static_cast<uint8_t>(s_acc[0]), 1, static_cast<uint16_t>(nok)};
  }
  __syncthreads();
  TBJ_STAMP(4);
  if (s_acc[0] == 0) { /* reset_codeblocks_crc (:423-428): a false-positive CB is somewhere; decode all again */
    for (uint32_t r = tid; r < C; r += TBJ_THREADS) {
      cb_res[d.result_index + r].crc_pass = 0;
    }
  }
}


/* ---- LDPC encoder: ldpc_encoder_impl::encode + ldpc_encoder_generic (ldpc_encoder_impl.cpp:47-81,
 * ldpc_encoder_generic.cpp:32-230), one 256-thread workgroup per codeblock, bit-packed in LDS. SURVEY.md section 8 f2.
 * Every lifted column of Z bits is a run of 32-bit words, LSB first (bit j of a column at word j / 32, bit j % 32). A
 * check row of the base graph with edge (c, s) reads column c rotated by s: 32 of its bits starting at (s + 32 w) mod
 * Z, which is one funnel shift (v_alignbit) of two words of the column's doubled copy (its bits repeated to 2 Z + 64),
 * so a row's 32 check nodes cost two LDS reads and one XOR per edge instead of 32 byte reads (the previous kernel:
 * one byte per bit, 81.5 us for a 128-CB BG1 Z=384 TB, profiles/r04/hal_kernel_trace.txt).
 *   message: K Z bits from the packed (MSB first) source at a bit offset, data_bits of them, zeros after; with crc_at
 *            = S > 0 the CRC24B of bits [0, S) goes to bits [S, S + 24) (TS 38.212 5.2.2: the codeblock CRC of a
 *            segmented TB, which the accelerator attaches in TB mode, hw_accelerator_pdsch_enc.h), computed by the
 *            slicing tables and the x^(32 e) mod G columns of the context's CRC tables (the decoder's block_crc)
 *   preprocess_systematic_bits (generic.cpp:57-101): aux rows 0-3 and the extension parity words from the message
 *   high-rate region (generic.cpp:133-230): the four core parity columns from the aux rows
 *   extension region (generic.cpp:103-120): each extension parity column ^= the row's rotated core parity columns
 *   write_codeblock: codeword bits [2Z, 2Z + cw_length), packed MSB first (bit-reversed words). ---- */
constexpr int ENC_ZW      = MAX_Z / 32;          /* words of one column                           */
constexpr int ENC_ZS      = ENC_ZW + 1;          /* its stride (a funnel shift reads one word on) */
constexpr int ENC_WC      = 2 * ENC_ZW + 2;      /* words of a doubled column                     */
constexpr int ENC_MW      = 22 * MAX_Z / 32 + 2; /* message words                                 */
constexpr int ENC_RAW     = 22 * MAX_Z / 8 + 16; /* message source bytes (bit offset, window)     */

/* 32 bits of the LSB-first bit string v from bit o */
__device__ __forceinline__ uint32_t enc_get32(const uint32_t* v, uint32_t o)
{
  return __builtin_amdgcn_alignbit(v[(o >> 5) + 1], v[o >> 5], o & 31U);
}

/* word q of the doubled copy of a Z-bit column whose bit j is bit base + j of v: bit t = column bit (32 q + t) mod Z */
__device__ __forceinline__ uint32_t enc_dbl(const uint32_t* v, uint32_t base, uint32_t q, uint32_t Z)
{
  if (Z >= 32) { /* at most one wrap in a word */
    const uint32_t o = (32U * q) % Z;
    const uint32_t a = Z - o;
    uint32_t       w = enc_get32(v, base + o);
    if (a < 32) {
      w = (w & ((1U << a) - 1U)) | (enc_get32(v, base) << a);
    }
    return w;
  }
  uint32_t w = 0;
  for (uint32_t t = 0; t != 32; ++t) {
    const uint32_t i = base + (32U * q + t) % Z;
    w |= ((v[i >> 5] >> (i & 31U)) & 1U) << t;
  }
  return w;
}

/* The encoder's LDS state: the codeword's columns, bit-packed. */
constexpr int ENC_OBUF = 4096; /* rate-matched bytes staged per chunk (pdsch_rate_match) */
struct enc_lds {
  uint4    obuf[ENC_OBUF / 16];
  uint8_t  raw[ENC_RAW];
  uint32_t m[ENC_MW];                  /* the message, K Z bits                     */
  uint32_t d[(22 + 5) * ENC_WC];       /* doubled: message columns, p0..p3, aux sum */
  uint32_t a[4 * ENC_ZS];              /* aux rows 0-3                              */
  uint32_t p[4 * ENC_ZS];              /* core parity columns K .. K+3              */
  uint32_t x[(MAX_ROWS - 4) * ENC_ZS]; /* extension parity columns K+4 ..           */
  uint32_t s[ENC_ZS];                  /* aux row sum                               */
  uint32_t rows[MAX_ROWS];
  uint32_t edge[MAX_EDGES];            /* (column << 16) | shift                    */
  uint32_t red[ENC_THREADS / 64];
};

struct enc_geom {
  uint32_t Z, K, NF;
  /* codeword column c's bits: bit j at bit base + j of the returned LSB-first string */
  __device__ __forceinline__ const uint32_t* col(const enc_lds& L, uint32_t c, uint32_t& base) const
  {
    base = 0;
    if (c < K) {
      base = c * Z;
      return L.m;
    }
    return c < K + 4 ? L.p + (c - K) * ENC_ZS : L.x + (c - K - 4) * ENC_ZS;
  }
};

/* Encodes codeblock d into L (every column of the codeword up to the layers d.cw_length needs); block-uniform. */
__device__ __forceinline__ enc_geom enc_build(const enc_cb& d, const uint8_t* __restrict__ msg_base,
                                              const uint32_t* __restrict__ crc_tables, enc_lds& L)
{
  uint8_t*  s_raw  = L.raw;
  uint32_t* s_m    = L.m;
  uint32_t* s_d    = L.d;
  uint32_t* s_a    = L.a;
  uint32_t* s_p    = L.p;
  uint32_t* s_x    = L.x;
  uint32_t* s_s    = L.s;
  uint32_t* s_rows = L.rows;
  uint32_t* s_edge = L.edge;
  uint32_t* s_red  = L.red;

  const graph_desc* gr  = &c_graphs[d.graph_slot];
  const uint32_t    tid = threadIdx.x;
  const uint32_t    Z = gr->Z, K = gr->K, NF = gr->N_full, M = gr->M;
  const uint32_t    ZW = (Z + 31) / 32, WC = 2 * ZW + 2;
  const uint8_t*    msg = msg_base + d.msg_offset;

  /* codeblock length: max(output + 2Z, (K + 4) Z), a multiple of Z (ldpc_encoder_impl.cpp:68-77) */
  uint32_t cb_len = max(d.cw_length + 2 * Z, (K + 4) * Z);
  cb_len          = (cb_len + Z - 1) / Z * Z;
  const uint32_t nof_layers = cb_len / Z - K;

  /* the source bytes (one load per byte, all issued before any is used: the source may be pinned host memory read
   * over PCIe), the graph's rows and edges */
  const uint32_t nbytes = (d.msg_bit_off + d.data_bits + 7) / 8;
  constexpr int  NRAW   = (ENC_RAW + ENC_THREADS - 1) / ENC_THREADS;
  constexpr int  NEDGE  = (MAX_EDGES + ENC_THREADS - 1) / ENC_THREADS;
  static_assert(MAX_ROWS <= ENC_THREADS, "one row word per thread");
  uint32_t raw[NRAW], edge[NEDGE], row = 0;
  /* every load issued before any is stored (a loop of load -> LDS store waited for each over PCIe) */
#pragma unroll
  for (int k = 0; k < NRAW; ++k) {
    const uint32_t i = tid + k * ENC_THREADS;
    raw[k]           = i < nbytes ? msg[i] : 0U;
  }
#pragma unroll
  for (int k = 0; k < NEDGE; ++k) {
    const uint32_t e = tid + k * ENC_THREADS;
    edge[k]          = e < gr->n_edges ? gr->edges[e] : 0U;
  }
  if (tid < M) {
    row = gr->rows[tid];
  }
#pragma unroll
  for (int k = 0; k < NRAW; ++k) {
    const uint32_t i = tid + k * ENC_THREADS;
    if (i < static_cast<uint32_t>(ENC_RAW)) {
      s_raw[i] = static_cast<uint8_t>(raw[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < NEDGE; ++k) {
    const uint32_t e = tid + k * ENC_THREADS;
    if (e < gr->n_edges) {
      s_edge[e] = (((edge[k] & 0xffffU) / Z) << 16) | (edge[k] >> 16);
    }
  }
  if (tid < M) {
    s_rows[tid] = row;
  }
  __syncthreads();
  /* message words: 32 source bits from bit 32 u + msg_bit_off (a 40-bit big-endian window), bit-reversed to LSB first;
   * bits from data_bits on are 0 (a short last segment, the CRC and filler positions) */
  for (uint32_t u = tid; u < static_cast<uint32_t>(ENC_MW); u += ENC_THREADS) {
    uint32_t w = 0;
    if (32 * u < d.data_bits) {
      const uint32_t b = 4 * u;
      const uint64_t x = (static_cast<uint64_t>(s_raw[b]) << 32) | (static_cast<uint64_t>(s_raw[b + 1]) << 24) |
                         (static_cast<uint64_t>(s_raw[b + 2]) << 16) | (static_cast<uint64_t>(s_raw[b + 3]) << 8) |
                         s_raw[b + 4];
      w                 = __builtin_bitreverse32(static_cast<uint32_t>(x >> (8 - d.msg_bit_off)));
      const uint32_t nv = d.data_bits - 32 * u;
      if (nv < 32) {
        w &= (1U << nv) - 1U;
      }
    }
    s_m[u] = w;
  }
  __syncthreads();
  if (d.crc_at != 0) {
    /* CRC24B of bits [0, S): front-padded to nw words (leading zeros do not change a zero-init CRC); word w's CRC by
     * four slicing-table lookups, times x^(32 (nw - 1 - w)) mod G as the XOR of precomputed columns (block_crc) */
    const uint32_t  S    = d.crc_at;
    const uint32_t  nw   = (S + 31) / 32, pad = 32 * nw - S;
    const uint32_t* t0   = crc_tables + LDPC_HIP_CRC24B * CRC_TABLE_SIZE;
    const uint32_t* t1   = crc_tables + CRC_SLICE_OFFSET + LDPC_HIP_CRC24B * CRC_SLICE_WORDS;
    const uint32_t* mcol = crc_tables + CRC_MCOL_OFFSET + LDPC_HIP_CRC24B * CRC_MCOL_WORDS;
    uint32_t        acc  = 0;
    for (uint32_t w = tid; w < nw; w += ENC_THREADS) {
      const uint32_t  v    = (w == 0) ? (s_m[0] << pad) : enc_get32(s_m, 32 * w - pad);
      const uint32_t  W    = __builtin_bitreverse32(v); /* MSB first */
      const uint32_t  crc  = (t1[2 * 256 + (W >> 24)] ^ t1[256 + ((W >> 16) & 0xffU)] ^ t1[(W >> 8) & 0xffU] ^
                            t0[W & 0xffU]) & 0xffffffU;
      const uint32_t* col  = mcol + (nw - 1 - w) * 24;
      uint32_t        prod = 0;
      for (int i = 0; i < 24; ++i) {
        prod ^= col[i] & (0U - ((crc >> i) & 1U));
      }
      acc ^= prod;
    }
    acc = wave_xor(acc);
    if ((tid & 63) == 0) {
      s_red[tid >> 6] = acc;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t crc = 0;
      for (int i = 0; i < ENC_THREADS / 64; ++i) {
        crc ^= s_red[i];
      }
      const uint32_t v = __builtin_bitreverse32(crc << 8); /* CRC bit 23 (sent first) at bit 0 */
      const uint32_t s = S & 31U;
      s_m[S >> 5] |= v << s;
      if (s > 8) {
        s_m[(S >> 5) + 1] |= v >> (32 - s);
      }
    }
    __syncthreads();
  }
  /* doubled message columns */
  for (uint32_t i = tid; i < K * WC; i += ENC_THREADS) {
    const uint32_t c = i / WC, q = i - c * WC;
    s_d[c * ENC_WC + q] = enc_dbl(s_m, c * Z, q, Z);
  }
  __syncthreads();
  /* preprocess_systematic_bits: each row's systematic edges */
  for (uint32_t i = tid; i < nof_layers * ZW; i += ENC_THREADS) {
    const uint32_t m = i / ZW, w = i - m * ZW;
    const uint32_t rw = s_rows[m], e0 = rw & 0xffffU, deg = rw >> 16;
    uint32_t       x  = 0;
    for (uint32_t k = 0; k < deg; ++k) {
      const uint32_t ed = s_edge[e0 + k], col = ed >> 16;
      if (col < K) {
        x ^= enc_get32(s_d + col * ENC_WC, (ed & 0xffffU) + 32 * w);
      }
    }
    (m < 4 ? s_a + m * ENC_ZS : s_x + (m - 4) * ENC_ZS)[w] = x;
  }
  __syncthreads();
  /* high-rate region (generic.cpp:133-230): p0 = the aux sum rotated by r, then p1..p3 from the aux rows and p0 or p0
   * rotated by one */
  const bool     bg1     = gr->bg == 1;
  const bool     special = bg1 ? (gr->ils == 6) : (gr->ils == 3 || gr->ils == 7);
  const uint32_t r       = (special && bg1) ? (Z - 105 % Z) % Z : ((!special && !bg1) ? Z - 1 : 0);
  uint32_t*      dsum    = s_d + (K + 4) * ENC_WC;
  for (uint32_t w = tid; w < static_cast<uint32_t>(ENC_ZS); w += ENC_THREADS) {
    s_s[w] = w < ZW ? (s_a[w] ^ s_a[ENC_ZS + w] ^ s_a[2 * ENC_ZS + w] ^ s_a[3 * ENC_ZS + w]) : 0U;
  }
  __syncthreads();
  for (uint32_t q = tid; q < WC; q += ENC_THREADS) {
    dsum[q] = enc_dbl(s_s, 0, q, Z);
  }
  __syncthreads();
  for (uint32_t w = tid; w < static_cast<uint32_t>(ENC_ZS); w += ENC_THREADS) {
    s_p[w] = w < ZW ? enc_get32(dsum, r + 32 * w) : 0U;
  }
  __syncthreads();
  for (uint32_t q = tid; q < WC; q += ENC_THREADS) {
    s_d[K * ENC_WC + q] = enc_dbl(s_p, 0, q, Z);
  }
  __syncthreads();
  for (uint32_t w = tid; w < static_cast<uint32_t>(ENC_ZS); w += ENC_THREADS) {
    uint32_t p1 = 0, p2 = 0, p3 = 0;
    if (w < ZW) {
      const uint32_t a0 = s_a[w], a1 = s_a[ENC_ZS + w], a2 = s_a[2 * ENC_ZS + w], a3 = s_a[3 * ENC_ZS + w];
      const uint32_t p0 = s_p[w], p0r = enc_get32(s_d + K * ENC_WC, 32 * w + 1); /* p0[k], p0[k + 1 mod Z] */
      if (bg1) {
        const uint32_t qv = special ? p0 : p0r;
        p1                = a0 ^ qv;
        p3                = a3 ^ qv;
        p2                = a2 ^ p3;
      } else {
        const uint32_t qv = special ? p0r : p0;
        p1                = a0 ^ qv;
        p2                = a1 ^ p1;
        p3                = a3 ^ qv;
      }
    }
    s_p[ENC_ZS + w]     = p1;
    s_p[2 * ENC_ZS + w] = p2;
    s_p[3 * ENC_ZS + w] = p3;
  }
  __syncthreads();
  for (uint32_t i = tid; i < 3 * WC; i += ENC_THREADS) {
    const uint32_t j = i / WC, q = i - j * WC;
    s_d[(K + 1 + j) * ENC_WC + q] = enc_dbl(s_p + (1 + j) * ENC_ZS, 0, q, Z);
  }
  __syncthreads();
  /* extension region (generic.cpp:103-120): the rows' core parity edges */
  for (uint32_t i = tid; i < (nof_layers - 4) * ZW; i += ENC_THREADS) {
    const uint32_t m = 4 + i / ZW, w = i - (m - 4) * ZW;
    const uint32_t rw = s_rows[m], e0 = rw & 0xffffU, deg = rw >> 16;
    uint32_t       x  = 0;
    for (uint32_t k = 0; k < deg; ++k) {
      const uint32_t ed = s_edge[e0 + k], col = ed >> 16;
      if (col >= K && col < K + 4) {
        x ^= enc_get32(s_d + col * ENC_WC, (ed & 0xffffU) + 32 * w);
      }
    }
    s_x[(m - 4) * ENC_ZS + w] ^= x;
  }
  __syncthreads();
  return enc_geom{Z, K, NF};
}

/* write_codeblock: output bit i = codeword bit 2Z + i, in column (2Z + i) / Z; packed MSB first */
__device__ __forceinline__ void enc_write_codeblock(const enc_cb& d, const enc_lds& L, const enc_geom& g,
                                                    uint8_t* __restrict__ cw)
{
  const uint32_t Z = g.Z, NF = g.NF;
  const uint32_t nb = (d.cw_length + 7) / 8;
  for (uint32_t u = threadIdx.x; u < (d.cw_length + 31) / 32; u += ENC_THREADS) {
    const uint32_t p = 2 * Z + 32 * u;
    uint32_t       w = 0;
    if (Z >= 32) { /* at most two columns in a word */
      const uint32_t  c = p / Z, off = p - c * Z, a = Z - off;
      uint32_t        base;
      const uint32_t* v = g.col(L, c, base);
      w                 = enc_get32(v, base + off);
      if (a < 32) {
        w &= (1U << a) - 1U;
        if (c + 1 < NF) {
          const uint32_t* v2 = g.col(L, c + 1, base);
          w |= enc_get32(v2, base) << a;
        }
      }
    } else {
      for (uint32_t t = 0; t != 32; ++t) {
        const uint32_t c = (p + t) / Z;
        if (c < NF) {
          uint32_t        base;
          const uint32_t* v = g.col(L, c, base);
          const uint32_t  j = base + (p + t - c * Z);
          w |= ((v[j >> 5] >> (j & 31U)) & 1U) << t;
        }
      }
    }
    const uint32_t nv = d.cw_length - 32 * u;
    if (nv < 32) {
      w &= (1U << nv) - 1U;
    }
    const uint32_t y = __builtin_bitreverse32(w); /* MSB first: byte 0 = bits 31..24 */
    for (uint32_t k = 0; k != 4; ++k) {
      if (4 * u + k < nb) {
        cw[4 * u + k] = static_cast<uint8_t>(y >> (24 - 8 * k));
      }
    }
  }
}

__global__ void __launch_bounds__(ENC_THREADS) ldpc_encode_kernel(const enc_cb* __restrict__ cbs,
                                                                  const uint8_t* __restrict__ msg_base,
                                                                  uint8_t* __restrict__ cw_base,
                                                                  const uint32_t* __restrict__ crc_tables)
{
  __shared__ enc_lds L;
  const enc_cb       d = cbs[blockIdx.x];
  const enc_geom     g = enc_build(d, msg_base, crc_tables, L);
  enc_write_codeblock(d, L, g, cw_base + d.cw_offset);
}

/* ldpc_rate_matcher_impl::rate_match of codeblock d (ldpc_rate_match_kernel's arithmetic, below) from the codeword in
 * L: one output bit per thread and round, each wave's 64 bits packed by a ballot */
__device__ __forceinline__ void pdsch_rate_match(const ratematch_cb& d, enc_lds& L, const enc_geom& g,
                                                 uint8_t* __restrict__ out_base)
{
  uint8_t*             out = out_base + d.out_offset;
  const uint32_t       fl = min(d.fill_lo, d.Ncb), fh = min(d.fill_hi, d.Ncb);
  const uint32_t       Ls = d.Ncb - (fh - fl);
  uint32_t             k0 = d.k0;
  if (k0 >= fl && k0 < fh) {
    k0 = fh;
  }
  k0                = (k0 >= d.Ncb) ? 0 : k0;
  const uint32_t r0 = (k0 < fl) ? k0 : k0 - (fh - fl);
  const uint32_t E  = d.rm_length, Qm = d.Qm;
  const uint32_t EQ = E / Qm;
  const uint32_t nb = (E + 7) / 8;
  const uint32_t qs = Qm == 8 ? 3U : (Qm == 4 ? 2U : (Qm == 2 ? 1U : 0U));
  /* x / y for x < 2^21 from a float reciprocal (|error| < 1/2 before the correction); exact division above */
  const bool  fast   = r0 + E < (1U << 21);
  const float inv_ls = 1.0f / static_cast<float>(Ls), inv_z = 1.0f / static_cast<float>(g.Z);
  auto        fdiv   = [](uint32_t x, uint32_t y, float inv) {
    uint32_t  q  = static_cast<uint32_t>(static_cast<float>(x) * inv);
    const int rr = static_cast<int>(x - q * y);
    return rr < 0 ? q - 1 : (rr >= static_cast<int>(y) ? q + 1 : q);
  };
  /* one output bit per thread and round; each wave's 64 bits packed by a ballot, lanes 0-7 put its 8 bytes into LDS;
   * each chunk of ENC_OBUF bytes then leaves in 16-byte stores (the output is often pinned host memory: byte stores
   * went out as one small PCIe write each) */
  const uint32_t lane = threadIdx.x & 63U;
  uint8_t*       ob   = reinterpret_cast<uint8_t*>(L.obuf);
  for (uint32_t c0 = 0; c0 < E; c0 += 8 * ENC_OBUF) {
    const uint32_t cend = min(E, c0 + 8U * ENC_OBUF);
    for (uint32_t o0 = c0; o0 < cend; o0 += ENC_THREADS) {
      const uint32_t o   = o0 + threadIdx.x;
      uint32_t       bit = 0;
      if (o < E) {
        /* interleave_bits: output bit jj Qm + i takes selected bit i EQ + jj */
        const uint32_t  jj = Qm == 6 ? o / 6U : o >> qs;
        const uint32_t  i  = o - jj * Qm;
        const uint32_t  x  = r0 + i * EQ + jj;
        const uint32_t  r  = fast ? x - fdiv(x, Ls, inv_ls) * Ls : x % Ls;
        const uint32_t  p  = ((r < fl) ? r : r + (fh - fl)) + 2 * g.Z; /* codeword bit */
        const uint32_t  cc = fdiv(p, g.Z, inv_z);
        uint32_t        base;
        const uint32_t* src = g.col(L, cc, base);
        const uint32_t  j   = base + (p - cc * g.Z);
        bit                 = (src[j >> 5] >> (j & 31U)) & 1U;
      }
      const uint64_t m  = __ballot(bit != 0U);
      const uint32_t b0 = (o0 + (threadIdx.x & ~63U)) / 8;
      if (lane < 8 && b0 + lane < nb) {
        /* output bit 8 k + t is ballot bit 8 k + t of this wave, sent MSB first */
        ob[b0 + lane - c0 / 8] =
            static_cast<uint8_t>(__builtin_bitreverse32((static_cast<uint32_t>(m >> (8 * lane)) & 0xffU)) >> 24);
      }
    }
    __syncthreads();
    const uint32_t nbc = min(nb - c0 / 8, static_cast<uint32_t>(ENC_OBUF));
    uint8_t*       dst = out + c0 / 8;
    const uint32_t n16 = (reinterpret_cast<uintptr_t>(dst) & 15U) == 0 ? nbc / 16 : 0U;
    for (uint32_t k = threadIdx.x; k < n16; k += ENC_THREADS) {
      reinterpret_cast<uint4*>(dst)[k] = L.obuf[k];
    }
    for (uint32_t k = 16 * n16 + threadIdx.x; k < nbc; k += ENC_THREADS) {
      dst[k] = ob[k];
    }
    __syncthreads();
  }
}

/* The PDSCH encoder queue's batch (ldpc_hip_enc_queue.cpp): encoder and rate matcher in one workgroup per codeblock,
 * the rate matcher reading the codeword's bits from LDS (no codeword buffer, one launch per batch). Descriptors by
 * value for one codeblock (cbs == nullptr), else from the queue's pinned buffer. The rate matcher's arithmetic is
 * ldpc_rate_match_kernel's (below), bit for bit. */
__global__ void __launch_bounds__(ENC_THREADS) ldpc_pdsch_encode_kernel(const pdsch_enc_cb* cbs, pdsch_enc_cb one,
                                                                        const uint8_t* __restrict__ msg_base,
                                                                        uint8_t* __restrict__ out_base,
                                                                        const uint32_t* __restrict__ crc_tables)
{
  __shared__ enc_lds   L;
  const pdsch_enc_cb   c = cbs != nullptr ? cbs[blockIdx.x] : one;
  const enc_geom       g = enc_build(c.enc, msg_base, crc_tables, L);
  pdsch_rate_match(c.rm, L, g, out_base);
}

/* The PDSCH encoder queue's work-queue kernel (ldpc_hip_dwq.h key DWQ_KEY_ENC): a small batch's codeblocks as items of
 * the resident grid, no launch per batch (the payload, dwq_enc_payload, in the item's first words). */
__global__ void __launch_bounds__(ENC_THREADS) ldpc_dwq_encode_kernel(dwq_args a)
{
  __shared__ enc_lds L;
  dwq_loop(a, [&](const dwq_item& it) __attribute__((always_inline)) {
    dwq_enc_payload pl;
    __builtin_memcpy(&pl, &it, sizeof(pl));
    const enc_geom g = enc_build(pl.c.enc, pl.msg_base, pl.crc_tables, L);
    pdsch_rate_match(pl.c.rm, L, g, pl.out_base);
  });
}
const void* dwq_kernel_encode() { return reinterpret_cast<const void*>(&ldpc_dwq_encode_kernel); }

/* The HAL decoder's early copy (ldpc_hip_api.cpp hal_copy_staged): each item moves one piece of a large batch's staged
 * LLRs from pinned host memory into HBM while the caller is still enqueueing, COPY_UNROLL 16-byte loads per thread in
 * flight before any store (one PCIe round trip per 64 KiB per workgroup), so the batch kernel reads HBM. */
__global__ void __launch_bounds__(COPY_THREADS) ldpc_dwq_copy_kernel(dwq_args a)
{
  dwq_loop(a, [&](const dwq_item& it) __attribute__((always_inline)) {
    dwq_copy_payload pl;
    __builtin_memcpy(&pl, &it, sizeof(pl));
    for (uint64_t k0 = 0; k0 < pl.n16; k0 += COPY_THREADS * COPY_UNROLL) {
      uint4 v[COPY_UNROLL];
#pragma unroll
      for (int u = 0; u < COPY_UNROLL; ++u) {
        const uint64_t k = k0 + static_cast<uint64_t>(u) * COPY_THREADS + threadIdx.x;
        v[u]             = k < pl.n16 ? reinterpret_cast<const uint4*>(pl.src)[k] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < COPY_UNROLL; ++u) {
        const uint64_t k = k0 + static_cast<uint64_t>(u) * COPY_THREADS + threadIdx.x;
        if (k < pl.n16) {
          reinterpret_cast<uint4*>(pl.dst)[k] = v[u];
        }
      }
    }
  });
}
const void* dwq_kernel_copy() { return reinterpret_cast<const void*>(&ldpc_dwq_copy_kernel); }


/* ---- rate matcher: ldpc_rate_matcher_impl::rate_match (ldpc_rate_matcher_impl.cpp:36-160): bit selection from k0
 * around the circular buffer [0, Ncb) skipping the filler range, then the Qm interleaver. Every output bit is computed
 * independently from its rank in the filler-free circular sequence. ---- */
__global__ void __launch_bounds__(256) ldpc_rate_match_kernel(const ratematch_cb* __restrict__ cbs,
                                                              const uint8_t* __restrict__ cw_base,
                                                              uint8_t* __restrict__ out_base)
{
  const ratematch_cb d  = cbs[blockIdx.x];
  const uint8_t*     cw = cw_base + d.cw_offset;
  uint8_t*           out = out_base + d.out_offset;
  const uint32_t     fl = min(d.fill_lo, d.Ncb), fh = min(d.fill_hi, d.Ncb);
  const uint32_t     L  = d.Ncb - (fh - fl);             /* selectable bits in the circular buffer */
  uint32_t           k0 = d.k0;
  if (k0 >= fl && k0 < fh) {
    k0 = fh;                                              /* select_bits: skip a filler start */
  }
  k0                 = (k0 >= d.Ncb) ? 0 : k0;
  const uint32_t r0  = (k0 < fl) ? k0 : k0 - (fh - fl);   /* rank of the first selected bit */
  const uint32_t EQ  = d.rm_length / d.Qm;
  const uint32_t nb  = (d.rm_length + 7) / 8;
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
    uint32_t v = 0;
    for (uint32_t q = 0; q < 8; ++q) {
      const uint32_t o = 8 * b + q;
      if (o < d.rm_length) {
        /* interleave_bits (:162-): output bit o = jj * Qm + i takes selected bit i * EQ + jj */
        const uint32_t jj = o / d.Qm, i = o - jj * d.Qm;
        const uint32_t e  = i * EQ + jj;
        const uint32_t r  = (r0 + e) % L;
        const uint32_t p  = (r < fl) ? r : r + (fh - fl);
        v |= ((cw[p >> 3] >> (7 - (p & 7))) & 1U) << (7 - q);
      }
    }
    out[b] = static_cast<uint8_t>(v);
  }
}

/* ---- host-side launch helpers (called from ldpc_hip_api.cpp) ---- */

/* the specialised kernels instantiated in ldpc_spec_kernels_*.hip (their host launch stubs) */
#define LDPC_SPEC_KERNEL_DECL(id, bg, z, ils) const void* spec_kernel_##id(); const void* spec_split_kernel_##id();
LDPC_SPEC_GRAPHS_MID_A(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_MID_B(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_MID_C(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_MID_D(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_MID_E(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_MID_F(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_MID_G(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_MID_H(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_SMALL_I(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_SMALL_J(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_SMALL_K(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_SMALL_L(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_SMALL_M(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_SMALL_N(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_SMALL_O(LDPC_SPEC_KERNEL_DECL)
LDPC_SPEC_GRAPHS_SMALL_P(LDPC_SPEC_KERNEL_DECL)
#undef LDPC_SPEC_KERNEL_DECL
int spec_waves(int id); /* ldpc_graph.cpp */
long quad_table_offset(int id);

/* host launch stub of specialised kernel `id` (core: this unit; mid: ldpc_spec_kernels_*.hip) */
const void* spec_kernel_ptr(int id)
{
#define LDPC_SPEC_KERNEL(id, bg, z, ils) reinterpret_cast<const void*>(&ldpc_decode_kernel<true, id>),
#define LDPC_SPEC_KERNEL_EXT(id, bg, z, ils) spec_kernel_##id(),
  static const void* const spec_kernels[] = {
      LDPC_SPEC_GRAPHS_CORE(LDPC_SPEC_KERNEL) LDPC_SPEC_GRAPHS_MID_A(LDPC_SPEC_KERNEL_EXT)
          LDPC_SPEC_GRAPHS_MID_B(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_MID_C(LDPC_SPEC_KERNEL_EXT)
              LDPC_SPEC_GRAPHS_MID_D(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_MID_E(LDPC_SPEC_KERNEL_EXT)
                  LDPC_SPEC_GRAPHS_MID_F(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_MID_G(LDPC_SPEC_KERNEL_EXT)
                      LDPC_SPEC_GRAPHS_MID_H(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_I(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_J(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_K(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_L(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_M(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_N(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_O(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_P(LDPC_SPEC_KERNEL_EXT)};
#undef LDPC_SPEC_KERNEL
#undef LDPC_SPEC_KERNEL_EXT
  static_assert(sizeof(spec_kernels) / sizeof(spec_kernels[0]) == spec::NOF_SPECS, "specialised kernel table");
  return (id >= 0 && id < spec::NOF_SPECS) ? spec_kernels[id] : nullptr;
}

/* host launch stub of the split-row address table writer of specialised graph `id` */
const void* spec_split_kernel_ptr(int id)
{
#define LDPC_SPEC_KERNEL(id, bg, z, ils) reinterpret_cast<const void*>(&ldpc_split_table_kernel<id>),
#define LDPC_SPEC_KERNEL_EXT(id, bg, z, ils) spec_split_kernel_##id(),
  static const void* const split_kernels[] = {
      LDPC_SPEC_GRAPHS_CORE(LDPC_SPEC_KERNEL) LDPC_SPEC_GRAPHS_MID_A(LDPC_SPEC_KERNEL_EXT)
          LDPC_SPEC_GRAPHS_MID_B(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_MID_C(LDPC_SPEC_KERNEL_EXT)
              LDPC_SPEC_GRAPHS_MID_D(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_MID_E(LDPC_SPEC_KERNEL_EXT)
                  LDPC_SPEC_GRAPHS_MID_F(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_MID_G(LDPC_SPEC_KERNEL_EXT)
                      LDPC_SPEC_GRAPHS_MID_H(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_I(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_J(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_K(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_L(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_M(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_N(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_O(LDPC_SPEC_KERNEL_EXT) LDPC_SPEC_GRAPHS_SMALL_P(LDPC_SPEC_KERNEL_EXT)};
#undef LDPC_SPEC_KERNEL
#undef LDPC_SPEC_KERNEL_EXT
  static_assert(sizeof(split_kernels) / sizeof(split_kernels[0]) == spec::NOF_SPECS, "split table writer table");
  return (id >= 0 && id < spec::NOF_SPECS) ? split_kernels[id] : nullptr;
}

/* The split-row address tables of every specialised BG1 graph into the context's table buffer (d_tables), one
 * workgroup per graph; spec_ids[p] = the specialised id of BG1 lifting size p, or -1. Synchronous (context open). */
hipError_t write_split_tables(uint32_t* d_tables, const int* spec_ids, hipStream_t stream)
{
  /* the one-wave graphs' lane-split address tables (their graphs have no split-row table) */
  for (int id = 0; id != spec::NOF_SPECS; ++id) {
    const long off = quad_table_offset(id);
    if (off < 0) {
      continue;
    }
    auto* k = reinterpret_cast<void (*)(uint32_t*)>(const_cast<void*>(spec_split_kernel_ptr(id)));
    hipLaunchKernelGGL(k, dim3(1), dim3(64 * spec_waves(id)), 0, stream, d_tables + off);
    if (hipGetLastError() != hipSuccess) {
      return hipErrorLaunchFailure;
    }
  }
  for (int p = 0; p != 51; ++p) {
    if (spec_ids[p] < 0 || quad_table_offset(spec_ids[p]) >= 0) {
      continue;
    }
    auto* k = reinterpret_cast<void (*)(uint32_t*)>(const_cast<void*>(spec_split_kernel_ptr(spec_ids[p])));
    hipLaunchKernelGGL(k, dim3(1), dim3(64 * spec_waves(spec_ids[p])), 0, stream,
                       d_tables + SPLIT_TAB_OFFSET + p * SPLIT_TAB_STRIDE);
    if (hipGetLastError() != hipSuccess) {
      return hipErrorLaunchFailure;
    }
  }
  return hipStreamSynchronize(stream);
}

hipError_t launch_decode(bool sf08, int spec, const dec_cb* d_cbs, uint32_t n, int graph_slot,
                         const step_task* tasks, const lds_layout& lay, int block, const int8_t* llr, uint8_t* out,
                         ldpc_hip_cb_result* res, const uint32_t* d_crc, hipStream_t stream, const dec_cb* host_one,
                         const dematch_cb* d_dm, const dematch_cb* host_dm_one, uint32_t dm_lds)
{
  if (n == 0) {
    return hipSuccess;
  }
  /* one CB with its descriptor on the host: passed by value, the kernel reads no descriptor table */
  const bool   inl = host_one != nullptr && n == 1;
  const dec_cb one = inl ? *host_one : dec_cb{};
  /* fused dematcher (d_dm or, one CB, its descriptor by value): its staging (and tables) need dm_lds
   * (dm_fused_budget; 0: DM_FUSED_LDS) */
  const bool       dm_inl = host_dm_one != nullptr && n == 1;
  const bool       fused  = d_dm != nullptr || dm_inl;
  const dematch_cb dm_one = dm_inl ? *host_dm_one : dematch_cb{};
  const uint32_t   lds    = fused ? std::max(lay.total, dm_lds != 0 ? dm_lds : DM_FUSED_LDS) : lay.total;
  using kernel_fn = void (*)(const dec_cb*, dec_cb, int, const step_task*, lds_layout, const int8_t*, uint8_t*,
                             ldpc_hip_cb_result*, const uint32_t*, const dematch_cb*, dematch_cb);
  if (spec >= spec::NOF_SPECS || (spec >= 0 && (block != 64 * spec_waves(spec) || !sf08))) {
    return hipErrorInvalidValue; /* a specialised kernel: its own wave count, scaling factor 0.8 */
  }
  kernel_fn k = spec >= 0 ? reinterpret_cast<kernel_fn>(const_cast<void*>(spec_kernel_ptr(spec)))
                          : (sf08 ? &ldpc_decode_kernel<true, -1> : &ldpc_decode_kernel<false, -1>);
  hipLaunchKernelGGL(k, dim3(n), dim3(block), lds, stream, inl ? nullptr : d_cbs, one, graph_slot, tasks, lay, llr,
                     out, res, d_crc, dm_inl ? nullptr : d_dm, dm_one);
  return hipGetLastError();
}

hipError_t launch_decode_mixed(bool sf08, const dec_cb* d_cbs, uint32_t n, const mixed_group* d_groups,
                               uint32_t ngroups, uint32_t lds_bytes, const step_task* tasks, const int8_t* llr,
                               uint8_t* out, ldpc_hip_cb_result* res, const uint32_t* d_crc, hipStream_t stream,
                               const dematch_cb* d_dm, uint32_t dm_lds)
{
  if (n == 0) {
    return hipSuccess;
  }
  auto* k = sf08 ? &ldpc_decode_mixed_kernel<true> : &ldpc_decode_mixed_kernel<false>;
  hipLaunchKernelGGL(k, dim3(n), dim3(MIXED_BLOCK),
                     d_dm != nullptr ? std::max(lds_bytes, dm_lds != 0 ? dm_lds : DM_FUSED_LDS) : lds_bytes,
                     stream, d_cbs, d_groups, ngroups, tasks, llr, out, res, d_crc, d_dm);
  return hipGetLastError();
}

hipError_t upload_graphs(const graph_desc* graphs, int n)
{
  return hipMemcpyToSymbol(HIP_SYMBOL(c_graphs), graphs, sizeof(graph_desc) * static_cast<size_t>(n));
}

hipError_t launch_tb_join(const tbj_block* d_blocks, uint32_t nblocks, const uint8_t* msgs, ldpc_hip_cb_result* cb,
                          uint8_t* tb, ldpc_hip_tb_result* res, const uint32_t* d_crc, uint32_t* d_work,
                          hipStream_t stream)
{
  if (nblocks == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ldpc_tb_join_kernel, dim3(nblocks), dim3(TBJ_THREADS), 0, stream, d_blocks, msgs, cb, tb, res,
                     d_crc, d_work);
  return hipGetLastError();
}

hipError_t launch_encode(const enc_cb* d_cbs, uint32_t n, const uint8_t* msg, uint8_t* cw, const uint32_t* d_crc,
                         hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ldpc_encode_kernel, dim3(n), dim3(ENC_THREADS), 0, stream, d_cbs, msg, cw, d_crc);
  return hipGetLastError();
}

hipError_t launch_pdsch_encode(const pdsch_enc_cb* d_cbs, const pdsch_enc_cb* host_one, uint32_t n,
                               const uint8_t* msg, uint8_t* out, const uint32_t* d_crc, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  const bool inl = host_one != nullptr && n == 1;
  hipLaunchKernelGGL(ldpc_pdsch_encode_kernel, dim3(n), dim3(ENC_THREADS), 0, stream, inl ? nullptr : d_cbs,
                     inl ? *host_one : pdsch_enc_cb{}, msg, out, d_crc);
  return hipGetLastError();
}

hipError_t launch_rate_match(const ratematch_cb* d_cbs, uint32_t n, const uint8_t* cw, uint8_t* out,
                             hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ldpc_rate_match_kernel, dim3(n), dim3(256), 0, stream, d_cbs, cw, out);
  return hipGetLastError();
}

hipError_t launch_dematch(const dematch_cb* d_cbs, uint32_t n, const demod_tables& tab, hipStream_t stream,
                          const dematch_cb* host_one)
{
  if (n == 0) {
    return hipSuccess;
  }
  const bool       inl = host_one != nullptr && n == 1; /* one CB: descriptor by value */
  const dematch_cb one = inl ? *host_one : dematch_cb{};
  hipLaunchKernelGGL(ldpc_rate_dematch_kernel, dim3(n), dim3(DM_THREADS), 0, stream, inl ? nullptr : d_cbs, one, tab);
  return hipGetLastError();
}

/* ---- soft demodulation mapper -------------------------------------------------------------
 * demodulation_mapper::demodulate_soft (demodulation_mapper_impl.cpp:78-106) with the reference's portable scalar
 * per-symbol functions: BPSK / pi/2-BPSK (demodulation_mapper_impl.cpp:33-76), QPSK (demodulation_mapper_qpsk.cpp:
 * 133-169), 16-QAM (demodulation_mapper_qam16.cpp:201-273), 64-QAM and 256-QAM by interval functions
 * (demodulation_mapper_intervals.h:33-63, demodulation_mapper_qam64.cpp:382-463, demodulation_mapper_qam256.cpp:
 * 346-427), then log_likelihood_ratio::quantize (log_likelihood_ratio.cpp:88-97). Float arithmetic in the
 * reference's order without contraction, divisions correctly rounded (HIP's default), so the LLRs equal the CPU
 * restatement's bit for bit. One thread per symbol, Qm LLR bytes per thread: HBM-bound (8 + 4 B in, Qm B out). */
template <int MOD>
__device__ __forceinline__ void dm_segment(const demod_seg& sg, uint32_t i, const demod_tables& tab,
                                           const float2* __restrict__ sym_base, const float* __restrict__ nv_base,
                                           int8_t* __restrict__ llr_base)
{
  constexpr int QM = (MOD <= 1) ? 1 : MOD;
  int8_t        o[8];
  dm_symbol<MOD>(sym_base[sg.sym_offset + i], nv_base[sg.noise_offset + i], i, tab, o);
  int8_t*         out = llr_base + sg.llr_offset + static_cast<uint64_t>(i) * QM;
  const uintptr_t a   = reinterpret_cast<uintptr_t>(llr_base + sg.llr_offset); /* segment-uniform alignment */
  auto            b   = [&](int k) { return static_cast<uint32_t>(static_cast<uint8_t>(o[k])); };
  if constexpr (QM == 8) {
    if ((a & 7U) == 0) {
      *reinterpret_cast<uint2*>(out) = make_uint2(b(0) | b(1) << 8 | b(2) << 16 | b(3) << 24,
                                                  b(4) | b(5) << 8 | b(6) << 16 | b(7) << 24);
      return;
    }
  } else if constexpr (QM == 4) {
    if ((a & 3U) == 0) {
      *reinterpret_cast<uint32_t*>(out) = b(0) | b(1) << 8 | b(2) << 16 | b(3) << 24;
      return;
    }
  } else if constexpr (QM == 2 || QM == 6) {
    if ((a & 1U) == 0) {
#pragma unroll
      for (int k = 0; k < QM; k += 2) {
        reinterpret_cast<uint16_t*>(out)[k / 2] = static_cast<uint16_t>(b(k) | b(k + 1) << 8);
      }
      return;
    }
  }
#pragma unroll
  for (int k = 0; k < QM; ++k) {
    out[k] = o[k];
  }
}

__global__ void __launch_bounds__(DEMOD_BLOCK)
    ldpc_demodulate_kernel(const demod_seg* __restrict__ segs, uint32_t nseg, demod_tables tab,
                           const float2* __restrict__ sym_base, const float* __restrict__ nv_base,
                           int8_t* __restrict__ llr_base)
{
  __shared__ demod_tables s_tab;
  constexpr int           NW = static_cast<int>(sizeof(demod_tables) / 4);
  static_assert(NW <= DEMOD_BLOCK, "tables copied one word per thread");
  if (threadIdx.x < NW) {
    reinterpret_cast<uint32_t*>(&s_tab)[threadIdx.x] = reinterpret_cast<const uint32_t*>(&tab)[threadIdx.x];
  }
  /* segment of this block: the last one with block0 <= blockIdx.x (segments are in block order) */
  uint32_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (segs[mid].block0 <= blockIdx.x) {
      lo = mid;
    } else {
      hi = mid;
    }
  }
  const demod_seg sg = segs[lo];
  __syncthreads();
  const uint32_t i = (blockIdx.x - sg.block0) * DEMOD_BLOCK + threadIdx.x;
  if (i >= sg.nof_symbols) {
    return;
  }
  switch (sg.modulation) { /* block-uniform */
    case 0: dm_segment<0>(sg, i, s_tab, sym_base, nv_base, llr_base); break;
    case 1: dm_segment<1>(sg, i, s_tab, sym_base, nv_base, llr_base); break;
    case 2: dm_segment<2>(sg, i, s_tab, sym_base, nv_base, llr_base); break;
    case 4: dm_segment<4>(sg, i, s_tab, sym_base, nv_base, llr_base); break;
    case 6: dm_segment<6>(sg, i, s_tab, sym_base, nv_base, llr_base); break;
    default: dm_segment<8>(sg, i, s_tab, sym_base, nv_base, llr_base); break;
  }
}

hipError_t launch_demodulate(const demod_seg* d_segs, uint32_t nseg, uint32_t nblocks, const demod_tables& tab,
                             const float* d_sym, const float* d_nv, int8_t* d_llr, hipStream_t stream)
{
  if (nblocks == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ldpc_demodulate_kernel, dim3(nblocks), dim3(DEMOD_BLOCK), 0, stream, d_segs, nseg, tab,
                     reinterpret_cast<const float2*>(d_sym), d_nv, d_llr);
  return hipGetLastError();
}

#if defined(LDPC_HIP_DIAG) || defined(LDPC_HIP_DIAG_PHASE) || defined(LDPC_HIP_DIAG_TBJ) || defined(LDPC_HIP_DIAG_DM)
extern "C" int ldpc_hip_diag_read(uint64_t* out, uint32_t n)
{
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), n * sizeof(uint64_t)) == hipSuccess ? 0 : -2;
}
extern "C" int ldpc_hip_diag2_read(uint64_t* out, uint32_t n)
{
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag2), n * sizeof(uint64_t)) == hipSuccess ? 0 : -2;
}
#endif

hipError_t configure_kernels(uint32_t max_lds)
{
  std::vector<const void*> ks = {reinterpret_cast<const void*>(&ldpc_decode_kernel<true, -1>),
                                 reinterpret_cast<const void*>(&ldpc_decode_kernel<false, -1>),
                                 reinterpret_cast<const void*>(&ldpc_decode_mixed_kernel<true>),
                                 reinterpret_cast<const void*>(&ldpc_decode_mixed_kernel<false>)};
  for (int id = 0; id != spec::NOF_SPECS; ++id) {
    ks.push_back(spec_kernel_ptr(id));
  }
  for (const void* k : ks) {
    const hipError_t e =
        hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(max_lds));
    if (e != hipSuccess) {
      return e;
    }
  }
  return hipSuccess;
}

} // namespace ldpc_hip
