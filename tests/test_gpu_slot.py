"""GPU parity of the device-resident PUSCH slot pipeline (rate dematch -> decode -> TB join, all in HBM;
srsran_projectvtlmo_amd.pusch.SlotPipeline) against the oracle restatement of pusch_decoder_impl +
pusch_codeblock_decoder (tests/tb_chain.SwFlow): per-CB CRC flags and iteration counts, TB CRC, TB bytes.
Covers a mixed BG1/BG2 slot in the shape of C4 at reduced size, and HARQ soft combining
across an RV {0, 2} retransmission kept in the pipeline's HBM soft buffers."""
import numpy as np
import pytest

import oracle as O
from tests.tb_chain import QM, SwFlow, TransportBlock

pytestmark = pytest.mark.gpu


def _slot(hip_ctx, rng, ues, rvs, amp, noise, iters=6, fuse=True):
    from srsran_projectvtlmo_amd import pusch
    tbs = [TransportBlock(rng, tbs_, bg, syms, mod, layers) for (tbs_, bg, syms, mod, layers) in ues]
    specs = [pusch.tb_slot_spec(tb.tbs, tb.bg, tb.Z, tb.F, [m["rm_length"] for m in tb.metas], tb.Qm, rvs[0], True,
                                0, iters, True) for tb in tbs]
    pipe = pusch.SlotPipeline(hip_ctx, specs, fuse_dematch=fuse)
    flows = [SwFlow(tb, nof_iters=iters, early_stop=True) for tb in tbs]
    import torch
    for tx, rv in enumerate(rvs):
        for s in specs:
            s.rv, s.new_data = rv, tx == 0
        if tx:
            pipe = _respec(pipe, specs)
        llrs = [tb.llrs(rng, rv, amp, noise) for tb in tbs]
        pipe.upload(llrs)
        pipe.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got, cbres = pipe.results()
        expect = [f.transmission(l, rv, tx == 0) for f, l in zip(flows, llrs)]
        i = 0
        for t, (tb, f, (ok, _bits), (tb_bytes, g_ok, written)) in enumerate(zip(tbs, flows, expect, got)):
            for r in range(tb.C):
                assert bool(cbres[i + r, 0]) == f.crc_ok[r], f"tx {tx} tb {t} cb {r} crc"
                if f.crc_ok[r]:
                    assert cbres[i + r, 1] == f.iters_used[r], f"tx {tx} tb {t} cb {r} iterations"
            i += tb.C
            assert g_ok == ok, f"tx {tx} tb {t}: tb_crc_ok"
            if ok:
                assert np.array_equal(np.unpackbits(tb_bytes)[: tb.tbs], tb.data), f"tx {tx} tb {t}: data"
    return pipe


def _respec(pipe, specs):
    """Same slot layout, new RV / new_data: rebuild the descriptors but keep the HBM soft buffers (HARQ state)."""
    from srsran_projectvtlmo_amd import pusch
    nxt = pusch.SlotPipeline(pipe.ctx, specs, fuse_dematch=pipe.fuse_dematch)
    nxt.d_soft, nxt.d_out, nxt.d_res = pipe.d_soft, pipe.d_out, pipe.d_res
    return nxt


def test_slot_mixed_bg1_bg2(hip_ctx):
    """A C4-shaped slot at reduced size: one multi-CB 256QAM BG1 TB, small QPSK BG2 TBs (CRC16, filler bits)."""
    rng = np.random.default_rng(31)
    ues = [(40000, 1, 14000, "QAM256", 4)] + [(256, 2, 156 * 4, "QPSK", 4)] * 5 + [(3000, 2, 1500, "QAM16", 2)]
    _slot(hip_ctx, rng, ues, [0], amp=2.0, noise=0.7)


def test_slot_graph_replay(hip_ctx):
    """The slot recorded once as a HIP graph (ldpc_hip_capture_begin / _end) and replayed twice, on another stream and
    with the outputs cleared first: the same TB bytes, TB flags and per-CB results as the eager launch."""
    import torch
    rng = np.random.default_rng(33)
    ues = [(40000, 1, 14000, "QAM256", 4)] + [(256, 2, 156 * 4, "QPSK", 4)] * 3 + [(3000, 2, 1500, "QAM16", 2)]
    pipe = _slot(hip_ctx, rng, ues, [0], amp=2.0, noise=0.7)
    ref, ref_cb = pipe.results()
    stream = torch.cuda.Stream()
    pipe.capture(stream.cuda_stream)
    pipe.d_out.zero_()
    pipe.d_tb.zero_()
    pipe.d_tbres.zero_()
    torch.cuda.synchronize()
    for _ in range(2):
        pipe.launch_graph(stream.cuda_stream)
    torch.cuda.synchronize()
    got, got_cb = pipe.results()
    pipe.release_graph()
    np.testing.assert_array_equal(got_cb, ref_cb)
    for (a, a_ok, a_w), (b, b_ok, b_w) in zip(ref, got):
        assert (a_ok, a_w) == (b_ok, b_w)
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("qm", [8, 6, 4, 2])
def test_slot_fused_demodulation(hip_ctx, qm):
    """A slot fed with equalised symbols: soft demodulation fused into the dematcher (ldpc_hip_demod_dematch_launch)
    gives the same HARQ soft buffers, CB results and TB bytes as demodulate -> dematch through HBM, which the
    demodulator and dematcher parity tests pin to the oracle."""
    import torch
    from srsran_projectvtlmo_amd import pusch
    from srsran_projectvtlmo_amd import segmentation as S
    from srsran_projectvtlmo_amd import synth
    rng = np.random.default_rng(40 + qm)
    ues = [(60000, 1, 40 * 156 * 2, qm, 2)] + [(256, 2, 156 * 4, 2, 4)] * 2
    specs, syms = [], []
    for k, (tbs, bg, nsym, q, layers) in enumerate(ues):
        metas = S.segment_rx(tbs, bg, nsym, q, layers)
        m0 = metas[0]
        msgs = S.segment_tx(rng.integers(0, 2, tbs).astype(np.uint8), metas)
        specs.append(pusch.tb_slot_spec(tbs, bg, m0.lifting_size, m0.nof_filler_bits, [m.rm_length for m in metas],
                                        q, 0, True, 0, 6, True))
        syms.append(synth.rate_matched_symbols(hip_ctx, bg, m0.lifting_size, msgs, [m.rm_length for m in metas], q,
                                               0, m0.nof_filler_bits, 0.01 if q >= 6 else 0.1, seed=50 + k))
    got = []
    for fused in (False, True):
        pipe = pusch.SlotPipeline(hip_ctx, specs)
        pipe.upload_symbols_device([a for a, _ in syms], [b for _, b in syms])
        assert pipe.fuse_demod
        pipe.fuse_demod = fused
        pipe.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        tbs_, cbres = pipe.results()
        got.append((pipe.d_soft.cpu().numpy(), cbres, tbs_))
    np.testing.assert_array_equal(got[0][0], got[1][0])
    np.testing.assert_array_equal(got[0][1], got[1][1])
    for (a, a_ok, a_w), (b, b_ok, b_w) in zip(got[0][2], got[1][2]):
        assert (a_ok, a_w) == (b_ok, b_w)
        np.testing.assert_array_equal(a, b)
    assert got[1][1][:, 0].any()


@pytest.mark.parametrize("fuse", [True, False])
def test_slot_harq_retransmission(hip_ctx, fuse):
    """Low SNR first transmission (some CBs fail), RV 2 retransmission combined in the HBM soft buffers; the
    dematcher fused into the decode kernels (ldpc_hip_dematch_decode_launch) and as its own kernel."""
    rng = np.random.default_rng(32)
    ues = [(20000, 1, 6000, "QAM16", 2), (5000, 2, 2500, "QAM16", 2)]
    _slot(hip_ctx, rng, ues, [0, 2], amp=1.0, noise=1.3, fuse=fuse)


def test_slot_mixed_separate_dematch(hip_ctx):
    """The mixed slot with the dematcher as its own kernel (SlotPipeline(fuse_dematch=False))."""
    rng = np.random.default_rng(31)
    ues = [(40000, 1, 14000, "QAM256", 4)] + [(256, 2, 156 * 4, "QPSK", 4)] * 5 + [(3000, 2, 1500, "QAM16", 2)]
    _slot(hip_ctx, rng, ues, [0], amp=2.0, noise=0.7, fuse=False)


@pytest.mark.parametrize("fuse", [True, False])
def test_slot_long_codeblock_unstaged(hip_ctx, fuse):
    """A one-CB TB whose E (40,000 LLRs, wrapping the circular buffer) exceeds the dematcher's 32 KiB LDS staging: the
    dematcher gathers straight from global memory, fused into the decode kernel and as its own kernel; a
    retransmission combines into the soft buffer."""
    rng = np.random.default_rng(33)
    ues = [(8000, 1, 20000, "QPSK", 1)]
    _slot(hip_ctx, rng, ues, [0, 3], amp=1.0, noise=1.2, fuse=fuse)
