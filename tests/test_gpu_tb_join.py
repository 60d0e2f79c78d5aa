"""GPU parity of the device transport-block join against the oracle restatement of
pusch_decoder_impl::join_and_notify / concatenate_codeblocks (pusch_decoder_impl.cpp:384-497).

Each TB goes through the device path end to end: codeword LLRs -> DecodePlan (CRC early stop: CRC24B per CB, or the
TB CRC for a single CB) -> tb_join, all in HBM. The checker decodes every CB with the oracle and joins with
oracle.tb_join; TB bytes, tb_crc_ok and whether the TB was written must match bit for bit."""
import numpy as np
import pytest

import oracle as O
from tests.tb_chain import TransportBlock

pytestmark = pytest.mark.gpu

HIP_CRC = {O.CRC16: 0, O.CRC24B: 1, O.CRC24A: 2}


def _run(hip_ctx, cases, seed):
    import torch
    from srsran_projectvtlmo_amd import channel_coding as cc
    from srsran_projectvtlmo_amd import pusch
    rng = np.random.default_rng(seed)
    specs, tb_specs, blobs, expect = [], [], [], []
    llr_off = out_off = tb_off = 0
    for tbs, bg, syms, amp, noise, corrupt in cases:
        tb = TransportBlock(rng, tbs, bg, syms, "QAM16", 2)
        K, Z, F, C = tb.K, tb.Z, tb.F, tb.C
        N = O.BG_N_SHORT[bg] * Z
        crc_poly = O.CRC24B if C > 1 else tb.tb_crc_poly
        cb_crc_bits = 24 if C > 1 else tb.tb_crc_len
        mbytes = (K * Z + 7) // 8
        stride = (mbytes + 15) // 16 * 16
        first_res = len(specs)
        msg_base = out_off
        ref_msgs = np.zeros((C, stride), np.uint8)
        ref_ok = []
        for r in range(C):
            cw = tb.cws[r]
            x = np.where(cw == 1, -amp, amp).astype(np.float32) + noise * rng.standard_normal(N).astype(np.float32)
            llr = O.quantize_array(x, 8.0)
            llr[cw == O.FILLER_BIT] = 127
            if corrupt and r == C // 2:
                llr[: 40 * Z] = -llr[: 40 * Z]     # make this CB fail
            specs.append(cc.cb_decode_spec(bg, Z, N, 8, cc.CRC_MODE_EARLY_STOP, HIP_CRC[crc_poly], F, 0.8, llr_off,
                                           out_off))
            blobs.append((llr_off, llr))
            out, it = O.ldpc_decode(bg, Z, llr, 8, crc_poly, F)
            ref_msgs[r, :mbytes] = out
            ref_ok.append(1 if it is not None else 0)
            llr_off += (N + 15) // 16 * 16
            out_off += stride
        tb_specs.append(pusch.tb_join_spec(tbs, C, K * Z, F, cb_crc_bits, msg_base, stride, first_res, tb_off))
        ref_tb = np.full((tbs + 7) // 8, 0xA5, np.uint8)
        _, ok = O.tb_join(ref_msgs, K * Z, F, cb_crc_bits, tbs, ref_ok, ref_tb)
        written = (C == 1 and ok) or (C > 1 and all(ref_ok))
        expect.append((tb_off, tbs, ref_tb, ok, written, tb))
        tb_off += (tbs // 8 + 15) // 16 * 16
    h_llr = np.zeros(llr_off, np.int8)
    for off, l in blobs:
        h_llr[off:off + l.size] = l
    d_llr = torch.from_numpy(h_llr).cuda()
    d_out = torch.zeros(out_off, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(len(specs) * 4, dtype=torch.uint8, device="cuda")
    d_tb = torch.full((tb_off,), 0xA5, dtype=torch.uint8, device="cuda")
    d_tbres = torch.zeros(len(tb_specs) * 4, dtype=torch.uint8, device="cuda")
    plan = cc.DecodePlan(hip_ctx, specs)
    stream = torch.cuda.current_stream().cuda_stream
    plan.launch(d_llr.data_ptr(), d_out.data_ptr(), d_res.data_ptr(), stream)
    pusch.tb_join_launch(hip_ctx, tb_specs, d_out.data_ptr(), d_res.data_ptr(), d_tb.data_ptr(), d_tbres.data_ptr(),
                         stream)
    torch.cuda.synchronize()
    plan.close()
    got_tb = d_tb.cpu().numpy()
    got_res = d_tbres.cpu().numpy().reshape(-1, 4)
    for i, (off, tbs, ref_tb, ok, written, tb) in enumerate(expect):
        assert bool(got_res[i, 0]) == ok, f"tb {i}: tb_crc_ok"
        assert bool(got_res[i, 1]) == written, f"tb {i}: written"
        np.testing.assert_array_equal(got_tb[off:off + tbs // 8], ref_tb, err_msg=f"tb {i}")
        if ok:
            assert np.array_equal(np.unpackbits(got_tb[off:off + tbs // 8]), tb.data)


def test_tb_join_clean_channel(hip_ctx):
    """C = 1 (CRC16 and CRC24A TBs) and multi-CB BG1/BG2 TBs at high SNR: every TB recovered, TB CRC24A passes."""
    _run(hip_ctx, [(256, 2, 624, 2.0, 0.5, False), (4000, 2, 3000, 2.0, 0.5, False),
                   (20496, 1, 10000, 2.0, 0.5, False), (9000, 2, 6000, 2.0, 0.5, False),
                   (60000, 1, 30000, 2.0, 0.5, False)], seed=11)


def test_tb_join_failed_codeblock_leaves_tb_untouched(hip_ctx):
    """One corrupted CB: its CRC fails, the TB is not written and tb_crc_ok is false, as in join_and_notify."""
    _run(hip_ctx, [(20496, 1, 10000, 2.0, 0.5, True), (4000, 2, 3000, 2.0, 0.5, True),
                   (9000, 2, 6000, 2.0, 0.5, False)], seed=12)


def _join_only(hip_ctx, tbs_list, corrupt, seed):
    """The join kernel alone on encoder-side CB messages (tests/tb_chain.TransportBlock), every CB flagged as passed:
    many 4 KiB chunks per TB. corrupt[i]: flip one data bit of TB i's middle CB while keeping its flag, so the CB
    CRCs pass and the TB CRC24A fails -- the false-positive path that resets the TB's CB flags
    (pusch_decoder_impl.cpp:423-428)."""
    import torch
    from srsran_projectvtlmo_amd import pusch
    rng = np.random.default_rng(seed)
    tb_specs, expect = [], []
    msgs_all, res_all = [], []
    out_off = tb_off = 0
    for i, (tbs, bg, syms) in enumerate(tbs_list):
        tb = TransportBlock(rng, tbs, bg, syms, "QAM256", 4)
        K, Z, F, C = tb.K, tb.Z, tb.F, tb.C
        mbytes = (K * Z + 7) // 8
        stride = (mbytes + 15) // 16 * 16
        m = np.zeros((C, stride), np.uint8)
        for r in range(C):
            bits = tb.msgs[r].copy()
            bits[bits == O.FILLER_BIT] = 0
            m[r, :mbytes] = np.packbits(bits)
        if corrupt[i]:
            m[C // 2, 5] ^= 0x10
        first = len(res_all)
        msgs_all.append((out_off, m))
        res_all += [1] * C
        tb_specs.append(pusch.tb_join_spec(tbs, C, K * Z, F, 24 if C > 1 else tb.tb_crc_len, out_off, stride, first,
                                           tb_off))
        ref_tb = np.full((tbs + 7) // 8, 0xA5, np.uint8)
        _, ok = O.tb_join(m[:, :mbytes], K * Z, F, 24 if C > 1 else tb.tb_crc_len, tbs, [1] * C, ref_tb)
        assert ok == (not corrupt[i])
        expect.append((tb_off, tbs, ref_tb, ok, first, C, tb))
        out_off += C * stride
        tb_off += (tbs // 8 + 15) // 16 * 16
    h_out = np.zeros(out_off, np.uint8)
    for off, m in msgs_all:
        h_out[off:off + m.size] = m.reshape(-1)
    h_res = np.zeros((len(res_all), 4), np.uint8)
    h_res[:, 0] = 1
    h_res[:, 1] = 1
    h_res[:, 2] = 1                                              # status: output written
    d_out = torch.from_numpy(h_out).cuda()
    d_res = torch.from_numpy(h_res.reshape(-1)).cuda()
    d_tb = torch.full((tb_off,), 0xA5, dtype=torch.uint8, device="cuda")
    d_tbres = torch.zeros(len(tb_specs) * 4, dtype=torch.uint8, device="cuda")
    pusch.tb_join_launch(hip_ctx, tb_specs, d_out.data_ptr(), d_res.data_ptr(), d_tb.data_ptr(), d_tbres.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got_tb = d_tb.cpu().numpy()
    got_res = d_tbres.cpu().numpy().reshape(-1, 4)
    got_cb = d_res.cpu().numpy().reshape(-1, 4)
    for i, (off, tbs, ref_tb, ok, first, C, tb) in enumerate(expect):
        assert bool(got_res[i, 0]) == ok, f"tb {i}: tb_crc_ok"
        np.testing.assert_array_equal(got_tb[off:off + tbs // 8], ref_tb, err_msg=f"tb {i}")
        if ok:
            assert np.array_equal(np.unpackbits(got_tb[off:off + tbs // 8]), tb.data)
            assert got_cb[first:first + C, 0].all()
        elif C > 1:
            assert not got_cb[first:first + C, 0].any(), f"tb {i}: CB flags not reset"


def test_tb_join_many_chunks(hip_ctx):
    """C4's 128-CB TB (TBS 1,078,248: 33 chunks), a 152-CB TB (TBS 1,277,992: 40 chunks) and small ones, clean
    and with a TB CRC failure behind passing CB CRCs: bytes, TB flags and the CB-flag reset vs oracle.tb_join."""
    cases = [(1078248, 1, 250 * 156 * 4), (1078248, 1, 250 * 156 * 4), (1277992, 1, 273 * 156 * 4),
             (256, 2, 156 * 4), (60000, 1, 40 * 156 * 4)]
    _join_only(hip_ctx, cases, [False, True, False, False, True], seed=21)
