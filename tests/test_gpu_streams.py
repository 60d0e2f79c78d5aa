"""The C ABI's stream argument with the special HIP handles, and the ordering it gives against torch's default stream.

Round 4 passed hipStreamLegacy ((hipStream_t)1) through to the runtime and a multi-group plan's fork crashed in it;
the ABI now maps hipStreamLegacy to the null stream and passes hipStreamPerThread ((hipStream_t)2) to the runtime,
which resolves it (ldpc_hip_api.cpp abi_stream; the probe of every runtime call the fork makes is
tools/ubench/stream_probe.hip). Every *_launch entry point and the multi-group fork run here on both handles,
bit-exact vs the oracle. The Python wrappers now join torch's current stream for a stream of 0 / None
(srsran_projectvtlmo_amd._lib.stream_arg) instead of synchronising it on the host; the last test pins the ordering
race that gave an all-zero encoder output and a wrong CRC flag in round 4: a launch queued right behind a large
default-stream fill of its own input and output."""
import numpy as np
import pytest

import oracle as O
from tests.vectors import codeword_llrs, random_llrs

pytestmark = pytest.mark.gpu

LEGACY, PER_THREAD = 1, 2
HIP_CRC = {O.NO_CRC: -1, O.CRC16: 0, O.CRC24B: 1, O.CRC24A: 2}


def _cases(rng, graphs):
    cases = []
    for bg, Z in graphs:
        cases.append((bg, Z, 4, O.NO_CRC, random_llrs(rng, O.BG_N_SHORT[bg] * Z, "mixed")))
        if O.BG_K[bg] * Z > 40:
            llr, _ = codeword_llrs(rng, bg, Z, 2.0, 1.1, crc=O.CRC24B)
            cases.append((bg, Z, 6, O.CRC24B, llr))
    return cases


def _decode(ctx, cases, stream, fill_first=False):
    import torch
    from srsran_projectvtlmo_amd import channel_coding as cc
    specs, offs = [], []
    lo = oo = 0
    for bg, Z, it, crc, llr in cases:
        mode = cc.CRC_MODE_NONE if crc == O.NO_CRC else cc.CRC_MODE_EARLY_STOP
        specs.append(cc.cb_decode_spec(bg, Z, llr.size, it, mode, HIP_CRC[crc], 0, 0.8, lo, oo))
        offs.append(lo)
        lo += (llr.size + 15) // 16 * 16
        oo += (cc.message_bytes(bg, Z) + 15) // 16 * 16
    h = np.zeros(lo, np.int8)
    for off, c in zip(offs, cases):
        h[off:off + c[4].size] = c[4]
    plan = cc.DecodePlan(ctx, specs)
    d_llr = torch.empty(lo, dtype=torch.int8, device="cuda")
    d_out = torch.empty(oo, dtype=torch.uint8, device="cuda")
    d_res = torch.empty(len(specs) * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    if fill_first:
        # a large fill queued first on the default stream, then this launch's own input copy and output fills:
        # launched on a stream that does not wait for them, the decoder would read a stale input and its outputs
        # would be overwritten after it
        big = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        big.fill_(7)
        big.add_(1)
    d_llr.copy_(torch.from_numpy(h).pin_memory(), non_blocking=True)
    d_out.fill_(0x5A)
    d_res.fill_(0xEE)
    plan.launch(d_llr.data_ptr(), d_out.data_ptr(), d_res.data_ptr(), stream)
    torch.cuda.synchronize()
    plan.close()
    return specs, d_out.cpu().numpy(), d_res.cpu().numpy().reshape(-1, 4)


def _check(specs, cases, out, res):
    from srsran_projectvtlmo_amd import channel_coding as cc
    for i, (s, (bg, Z, it, crc, llr)) in enumerate(zip(specs, cases)):
        eo, er = O.ldpc_decode(bg, Z, llr, it, crc)
        nb = cc.message_bytes(bg, Z)
        np.testing.assert_array_equal(out[s.out_offset:s.out_offset + nb], eo, err_msg=f"cb {i} BG{bg} Z={Z}")
        assert (res[i, 0] == 1) == (er is not None), f"cb {i} BG{bg} Z={Z}: CRC flag"


@pytest.mark.parametrize("handle", [LEGACY, PER_THREAD])
def test_multi_group_fork_on_special_handle(handle):
    """A plan of many (BG, Z) groups launched per group on forked auxiliary streams (LDPC_HIP_LAUNCH_NO_MIXED: the fork
    records an event on the caller's stream, the auxiliary streams wait for it, and the caller's stream waits for
    theirs) on the special handle: bit-exact vs the oracle. This is the path that crashed in round 4."""
    from srsran_projectvtlmo_amd import _lib
    ctx = _lib.Context(0, launch_flags=_lib.LAUNCH_NO_MIXED)
    try:
        rng = np.random.default_rng(500 + handle)
        cases = _cases(rng, [(1, 384), (2, 208), (1, 36), (2, 52), (1, 7), (2, 96), (1, 144), (2, 15)])
        specs, out, res = _decode(ctx, cases, handle)
        _check(specs, cases, out, res)
    finally:
        ctx.close()


@pytest.mark.parametrize("handle", [LEGACY, PER_THREAD])
def test_every_launch_entry_point_on_special_handle(hip_ctx, handle):
    """The slot pipeline's entry points (fused demod/dematch + decode, separate dematch launch, decode launch, TB
    join) on the special handle, against the oracle's pusch_decoder_impl flow; the encoder and rate matcher launches
    against the oracle's; and capture refused on it (a default stream cannot be captured)."""
    import torch
    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    from srsran_projectvtlmo_amd import pusch
    from tests.tb_chain import SwFlow, TransportBlock
    rng = np.random.default_rng(600 + handle)
    tbs = [TransportBlock(rng, 20496, 1, 156 * 24, "QAM64", 2), TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4)]
    for fuse in (True, False):
        specs = [pusch.tb_slot_spec(tb.tbs, tb.bg, tb.Z, tb.F, [m["rm_length"] for m in tb.metas], tb.Qm, 0, True,
                                    0, 6, True) for tb in tbs]
        pipe = pusch.SlotPipeline(hip_ctx, specs, fuse_dematch=fuse)
        llrs = [tb.llrs(rng, 0, 2.5, 0.8) for tb in tbs]
        pipe.upload(llrs)
        pipe.launch(handle)
        torch.cuda.synchronize()
        got, cbres = pipe.results()
        for tb, l, (tb_bytes, ok, _w) in zip(tbs, llrs, got):
            exp_ok, _ = SwFlow(tb, nof_iters=6, early_stop=True).transmission(l, 0, True)
            assert ok == exp_ok
            if ok:
                assert np.array_equal(np.unpackbits(tb_bytes)[: tb.tbs], tb.data)
        with pytest.raises(_lib.LdpcHipError):
            _lib.check(hip_ctx.handle, hip_ctx.lib.ldpc_hip_capture_begin(hip_ctx.handle, handle), "capture_begin")
    # encoder + rate matcher launches
    bg, Z, F = 2, 36, 88
    msg = rng.integers(0, 2, O.BG_K[bg] * Z).astype(np.uint8)
    msg[-F:] = O.FILLER_BIT
    N = O.BG_N_SHORT[bg] * Z
    ref = O.ldpc_encode(bg, Z, msg, N)
    d_msg = torch.from_numpy(np.packbits(np.where(msg == O.FILLER_BIT, 0, msg)).astype(np.uint8)).cuda()
    d_cw = torch.zeros((N + 7) // 8 + 16, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    cc.encode_launch(hip_ctx, [cc.cb_encode_spec(bg, Z, N, 0, 0)], d_msg.data_ptr(), d_cw.data_ptr(), handle)
    E = 1248
    d_rm = torch.zeros((E + 7) // 8 + 16, dtype=torch.uint8, device="cuda")
    cc.rate_match_launch(hip_ctx, [cc.cb_rate_match_spec(N, E, 2, 0, 0, F, 0, 0)], d_cw.data_ptr(), d_rm.data_ptr(),
                         handle)
    torch.cuda.synchronize()
    bits = np.unpackbits(d_cw.cpu().numpy())[:N]
    np.testing.assert_array_equal(bits, np.where(ref == O.FILLER_BIT, 0, ref))
    np.testing.assert_array_equal(np.unpackbits(d_rm.cpu().numpy())[:E], O.rate_match(ref, E, 0, 2, 0, bg, Z))


def test_default_stream_launch_ordered_behind_fill():
    """Deterministic form of round 4's ordering race: behind a 1 GiB fill and add on torch's default stream, the
    launch's input copy and output fills are queued, then the decode is launched with stream 0 (the wrappers' "torch's
    current stream", the null stream through hipStreamLegacy). Every output and CRC flag equals the oracle's: the
    launch ran after the copy and the fills, not beside them. Multi-group (fork) and mixed plans both."""
    from srsran_projectvtlmo_amd import _lib
    rng = np.random.default_rng(700)
    cases = _cases(rng, [(1, 384), (2, 208), (2, 36), (1, 96)])
    for flags in (0, _lib.LAUNCH_NO_MIXED):
        ctx = _lib.Context(0, launch_flags=flags)
        try:
            specs, out, res = _decode(ctx, cases, 0, fill_first=True)
            _check(specs, cases, out, res)
        finally:
            ctx.close()
