"""Transport-block side of the PUSCH decode path on the device.

pusch_decoder_impl joins the decoded codeblocks of a transport block on the host (join_and_notify /
concatenate_codeblocks, pusch_decoder_impl.cpp:384-497). tb_join keeps that step on the GPU: the CB messages produced
by DecodePlan.launch stay in HBM, the data bits are concatenated into the TB buffer and the TB CRC24A is checked
against the checksum carried by the last CB (one CB: its CRC is the TB CRC). Only the TB and a 4-byte result cross
PCIe afterwards."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Sequence

from . import _lib
from ._lib import TbDesc, TbResult

__all__ = ["tb_join_spec", "tb_join_launch", "TbResult"]


@dataclass
class tb_join_spec:
    tbs: int               # transport block size in bits (multiple of 8)
    nof_cbs: int           # C
    cb_msg_bits: int       # K * Z
    nof_filler_bits: int   # F
    cb_crc_bits: int       # 24 when C > 1, the TB CRC length (16 / 24) when C = 1
    msg_offset: int        # byte offset of CB 0's message in the message buffer
    msg_stride: int        # bytes between consecutive CB messages
    result_index: int      # CB 0's entry in the CB result array
    tb_offset: int = 0     # byte offset of the TB in the TB buffer


def tb_join_descriptors(specs: Sequence[tb_join_spec]):
    """The ldpc_hip_tb_desc array of `specs` (build once, launch many times)."""
    arr = (TbDesc * max(1, len(specs)))()
    for i, s in enumerate(specs):
        d = arr[i]
        d.msg_offset, d.tb_offset, d.msg_stride = s.msg_offset, s.tb_offset, s.msg_stride
        d.tbs, d.result_index, d.nof_cbs = s.tbs, s.result_index, s.nof_cbs
        d.cb_msg_bits, d.nof_filler_bits, d.cb_crc_bits = s.cb_msg_bits, s.nof_filler_bits, s.cb_crc_bits
    return arr


def tb_join_launch(ctx: _lib.Context, specs, d_msgs: int, d_cb_results: int, d_tb: int,
                   d_tb_results: int, stream: int = 0, n: int = -1) -> None:
    """ldpc_hip_tb_join_launch: asynchronous on `stream` (0 = the context stream); all buffers are device pointers.
    d_tb_results receives one TbResult (4 bytes) per spec. `specs`: tb_join_spec list, or a prebuilt
    tb_join_descriptors() array with its length n."""
    if n < 0:
        n = len(specs)
        arr = tb_join_descriptors(specs)
    else:
        arr = specs
    rc = ctx.lib.ldpc_hip_tb_join_launch(ctx.handle, n, arr, d_msgs, d_cb_results, d_tb, d_tb_results,
                                         _lib.stream_arg(stream))
    _lib.check(ctx.handle, rc, "ldpc_hip_tb_join_launch")


# ---------------------------------------------------------------------------------------------------------------------
# Device-resident PUSCH slot: rate dematch -> LDPC decode -> transport-block join, all in HBM.
# ---------------------------------------------------------------------------------------------------------------------
@dataclass
class tb_slot_spec:
    """One transport block of a slot, with its RX segmentation (codeblock_metadata per CB, ldpc_segmenter_impl)."""
    tbs: int                     # TB size in bits
    base_graph: int
    lifting_size: int
    nof_filler_bits: int
    rm_lengths: Sequence[int]    # E_r per CB
    modulation_order: int        # Qm
    rv: int = 0
    new_data: bool = True
    Nref: int = 0
    max_iterations: int = 6
    use_early_stop: bool = True
    modulation: int = -1         # modulation_scheme of the codeword's symbols (upload_symbols); -1: the one of Qm

    @property
    def modulation_scheme(self) -> int:
        return self.modulation if self.modulation >= 0 else self.modulation_order

    @property
    def nof_cbs(self) -> int:
        return len(self.rm_lengths)

    @property
    def tb_crc_bits(self) -> int:
        return 16 if self.tbs <= 3824 else 24     # pusch_decoder_impl select_crc / TS 38.212 7.2.1


class SlotPipeline:
    """The PUSCH decode path of one slot on the device, mirroring pusch_decoder_impl (pusch_decoder_impl.cpp:
    309-497) with pusch_codeblock_decoder (pusch_codeblock_decoder.cpp:35-71) per CB:

      rate-dematch every CB's E LLRs into its N-LLR soft buffer (HARQ state, kept in HBM across launches)
      -> decode every CB (CRC early stop with CRC24B, or the TB CRC for a single-CB TB; or CRC after decoding)
      -> join each TB's codeblocks and check the TB CRC24A.

    Buffers are torch device tensors owned by the pipeline; upload() stages the slot's E-LLRs (one host-to-device
    copy), launch() enqueues the three kernels on a stream, results() reads the TB bytes and flags back."""

    def __init__(self, ctx: _lib.Context, tbs: Sequence[tb_slot_spec], fuse_dematch: bool = True):
        import numpy as np
        import torch

        from . import channel_coding as cc
        from . import channel_modulation
        from ._lib import (CRC16, CRC24A, CRC24B, CRC_MODE_CHECK_AFTER, CRC_MODE_EARLY_STOP, CRC_MODE_FLAG_KEEP_PASSED,
                           DematchDesc)

        self.ctx, self.tbs = ctx, list(tbs)
        dm, llr_off, soft_off, dec, joins = [], [], [], [], []
        lo = so = oo = to = 0
        self.tb_offsets, self.cb_llr_offsets = [], []
        self.demod_segments, self.tb_symbol_offsets = [], []
        symo = 0
        for tb in self.tbs:
            bg, Z, C = tb.base_graph, tb.lifting_size, tb.nof_cbs
            N = cc.BG_N_SHORT[bg] * Z
            mbytes = cc.message_bytes(bg, Z)
            stride = (mbytes + 15) // 16 * 16
            crc_poly = CRC24B if C > 1 else (CRC24A if tb.tb_crc_bits == 24 else CRC16)
            # a retransmission skips the CBs whose CRC already passed (pusch_decoder_impl.cpp:336-346); new data
            # decodes every CB, and the decoder's fresh result records replace the old flags (no clearing pass)
            mode = (CRC_MODE_EARLY_STOP if tb.use_early_stop else CRC_MODE_CHECK_AFTER) | \
                (0 if tb.new_data else CRC_MODE_FLAG_KEEP_PASSED)
            first_res, first_out = len(dec), oo
            offs = []
            self.tb_symbol_offsets.append(symo)
            for E in tb.rm_lengths:
                # the CB's E LLRs are the soft demodulation of its E / Qm symbols of the codeword
                self.demod_segments.append(channel_modulation.demod_segment(E // tb.modulation_order,
                                                                            tb.modulation_scheme, symo, symo, lo))
                symo += E // tb.modulation_order
                d = DematchDesc()
                d.modulation_order, d.rv, d.new_data = tb.modulation_order, tb.rv, 1 if tb.new_data else 0
                d.cb_length, d.rm_length, d.Nref, d.nof_filler_bits = N, E, tb.Nref, tb.nof_filler_bits
                dm.append(d)
                llr_off.append(lo)
                soft_off.append(so)
                offs.append(lo)
                dec.append(cc.cb_decode_spec(bg, Z, N, tb.max_iterations, mode, crc_poly, tb.nof_filler_bits, 0.8,
                                             so, oo))
                lo += (E + 15) // 16 * 16
                so += (N + 15) // 16 * 16
                oo += stride
            self.cb_llr_offsets.append(offs)
            joins.append(tb_join_spec(tb.tbs, C, cc.BG_K[bg] * Z, tb.nof_filler_bits, 24 if C > 1 else tb.tb_crc_bits,
                                      first_out, stride, first_res, to))
            self.tb_offsets.append(to)
            to += (tb.tbs // 8 + 15) // 16 * 16
        self.nof_cbs = len(dec)
        self._dm = (DematchDesc * max(1, len(dm)))(*dm)
        self._llr_off = (ctypes.c_uint64 * max(1, len(llr_off)))(*llr_off)
        self._soft_off = (ctypes.c_uint64 * max(1, len(soft_off)))(*soft_off)
        self.plan = cc.DecodePlan(ctx, dec)
        self.joins = joins
        self._tb_arr = tb_join_descriptors(joins)
        dev = torch.device("cuda", ctx.device)
        self.h_llr = torch.zeros(max(16, lo), dtype=torch.int8).pin_memory()
        self.d_llr = torch.zeros(max(16, lo), dtype=torch.int8, device=dev)
        self.d_soft = torch.zeros(max(16, so), dtype=torch.int8, device=dev)     # HARQ soft buffers
        self.d_out = torch.zeros(max(16, oo), dtype=torch.uint8, device=dev)
        self.d_res = torch.zeros(max(1, len(dec)) * 4, dtype=torch.uint8, device=dev)
        self.d_tb = torch.zeros(max(16, to), dtype=torch.uint8, device=dev)
        self.d_tbres = torch.zeros(max(1, len(joins)) * 4, dtype=torch.uint8, device=dev)
        self._np = np
        self.nof_symbols = symo
        self._demod_arr = channel_modulation.demod_descriptors(self.demod_segments)
        self.d_sym = None          # complex symbols (float re, im) and noise variances, allocated by upload_symbols
        self.d_nv = None
        self.from_symbols = False
        self._graph = None         # ldpc_hip_graph of capture()
        # from symbols: demodulation fused into the dematcher when every CB's E fits its LDS staging
        self.fuse_demod = all(d.rm_length <= 32768 for d in dm)
        # the dematcher fused into the decode kernels (ldpc_hip_dematch_decode_launch): one kernel less per slot
        self.fuse_dematch = fuse_dematch

    def upload_symbols(self, symbols_per_tb, noise_vars_per_tb) -> None:
        """Stage the slot's equalised symbols instead of LLRs: symbols_per_tb[i] holds TB i's
        codeword symbols (complex64, sum(E_r) / Qm of them) and noise_vars_per_tb[i] one noise variance per symbol,
        as pusch_demodulator_impl hands them to demodulation_mapper::demodulate_soft. launch() then soft-demodulates
        every CB's symbols straight into the dematcher's input on the device."""
        import torch
        np = self._np
        h_sym = np.zeros(max(1, self.nof_symbols), np.complex64)
        h_nv = np.zeros(max(1, self.nof_symbols), np.float32)
        for o, tb, z, n in zip(self.tb_symbol_offsets, self.tbs, symbols_per_tb, noise_vars_per_tb):
            cnt = sum(tb.rm_lengths) // tb.modulation_order
            if len(z) != cnt or len(n) != cnt:
                raise ValueError(f"TB needs {cnt} symbols and noise variances")
            h_sym[o:o + cnt] = z
            h_nv[o:o + cnt] = n
        dev = torch.device("cuda", self.ctx.device)
        self.d_sym = torch.from_numpy(h_sym.view(np.float32)).to(dev)
        self.d_nv = torch.from_numpy(h_nv).to(dev)
        self.from_symbols = True

    def upload_symbols_device(self, symbols_per_tb, noise_vars_per_tb) -> None:
        """As upload_symbols(), from device tensors (complex64 symbols, float32 noise variances per TB)."""
        import torch
        dev = torch.device("cuda", self.ctx.device)
        self.d_sym = torch.zeros(2 * max(1, self.nof_symbols), dtype=torch.float32, device=dev)
        self.d_nv = torch.zeros(max(1, self.nof_symbols), dtype=torch.float32, device=dev)
        for o, tb, z, n in zip(self.tb_symbol_offsets, self.tbs, symbols_per_tb, noise_vars_per_tb):
            cnt = sum(tb.rm_lengths) // tb.modulation_order
            if z.numel() != cnt or n.numel() != cnt:
                raise ValueError(f"TB needs {cnt} symbols and noise variances")
            self.d_sym[2 * o:2 * (o + cnt)].copy_(torch.view_as_real(z.reshape(-1)).reshape(-1))
            self.d_nv[o:o + cnt].copy_(n.reshape(-1))
        self.from_symbols = True

    def upload(self, llrs_per_tb, stream=None) -> None:
        """llrs_per_tb[i][r]: int8 E-LLRs of CB r of TB i (host arrays). One pinned host-to-device copy."""
        h = self.h_llr.numpy()
        for offs, llrs in zip(self.cb_llr_offsets, llrs_per_tb):
            for off, l in zip(offs, llrs):
                h[off:off + l.size] = l
        # blocking: the launch may go to the context's own non-blocking stream, which the default stream's copy does
        # not order (a non-blocking copy here once let a launch read the LLRs before they had landed)
        self.d_llr.copy_(self.h_llr)

    def upload_device(self, llrs_per_tb) -> None:
        """As upload(), from per-CB device int8 tensors (e.g. srsran_projectvtlmo_amd.synth): device-to-device."""
        import torch
        for offs, llrs in zip(self.cb_llr_offsets, llrs_per_tb):
            for off, l in zip(offs, llrs):
                self.d_llr[off:off + l.numel()].copy_(l.reshape(-1))
        torch.cuda.current_stream().synchronize()  # before a launch on another stream (see upload)

    def launch(self, stream: int = 0) -> None:
        """[Soft demodulation ->] dematch -> decode -> TB join on `stream` (dematch and decode one fused kernel unless
        fuse_dematch is off). CBs whose CRC passed in an earlier launch are only dematched (pusch_decoder_impl.cpp:
        336-346); new-data TBs decode every CB."""
        L, c = self.ctx.lib, self.ctx.handle
        if self.fuse_dematch:
            # each decoder workgroup dematches (and, from symbols, demodulates) its CB first: one launch
            if self.from_symbols and not self.fuse_demod:
                from . import channel_modulation
                channel_modulation.demodulate_launch(self.ctx, self._demod_arr, self.d_sym.data_ptr(),
                                                     self.d_nv.data_ptr(), self.d_llr.data_ptr(), stream,
                                                     n=len(self.demod_segments))
            sym = self.from_symbols and self.fuse_demod
            rc = L.ldpc_hip_dematch_decode_launch(
                self.plan.handle, self._dm, None if sym else self.d_llr.data_ptr(), None if sym else self._llr_off,
                self._demod_arr if sym else None, self.d_sym.data_ptr() if sym else None,
                self.d_nv.data_ptr() if sym else None, self.d_soft.data_ptr(), self.d_out.data_ptr(),
                self.d_res.data_ptr(), _lib.stream_arg(stream))
            _lib.check(c, rc, "ldpc_hip_dematch_decode_launch")
            tb_join_launch(self.ctx, self._tb_arr, self.d_out.data_ptr(), self.d_res.data_ptr(), self.d_tb.data_ptr(),
                           self.d_tbres.data_ptr(), stream, n=len(self.joins))
            return
        if self.from_symbols and self.fuse_demod:
            # each CB's symbols demodulated straight into the dematcher's LDS staging (no LLR round trip)
            rc = L.ldpc_hip_demod_dematch_launch(c, self.nof_cbs, self._dm, self._demod_arr, self.d_sym.data_ptr(),
                                                 self.d_nv.data_ptr(), self.d_soft.data_ptr(), self._soft_off,
                                                 _lib.stream_arg(stream))
            _lib.check(c, rc, "ldpc_hip_demod_dematch_launch")
        else:
            if self.from_symbols:
                from . import channel_modulation
                channel_modulation.demodulate_launch(self.ctx, self._demod_arr, self.d_sym.data_ptr(),
                                                     self.d_nv.data_ptr(), self.d_llr.data_ptr(), stream,
                                                     n=len(self.demod_segments))
            rc = L.ldpc_hip_rate_dematch_launch(c, self.nof_cbs, self._dm, self.d_llr.data_ptr(), self._llr_off,
                                                self.d_soft.data_ptr(), self._soft_off, _lib.stream_arg(stream))
            _lib.check(c, rc, "ldpc_hip_rate_dematch_launch")
        self.plan.launch(self.d_soft.data_ptr(), self.d_out.data_ptr(), self.d_res.data_ptr(), stream)
        tb_join_launch(self.ctx, self._tb_arr, self.d_out.data_ptr(), self.d_res.data_ptr(), self.d_tb.data_ptr(),
                       self.d_tbres.data_ptr(), stream, n=len(self.joins))

    def capture(self, stream: int) -> None:
        """Record launch() on `stream` as one HIP graph (ldpc_hip_capture_begin / _end); launch_graph() then replays
        the whole slot with one submission. The slot is launched once first so that every descriptor is resident.
        The graph works on this pipeline's buffers: a later upload() feeds the next replay."""
        import torch
        if not stream:
            raise ValueError("capture() needs an explicit (non-null) stream")
        self.release_graph()
        L, c = self.ctx.lib, self.ctx.handle
        ext = torch.cuda.ExternalStream(stream)
        with torch.cuda.stream(ext):           # any torch work inside launch() goes to the captured stream
            self.launch(stream)
            ext.synchronize()
            _lib.check(c, L.ldpc_hip_capture_begin(c, stream), "ldpc_hip_capture_begin")
            try:
                self.launch(stream)
            finally:
                g = ctypes.c_void_p()
                rc = L.ldpc_hip_capture_end(c, stream, ctypes.byref(g))
        _lib.check(c, rc, "ldpc_hip_capture_end")
        self._graph = g

    def launch_graph(self, stream: int) -> None:
        """One replay of the captured slot on `stream` (ldpc_hip_graph_launch)."""
        if not self._graph:
            raise RuntimeError("launch_graph() before capture()")
        _lib.check(self.ctx.handle, self.ctx.lib.ldpc_hip_graph_launch(self._graph, _lib.stream_arg(stream)),
                   "ldpc_hip_graph_launch")

    def release_graph(self) -> None:
        if getattr(self, "_graph", None):
            self.ctx.lib.ldpc_hip_graph_destroy(self._graph)
        self._graph = None

    def results(self):
        """[(tb_bytes, tb_crc_ok, written)], and the per-CB results array (n, 4) = crc_pass, iterations, status."""
        tb = self.d_tb.cpu().numpy()
        res = self.d_tbres.cpu().numpy().reshape(-1, 4)
        out = [(tb[o:o + s.tbs // 8].copy(), bool(res[i, 0]), bool(res[i, 1]))
               for i, (o, s) in enumerate(zip(self.tb_offsets, self.tbs))]
        return out, self.d_res.cpu().numpy().reshape(-1, 4)[: self.nof_cbs]
