"""Python mirror of srsRAN's channel-coding plugin surface for the LDPC decode path, backed by the HIP library.

Mirrors (same names, argument meaning and error behaviour):
  * ldpc_decoder / ldpc_decoder::configuration   include/srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h:37-75
  * ldpc_rate_dematcher                          include/srsran/phy/upper/channel_coding/ldpc/ldpc_rate_dematcher.h:35-56
  * codeblock_metadata                           include/srsran/phy/upper/codeblock_metadata.h:41-79
  * create_ldpc_decoder_factory_sw(type),        channel_coding_factories.h:52-77, channel_coding_factories.cpp:92-192
    create_ldpc_rate_dematcher_factory_sw(type)  (new type strings "hip" / "hip:<n>"; decoder type "auto" resolves
                                                 to the GPU when a gfx950 is visible, dematcher "auto" stays on the CPU)
  * crc_calculator (generator polynomial carrier) include/srsran/phy/upper/channel_coding/crc_calculator.h

Contract violations raise `LdpcHipError` (the reference aborts via srsran_assert). There is no CPU fallback.
`DecodePlan` is the batched device-resident path used for throughput (one HIP launch per (BG, Z) group).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (CRC16, CRC24A, CRC24B, CRC_MODE_EARLY_STOP, CRC_MODE_NONE, CbResult, DecDesc, DematchDesc,
                   LdpcHipError, STATUS_OUTPUT_WRITTEN)

BG1, BG2 = 1, 2
BG_K = {BG1: 22, BG2: 10}
BG_N_SHORT = {BG1: 66, BG2: 50}

# modulation_scheme -> bits per symbol (include/srsran/ran/sch/modulation_scheme.h)
MODULATION_BITS = {"BPSK": 1, "PI_2_BPSK": 1, "QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}


def message_bytes(bg: int, Z: int) -> int:
    return (BG_K[bg] * Z + 7) // 8


@dataclass
class tb_common_metadata:
    base_graph: int = BG1
    lifting_size: int = 2
    rv: int = 0
    mod: str = "BPSK"
    Nref: int = 0
    cw_length: int = 0


@dataclass
class cb_specific_metadata:
    full_length: int = 0
    rm_length: int = 0
    nof_filler_bits: int = 0
    cw_offset: int = 0
    nof_crc_bits: int = 16


@dataclass
class codeblock_metadata:
    tb_common: tb_common_metadata = field(default_factory=tb_common_metadata)
    cb_specific: cb_specific_metadata = field(default_factory=cb_specific_metadata)


@dataclass
class algorithm_details:
    max_iterations: int = 6
    scaling_factor: float = 0.8


@dataclass
class configuration:
    """ldpc_decoder::configuration."""
    block_conf: codeblock_metadata = field(default_factory=codeblock_metadata)
    algorithm_conf: algorithm_details = field(default_factory=algorithm_details)


class crc_calculator:
    """Carrier of a CRC generator polynomial (crc_generator_poly), as passed to ldpc_decoder::decode."""
    _POLY = {"CRC16": CRC16, "CRC24B": CRC24B, "CRC24A": CRC24A}

    def __init__(self, poly: str):
        if poly not in self._POLY:
            raise LdpcHipError(f"unsupported CRC polynomial {poly} for the LDPC decoder")
        self.poly = poly

    def get_generator_poly(self) -> str:
        return self.poly

    @property
    def hip_id(self) -> int:
        return self._POLY[self.poly]


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class ldpc_decoder:
    """Abstract interface (ldpc_decoder.h:37-75)."""

    def decode(self, output: np.ndarray, input: np.ndarray, crc: Optional[crc_calculator],
               cfg: configuration) -> Optional[int]:
        raise NotImplementedError


class ldpc_decoder_hip(ldpc_decoder):
    """ldpc_decoder on the MI355X: one decode() = one codeblock through ldpc_hip_decode_sync (latency path; the
    throughput path is DecodePlan / the HAL queue). `output` is the packed message buffer (bit_buffer storage,
    MSB-first, ceil(K*Z/8) bytes, modified in place); `input` is int8 LLRs."""

    def __init__(self, ctx: Optional[_lib.Context] = None):
        self.ctx = ctx or _lib.default_context()

    def decode(self, output, input, crc, cfg):
        bc = cfg.block_conf
        bg, Z = int(bc.tb_common.base_graph), int(bc.tb_common.lifting_size)
        llr = np.ascontiguousarray(input, dtype=np.int8)
        nb = message_bytes(bg, Z)
        if not (isinstance(output, np.ndarray) and output.dtype == np.uint8 and output.size == nb):
            raise LdpcHipError(f"The output size {getattr(output, 'size', None)} is not the message size {nb} bytes.")
        d = DecDesc()
        d.base_graph = bg
        d.max_iterations = int(cfg.algorithm_conf.max_iterations)
        d.crc_mode = CRC_MODE_NONE if crc is None else CRC_MODE_EARLY_STOP
        d.crc_poly = -1 if crc is None else crc.hip_id
        d.lifting_size = Z
        d.nof_filler_bits = int(bc.cb_specific.nof_filler_bits)
        d.llr_length = llr.size
        d.scaling_factor = float(cfg.algorithm_conf.scaling_factor)
        res = CbResult()
        ins = (ctypes.c_void_p * 1)(_ptr(llr))
        outs = (ctypes.c_void_p * 1)(_ptr(output))
        rc = self.ctx.lib.ldpc_hip_decode_sync(self.ctx.handle, 1, ctypes.byref(d), ins, outs, ctypes.byref(res))
        _lib.check(self.ctx.handle, rc, "ldpc_decoder_hip::decode")
        return int(res.nof_iterations) if res.crc_pass else None


class ldpc_rate_dematcher:
    """Abstract interface (ldpc_rate_dematcher.h:35-56)."""

    def rate_dematch(self, output: np.ndarray, input: np.ndarray, new_data: bool, cfg: codeblock_metadata) -> None:
        raise NotImplementedError


class ldpc_rate_dematcher_hip(ldpc_rate_dematcher):
    """ldpc_rate_dematcher on the MI355X (ldpc_hip_rate_dematch_sync). `output` (N int8 LLRs) is in/out."""

    def __init__(self, ctx: Optional[_lib.Context] = None):
        self.ctx = ctx or _lib.default_context()

    def rate_dematch(self, output, input, new_data, cfg):
        if not (isinstance(output, np.ndarray) and output.dtype == np.int8 and output.flags.c_contiguous):
            raise LdpcHipError("output must be a contiguous int8 array")
        llr = np.ascontiguousarray(input, dtype=np.int8)
        d = DematchDesc()
        d.modulation_order = MODULATION_BITS[cfg.tb_common.mod] if isinstance(cfg.tb_common.mod, str) else int(
            cfg.tb_common.mod)
        d.rv = int(cfg.tb_common.rv)
        d.new_data = 1 if new_data else 0
        d.cb_length = output.size
        d.rm_length = llr.size
        d.Nref = int(cfg.tb_common.Nref)
        d.nof_filler_bits = int(cfg.cb_specific.nof_filler_bits)
        softs = (ctypes.c_void_p * 1)(_ptr(output))
        ins = (ctypes.c_void_p * 1)(_ptr(llr) if llr.size else _ptr(np.zeros(1, np.int8)))
        rc = self.ctx.lib.ldpc_hip_rate_dematch_sync(self.ctx.handle, 1, ctypes.byref(d), softs, ins)
        _lib.check(self.ctx.handle, rc, "ldpc_rate_dematcher_hip::rate_dematch")


def hip_device_of(type_str: str) -> Optional[int]:
    """The GPU a factory type string selects: "hip" -> 0, "hip:<n>" -> n (one cell per GPU: the upper PHY of cell c is
    configured with ldpc_decoder_type = f"hip:{c % G}", multi_gpu.cell_to_device); None: not a HIP type."""
    if type_str == "hip":
        return 0
    if type_str.startswith("hip:") and type_str[4:].isdigit():
        return int(type_str[4:])
    return None


def hip_device_of_decoder_type(dec_type: str) -> Optional[int]:
    """ldpc_decoder_factory_sw::create's GPU branch (channel_coding_factories.cpp:100-124 + INTEGRATION.md 2.1): "hip"
    / "hip:<n>", and "auto" -- what du_low_config_translator.cpp:160-162 sets -- when ldpc_hip_auto_device() finds a
    gfx950 (else None: the reference's CPU decoders)."""
    if dec_type == "auto":
        dev = _lib.load().ldpc_hip_auto_device()
        return dev if dev >= 0 else None
    return hip_device_of(dec_type)


def decode_work(bg: int, Z: int, llr, max_iterations: int, early_stop: bool = False) -> int:
    """ldpc_hip_decode_work: a codeblock's decoder work (edges of its layers x Z x iterations, the layer count from its
    last non-zero LLR as ldpc_decoder_impl.cpp:97-114; with CRC early stop min(max_iterations, 2) iterations), the
    quantity the "auto" type splits CPU and GPU calls by. Host only (no GPU)."""
    import numpy as np
    a = np.ascontiguousarray(llr, dtype=np.int8)
    d = _lib.DecDesc()
    d.base_graph, d.lifting_size, d.max_iterations, d.llr_length = bg, Z, max_iterations, a.size
    d.crc_mode = CRC_MODE_EARLY_STOP if early_stop else CRC_MODE_NONE
    return int(_lib.load().ldpc_hip_decode_work(ctypes.byref(d), a.ctypes.data if a.size else None))


def auto_prefers_gpu(bg: int, Z: int, llr, max_iterations: int, early_stop: bool = False) -> bool:
    """ldpc_decoder_hip_auto's choice (the "auto" type with a GPU): the GPU at or above ldpc_hip_auto_min_work()."""
    return decode_work(bg, Z, llr, max_iterations, early_stop) >= int(_lib.load().ldpc_hip_auto_min_work())


def hip_device_of_dematcher_type(dematcher_type: str) -> Optional[int]:
    """ldpc_rate_dematcher_factory_sw::create's GPU branch: "hip" / "hip:<n>" only; "auto" keeps the CPU dematcher
    (its output is the caller's host soft buffer: on the GPU it would add an N-byte PCIe round trip per codeblock)."""
    return hip_device_of(dematcher_type)


class ldpc_decoder_factory:
    def __init__(self, dec_type: str):
        self.dec_type = dec_type

    def create(self) -> Optional[ldpc_decoder]:
        dev = hip_device_of_decoder_type(self.dec_type)
        if dev is None:
            return None  # the reference returns an empty pointer for unsupported types
        return ldpc_decoder_hip(_lib.default_context(dev))


class ldpc_rate_dematcher_factory:
    def __init__(self, dematcher_type: str):
        self.dematcher_type = dematcher_type

    def create(self) -> Optional[ldpc_rate_dematcher]:
        dev = hip_device_of_dematcher_type(self.dematcher_type)
        if dev is None:
            return None
        return ldpc_rate_dematcher_hip(_lib.default_context(dev))


def create_ldpc_decoder_factory_sw(dec_type: str) -> ldpc_decoder_factory:
    return ldpc_decoder_factory(dec_type)


def create_ldpc_rate_dematcher_factory_sw(dematcher_type: str) -> ldpc_rate_dematcher_factory:
    return ldpc_rate_dematcher_factory(dematcher_type)


# ---------------------------------------------------------------------------------------------------------------------
# Batched, device-resident decoding (the throughput path).
# ---------------------------------------------------------------------------------------------------------------------
@dataclass
class cb_decode_spec:
    base_graph: int
    lifting_size: int
    llr_length: int
    max_iterations: int
    crc_mode: int = CRC_MODE_NONE
    crc_poly: int = -1
    nof_filler_bits: int = 0
    scaling_factor: float = 0.8
    llr_offset: int = 0
    out_offset: int = 0


class DecodePlan:
    """A batch of codeblocks with uploaded descriptors (ldpc_hip_decode_plan_create). launch() is asynchronous on the
    given HIP stream and takes raw device pointers (e.g. torch tensor data_ptr())."""

    def __init__(self, ctx: _lib.Context, specs: Sequence[cb_decode_spec]):
        self.ctx = ctx
        self.n = len(specs)
        arr = (DecDesc * max(1, self.n))()
        for i, s in enumerate(specs):
            d = arr[i]
            d.base_graph = s.base_graph
            d.max_iterations = s.max_iterations
            d.crc_mode = s.crc_mode
            d.crc_poly = s.crc_poly
            d.lifting_size = s.lifting_size
            d.nof_filler_bits = s.nof_filler_bits
            d.llr_length = s.llr_length
            d.scaling_factor = s.scaling_factor
            d.llr_offset = s.llr_offset
            d.out_offset = s.out_offset
        h = ctypes.c_void_p()
        rc = ctx.lib.ldpc_hip_decode_plan_create(ctx.handle, self.n, arr, ctypes.byref(h))
        _lib.check(ctx.handle, rc, "ldpc_hip_decode_plan_create")
        self.handle = h

    def launch(self, d_llr: int, d_out: int, d_results: int = 0, stream: int = 0) -> None:
        rc = self.ctx.lib.ldpc_hip_decode_launch(self.handle, d_llr, d_out, d_results or None, _lib.stream_arg(stream))
        _lib.check(self.ctx.handle, rc, "ldpc_hip_decode_launch")

    def close(self):
        if getattr(self, "handle", None):
            self.ctx.lib.ldpc_hip_decode_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def uniform_batch_specs(n: int, bg: int, Z: int, max_iterations: int, llr_length: Optional[int] = None,
                        crc_mode: int = CRC_MODE_NONE, crc_poly: int = -1, nof_filler_bits: int = 0):
    """n identical CB specs laid out back to back: LLRs at i*llr_stride, messages at i*out_stride (16-B aligned)."""
    L = llr_length if llr_length is not None else BG_N_SHORT[bg] * Z
    llr_stride = (L + 15) // 16 * 16
    out_stride = (message_bytes(bg, Z) + 15) // 16 * 16
    specs = [cb_decode_spec(bg, Z, L, max_iterations, crc_mode, crc_poly, nof_filler_bits, 0.8, i * llr_stride,
                            i * out_stride) for i in range(n)]
    return specs, llr_stride, out_stride


def schedule_groups(bg: int, Z: int) -> int:
    return int(_lib.load().ldpc_hip_schedule_groups(bg, Z))


def specialised(bg: int, Z: int) -> int:
    """1 when (bg, Z) decodes with the compile-time-schedule kernel (csrc/ldpc_spec.h), 0 with the generic one."""
    return int(_lib.load().ldpc_hip_specialised(bg, Z))


# ---------------------------------------------------------------------------------------------------------------------
# Encoder and rate matcher on device buffers (ldpc_encoder / ldpc_rate_matcher).
# ---------------------------------------------------------------------------------------------------------------------
@dataclass
class cb_encode_spec:
    base_graph: int
    lifting_size: int
    cw_length: int          # shortened codeword bits to produce (<= N_short * Z)
    msg_offset: int = 0     # byte offset of the packed K*Z-bit message
    cw_offset: int = 0      # byte offset of the packed codeword


@dataclass
class cb_rate_match_spec:
    cb_length: int          # N = N_short * Z
    rm_length: int          # E
    modulation_order: int   # Qm
    rv: int = 0
    Nref: int = 0
    nof_filler_bits: int = 0
    cw_offset: int = 0
    out_offset: int = 0


def encode_launch(ctx: _lib.Context, specs: Sequence[cb_encode_spec], d_msgs: int, d_cws: int, stream: int = 0):
    """ldpc_encoder::encode for a batch of CBs (ldpc_hip_encode_launch), asynchronous on `stream`."""
    arr = (_lib.EncDesc * max(1, len(specs)))()
    for i, sp in enumerate(specs):
        arr[i].msg_offset, arr[i].cw_offset, arr[i].cw_length = sp.msg_offset, sp.cw_offset, sp.cw_length
        arr[i].lifting_size, arr[i].base_graph = sp.lifting_size, sp.base_graph
    rc = ctx.lib.ldpc_hip_encode_launch(ctx.handle, len(specs), arr, d_msgs, d_cws, _lib.stream_arg(stream))
    _lib.check(ctx.handle, rc, "ldpc_hip_encode_launch")


def rate_match_launch(ctx: _lib.Context, specs: Sequence[cb_rate_match_spec], d_cws: int, d_out: int,
                      stream: int = 0):
    """ldpc_rate_matcher::rate_match for a batch of CBs (ldpc_hip_rate_match_launch), asynchronous on `stream`."""
    arr = (_lib.RmDesc * max(1, len(specs)))()
    for i, sp in enumerate(specs):
        a = arr[i]
        a.cw_offset, a.out_offset, a.cb_length, a.rm_length = sp.cw_offset, sp.out_offset, sp.cb_length, sp.rm_length
        a.Nref, a.nof_filler_bits, a.modulation_order, a.rv = sp.Nref, sp.nof_filler_bits, sp.modulation_order, sp.rv
    rc = ctx.lib.ldpc_hip_rate_match_launch(ctx.handle, len(specs), arr, d_cws, d_out, _lib.stream_arg(stream))
    _lib.check(ctx.handle, rc, "ldpc_hip_rate_match_launch")
