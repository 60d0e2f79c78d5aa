"""Soft demodulation mapper on the MI355X: the Python mirror of srsRAN's
`demodulation_mapper` interface (include/srsran/phy/upper/channel_modulation/demodulation_mapper.h:46-70) and of
`channel_modulation_factory::create_demodulation_mapper` (channel_modulation_factories.h:32-39), on top of the C ABI
(`ldpc_hip_demodulate_sync` / `ldpc_hip_demodulate_launch`, include/srsran_ldpc_hip.h).

The LLRs are those of the reference's portable per-symbol functions (demodulation_mapper_impl.cpp:33-76,
demodulation_mapper_{qpsk,qam16,qam64,qam256}.cpp scalar loops) bit for bit. There is no CPU fallback: without the HIP
library or a GPU the calls raise."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from enum import IntEnum
from typing import Optional, Sequence

import numpy as np

from . import _lib


class modulation_scheme(IntEnum):
    """include/srsran/ran/sch/modulation_scheme.h:39-52."""
    PI_2_BPSK = 0
    BPSK = 1
    QPSK = 2
    QAM16 = 4
    QAM64 = 6
    QAM256 = 8


def get_bits_per_symbol(mod: int) -> int:
    """modulation_scheme.h get_bits_per_symbol: 1 for (pi/2-)BPSK, else the scheme's value."""
    return 1 if int(mod) in (0, 1) else int(mod)


class demodulation_mapper:
    """demodulation_mapper.h:46-70."""

    def demodulate_soft(self, llrs: np.ndarray, symbols: np.ndarray, noise_vars: np.ndarray,
                        mod: modulation_scheme) -> None:
        raise NotImplementedError


class demodulation_mapper_hip(demodulation_mapper):
    """demodulate_soft on the GPU: host spans in, host LLRs out (one HIP round trip)."""

    def __init__(self, ctx: Optional[_lib.Context] = None):
        self.ctx = ctx if ctx is not None else _lib.default_context()

    def demodulate_soft(self, llrs, symbols, noise_vars, mod):
        sym = np.ascontiguousarray(symbols, dtype=np.complex64)
        nv = np.ascontiguousarray(noise_vars, dtype=np.float32)
        # demodulation_mapper_impl.cpp:82-83 (srsran_assert)
        if sym.size != nv.size:
            raise ValueError("Inputs symbols and noise_vars must have the same length.")
        if sym.size * get_bits_per_symbol(mod) != llrs.size or llrs.dtype != np.int8:
            raise ValueError("Input and output lengths are incompatible.")
        out = llrs if llrs.flags.c_contiguous else np.empty_like(llrs)
        _lib.check(self.ctx.handle,
                   _lib.load().ldpc_hip_demodulate_sync(self.ctx.handle, sym.size, int(mod), sym.ctypes.data,
                                                         nv.ctypes.data, out.ctypes.data),
                   "ldpc_hip_demodulate_sync")
        if out is not llrs:
            llrs[...] = out


class channel_modulation_factory:
    """channel_modulation_factories.h:32-39 (demodulation mapper only)."""

    def __init__(self, ctx: Optional[_lib.Context] = None):
        self.ctx = ctx

    def create_demodulation_mapper(self) -> demodulation_mapper:
        return demodulation_mapper_hip(self.ctx)


def create_channel_modulation_hip_factory(ctx: Optional[_lib.Context] = None) -> channel_modulation_factory:
    return channel_modulation_factory(ctx)


@dataclass
class demod_segment:
    """One ldpc_hip_demod_desc: offsets in symbols / floats / bytes from the launch's base pointers."""
    nof_symbols: int
    modulation: int
    symbol_offset: int = 0
    noise_offset: int = 0
    llr_offset: int = 0


def demod_descriptors(segments: Sequence[demod_segment]):
    """The ldpc_hip_demod_desc array of `segments` (build once, launch many times)."""
    arr = (_lib.DemodDesc * max(len(segments), 1))()
    for i, s in enumerate(segments):
        arr[i].symbol_offset = s.symbol_offset
        arr[i].noise_offset = s.noise_offset
        arr[i].llr_offset = s.llr_offset
        arr[i].nof_symbols = s.nof_symbols
        arr[i].modulation = int(s.modulation)
    return arr


def demodulate_launch(ctx: _lib.Context, segments, d_symbols: int, d_noise_vars: int, d_llrs: int,
                      stream: int = 0, n: int = -1) -> None:
    """ldpc_hip_demodulate_launch on device pointers (asynchronous on `stream`). `segments`: a sequence of
    demod_segment, or a prebuilt demod_descriptors() array with its length n."""
    if n < 0:
        n = len(segments)
        arr = demod_descriptors(segments)
    else:
        arr = segments
    _lib.check(ctx.handle,
               _lib.load().ldpc_hip_demodulate_launch(ctx.handle, n, arr, ctypes.c_void_p(d_symbols),
                                                      ctypes.c_void_p(d_noise_vars), ctypes.c_void_p(d_llrs),
                                                      ctypes.c_void_p(_lib.stream_arg(stream))),
               "ldpc_hip_demodulate_launch")
