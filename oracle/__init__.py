"""CPU ORACLE for the MI355X LDPC decode path -- TEST INFRASTRUCTURE ONLY.

ctypes/numpy wrapper around `oracle/ldpc_oracle.c`, the plain-C restatement of the reference algorithms (see
`oracle/ldpc_oracle.h` for per-function citations and the parity-pinning status: PARTIALLY PINNED by the
reference's in-source known-answer tests and round-trip properties; the reference's .dat fixtures are absent and
building/running the reference is denied).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may import this package, and only as the
checker. The product package `srsran_projectvtlmo_amd` never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "build" / "libldpc_oracle.so"

CRC24A, CRC24B, CRC24C, CRC16, CRC11, CRC6 = 0, 1, 2, 3, 4, 5
NO_CRC = -1
FILLER_BIT = 254

BG_K = {1: 22, 2: 10}
BG_M = {1: 46, 2: 42}
BG_N_SHORT = {1: 66, 2: 50}
LIFTING_SIZES = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44,
                 48, 52, 56, 60, 64, 72, 80, 88, 96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288,
                 320, 352, 384]


def build(force: bool = False) -> Path:
    """Compile the oracle with its Makefile (gcc). Building the checker is not using it."""
    if force or not _LIB_PATH.exists():
        subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(_LIB_PATH))
        i8p = ctypes.POINTER(ctypes.c_int8)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u16p = ctypes.POINTER(ctypes.c_uint16)
        U = ctypes.c_uint
        I = ctypes.c_int
        sig = {
            "orc_llr_add": (ctypes.c_int8, [ctypes.c_int8, ctypes.c_int8]),
            "orc_llr_sub": (ctypes.c_int8, [ctypes.c_int8, ctypes.c_int8]),
            "orc_llr_promotion_sum": (ctypes.c_int8, [ctypes.c_int8, ctypes.c_int8]),
            "orc_llr_quantize": (ctypes.c_int8, [ctypes.c_float, ctypes.c_float]),
            "orc_hard_decision": (I, [u8p, i8p, U]),
            "orc_crc_packed": (ctypes.c_uint32, [I, u8p, U]),
            "orc_crc_bytes": (ctypes.c_uint32, [I, u8p, U]),
            "orc_crc_bits": (ctypes.c_uint32, [I, u8p, U]),
            "orc_lifting_index": (I, [U]),
            "orc_lifting_position": (I, [U]),
            "orc_graph_row": (I, [I, U, U, u16p, u16p]),
            "orc_ldpc_decode": (I, [I, U, U, i8p, U, U, ctypes.c_float, I, u8p]),
            "orc_rate_dematch": (I, [i8p, U, i8p, U, I, U, U, U, U]),
            "orc_ldpc_encode": (I, [I, U, u8p, u8p, U]),
            "orc_rate_match": (I, [u8p, U, u8p, U, U, U, U, I, U]),
            "orc_pusch_cb_decode": (I, [u8p, i8p, U, i8p, U, I, I, U, U, U, U, U, I, I, U]),
            "orc_tb_join": (I, [u8p, U, U, U, U, U, U, u8p, u8p]),
            "orc_ldpc_decode_port": (I, [I, U, U, i8p, U, U, I, u8p]),
            "orc_crc_port": (ctypes.c_uint32, [I, u8p, U]),
            "orc_bench_port": (I, [I, U, i8p, U, U, U, U, ctypes.POINTER(ctypes.c_uint32),
                                   ctypes.POINTER(ctypes.c_double)]),
            "orc_demodulate_soft": (I, [I, U, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float), i8p]),
            "orc_bench_slot": (I, [ctypes.c_void_p, U, U, U, I, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_uint)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


# ---- LLR arithmetic ----------------------------------------------------------------------------------------------
def llr_add(a: int, b: int) -> int:
    return int(lib().orc_llr_add(a, b))


def llr_sub(a: int, b: int) -> int:
    return int(lib().orc_llr_sub(a, b))


def llr_promotion_sum(a: int, b: int) -> int:
    return int(lib().orc_llr_promotion_sum(a, b))


def llr_quantize(x: float, r: float) -> int:
    return int(lib().orc_llr_quantize(x, r))


def quantize_array(x: np.ndarray, r: float) -> np.ndarray:
    """Vectorised `log_likelihood_ratio::quantize` (log_likelihood_ratio.cpp:88-97), float32 arithmetic."""
    x = np.asarray(x, dtype=np.float32)
    r = np.float32(r)
    clipped = np.where(np.abs(x) > r, np.copysign(r, x), x).astype(np.float32)
    v = (clipped / r * np.float32(120)).astype(np.float32)
    # std::round: half away from zero
    return (np.sign(v) * np.floor(np.abs(v) + np.float32(0.5))).astype(np.int8)


def hard_decision(llr: np.ndarray):
    llr = np.ascontiguousarray(llr, dtype=np.int8)
    out = np.zeros((llr.size + 7) // 8, dtype=np.uint8)
    ok = lib().orc_hard_decision(_p(out, ctypes.c_uint8), _p(llr, ctypes.c_int8), llr.size)
    return out, bool(ok)


# ---- CRC -----------------------------------------------------------------------------------------------------------
def crc_packed(poly: int, packed: np.ndarray, nbits: int) -> int:
    packed = np.ascontiguousarray(packed, dtype=np.uint8)
    return int(lib().orc_crc_packed(poly, _p(packed, ctypes.c_uint8), nbits))


def crc_bits(poly: int, bits: np.ndarray) -> int:
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    return int(lib().orc_crc_bits(poly, _p(bits, ctypes.c_uint8), bits.size))


# ---- graph ---------------------------------------------------------------------------------------------------------
def lifting_index(Z: int) -> int:
    return int(lib().orc_lifting_index(Z))


def graph_row(bg: int, Z: int, m: int):
    cols = np.zeros(20, dtype=np.uint16)
    sh = np.zeros(20, dtype=np.uint16)
    d = lib().orc_graph_row(bg, Z, m, _p(cols, ctypes.c_uint16), _p(sh, ctypes.c_uint16))
    return cols[:d].tolist(), sh[:d].tolist()


# ---- decoder / dematcher ---------------------------------------------------------------------------------------------
def ldpc_decode(bg: int, Z: int, llr: np.ndarray, max_iterations: int, crc_poly: int = NO_CRC,
                nof_filler_bits: int = 0, scaling_factor: float = 0.8, out: np.ndarray | None = None):
    """Returns (packed message bytes, iterations-or-None). Mirrors ldpc_decoder::decode with a fresh object."""
    llr = np.ascontiguousarray(llr, dtype=np.int8)
    nbytes = (BG_K[bg] * Z + 7) // 8
    if out is None:
        out = np.zeros(nbytes, dtype=np.uint8)
    r = lib().orc_ldpc_decode(bg, Z, nof_filler_bits, _p(llr, ctypes.c_int8), llr.size, max_iterations,
                              scaling_factor, crc_poly, _p(out, ctypes.c_uint8))
    if r < 0:
        raise ValueError("oracle decoder: contract violation")
    return out, (r if r > 0 else None)


def rate_dematch(out: np.ndarray, llr_e: np.ndarray, new_data: bool, rv: int, Qm: int, Nref: int,
                 nof_filler_bits: int) -> np.ndarray:
    """In-place on `out` (HARQ soft buffer, N LLRs). Mirrors ldpc_rate_dematcher::rate_dematch."""
    assert out.dtype == np.int8 and out.flags.c_contiguous
    llr_e = np.ascontiguousarray(llr_e, dtype=np.int8)
    r = lib().orc_rate_dematch(_p(out, ctypes.c_int8), out.size, _p(llr_e, ctypes.c_int8), llr_e.size,
                               int(new_data), rv, Qm, Nref, nof_filler_bits)
    if r != 0:
        raise ValueError("oracle rate dematcher: contract violation")
    return out


def ldpc_encode(bg: int, Z: int, msg_bits: np.ndarray, cb_len: int | None = None) -> np.ndarray:
    msg_bits = np.ascontiguousarray(msg_bits, dtype=np.uint8)
    assert msg_bits.size == BG_K[bg] * Z
    if cb_len is None:
        cb_len = BG_N_SHORT[bg] * Z
    cw = np.zeros(cb_len, dtype=np.uint8)
    if lib().orc_ldpc_encode(bg, Z, _p(msg_bits, ctypes.c_uint8), _p(cw, ctypes.c_uint8), cb_len) != 0:
        raise ValueError("oracle encoder failed")
    return cw


def rate_match(cw_bits: np.ndarray, E: int, rv: int, Qm: int, Nref: int, bg: int, Z: int) -> np.ndarray:
    cw_bits = np.ascontiguousarray(cw_bits, dtype=np.uint8)
    out = np.zeros(E, dtype=np.uint8)
    if lib().orc_rate_match(_p(out, ctypes.c_uint8), E, _p(cw_bits, ctypes.c_uint8), cw_bits.size, rv, Qm, Nref,
                            bg, Z) != 0:
        raise ValueError("oracle rate matcher failed")
    return out


def pusch_cb_decode(soft_buf: np.ndarray, llr_e: np.ndarray, new_data: bool, bg: int, Z: int, rv: int, Qm: int,
                    Nref: int, nof_filler_bits: int, crc_poly: int, use_early_stop: bool, nof_iterations: int):
    """pusch_codeblock_decoder::decode: dematch into soft_buf then decode. Returns (packed, iterations-or-None)."""
    llr_e = np.ascontiguousarray(llr_e, dtype=np.int8)
    out = np.zeros((BG_K[bg] * Z + 7) // 8, dtype=np.uint8)
    r = lib().orc_pusch_cb_decode(_p(out, ctypes.c_uint8), _p(soft_buf, ctypes.c_int8), soft_buf.size,
                                  _p(llr_e, ctypes.c_int8), llr_e.size, int(new_data), bg, Z, rv, Qm, Nref,
                                  nof_filler_bits, crc_poly, int(use_early_stop), nof_iterations)
    if r < 0:
        raise ValueError("oracle pusch cb decode: contract violation")
    return out, (r if r > 0 else None)


def bench_port(bg: int, Z: int, llr: np.ndarray, max_iterations: int, threads: int, reps: int):
    """bench.py's CPU baseline loop (ldpc_cpu_bench.c): `threads` C threads, `reps` timed port decodes each.
    Returns (per-decode latencies in ns, shape (threads, reps); wall time of the run in s)."""
    llr = np.ascontiguousarray(llr, dtype=np.int8)
    lat = np.zeros((threads, reps), dtype=np.uint32)
    wall = ctypes.c_double(0.0)
    r = lib().orc_bench_port(bg, Z, _p(llr, ctypes.c_int8), llr.size, max_iterations, threads, reps,
                             _p(lat, ctypes.c_uint32), ctypes.byref(wall))
    if r < 0:
        raise ValueError("oracle bench_port: invalid argument or failed decode")
    return lat, wall.value


class SlotCb(ctypes.Structure):
    """orc_slot_cb (ldpc_oracle.h)."""
    _fields_ = [("bg", ctypes.c_int), ("Z", ctypes.c_uint), ("F", ctypes.c_uint), ("Qm", ctypes.c_uint),
                ("rv", ctypes.c_uint), ("iters", ctypes.c_uint), ("E", ctypes.c_uint), ("crc_poly", ctypes.c_int),
                ("llr", ctypes.c_void_p)]


def bench_slot(cbs, threads: int, reps: int, with_dematch: bool):
    """The CPU leg of the software-route slot (ldpc_cpu_slot.c): cbs = [(bg, Z, F, Qm, rv, iters, crc_poly, llr int8
    array)], decoded by `threads` C workers in pusch_decoder_impl's per-CB task order, `reps` timed slots after two
    warm-up ones. Returns (slot_us[reps], dec_us[reps, n], dm_us[reps, n], crc_ok of the last slot)."""
    n = len(cbs)
    keep = [np.ascontiguousarray(c[7], dtype=np.int8) for c in cbs]
    arr = (SlotCb * n)()
    for i, (c, l) in enumerate(zip(cbs, keep)):
        arr[i] = SlotCb(c[0], c[1], c[2], c[3], c[4], c[5], l.size, c[6], l.ctypes.data)
    slot = np.zeros(reps, np.float64)
    dec = np.zeros((reps, n), np.float64)
    dm = np.zeros((reps, n), np.float64)
    ok = ctypes.c_uint(0)
    r = lib().orc_bench_slot(ctypes.cast(arr, ctypes.c_void_p), n, threads, reps, 1 if with_dematch else 0,
                             _p(slot, ctypes.c_double), _p(dec, ctypes.c_double), _p(dm, ctypes.c_double),
                             ctypes.byref(ok))
    if r < 0:
        raise ValueError("oracle bench_slot: invalid argument or failed call")
    return slot, dec, dm, int(ok.value)


def ldpc_decode_port(bg: int, Z: int, llr: np.ndarray, max_iterations: int, crc_poly: int = NO_CRC,
                     nof_filler_bits: int = 0, out: np.ndarray | None = None):
    """The vectorisable CPU port (ldpc_cpu_port.c; scaling factor 0.8): same contract as ldpc_decode."""
    llr = np.ascontiguousarray(llr, dtype=np.int8)
    if out is None:
        out = np.zeros((BG_K[bg] * Z + 7) // 8, dtype=np.uint8)
    r = lib().orc_ldpc_decode_port(bg, Z, nof_filler_bits, _p(llr, ctypes.c_int8), llr.size, max_iterations,
                                   crc_poly, _p(out, ctypes.c_uint8))
    if r < 0:
        raise ValueError("oracle port decode: contract violation")
    return out, (r if r > 0 else None)


def tb_join(msgs: np.ndarray, cb_msg_bits: int, nof_filler_bits: int, cb_crc_bits: int, tbs: int,
            cb_crc_ok, tb_out: np.ndarray | None = None):
    """pusch_decoder_impl::join_and_notify / concatenate_codeblocks (pusch_decoder_impl.cpp:384-497).
    msgs: (C, msg_bytes) packed CB messages. Returns (tb_bytes, tb_crc_ok); tb_bytes is written as the reference
    writes the transport block (untouched when a CB CRC failed)."""
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    flags = np.ascontiguousarray(np.asarray(cb_crc_ok, dtype=np.uint8))
    out = np.zeros((tbs + 7) // 8, np.uint8) if tb_out is None else tb_out
    r = lib().orc_tb_join(_p(msgs, ctypes.c_uint8), msgs.shape[1], msgs.shape[0], cb_msg_bits, nof_filler_bits,
                          cb_crc_bits, tbs, _p(flags, ctypes.c_uint8), _p(out, ctypes.c_uint8))
    return out, bool(r)


# ---- segmenter (pure Python restatement of ldpc_segmenter_impl.cpp:58-69,254-331 / ldpc.h:124-217) -------------
def segment_rx(tbs: int, bg: int, nof_ch_symbols: int, Qm: int, nof_layers: int):
    tb_crc = 16 if tbs <= 3824 else 24
    B = tbs + tb_crc
    max_seg = 8448 if bg == 1 else 3840
    C = 1 if B <= max_seg else -(-B // (max_seg - 24))
    Bp = B + (24 * C if C > 1 else 0)
    kb = 22
    if bg == 2:
        kb = 10 if B > 640 else 9 if B > 560 else 8 if B > 192 else 6
    Z = next(z for z in LIFTING_SIZES if z * C * kb >= Bp)
    seg_len = BG_K[bg] * Z
    crc_len = 24 if C > 1 else 0
    max_info = -(-Bp // C) - crc_len
    sym_layer = nof_ch_symbols // nof_layers
    nof_short = C - (sym_layer % C)
    metas, off = [], 0
    for r in range(C):
        tmp = sym_layer // C if r < nof_short else -(-sym_layer // C)
        E = tmp * nof_layers * Qm
        metas.append(dict(bg=bg, Z=Z, C=C, full_length=seg_len * (3 if bg == 1 else 5),
                          nof_filler_bits=seg_len - (max_info + crc_len), nof_crc_bits=tb_crc if C == 1 else 24,
                          rm_length=E, cw_offset=off, tb_crc_bits=tb_crc))
        off += E
    return metas


def select_crc(tbs: int, nof_blocks: int) -> int:
    """select_crc (pusch_decoder_impl.cpp:35-46)."""
    if nof_blocks > 1:
        return CRC24B
    return CRC24A if tbs > 3824 else CRC16


__all__ = [n for n in dir() if not n.startswith("_")]


# ---- soft demodulation mapper (demodulation_mapper_*.cpp scalar paths) ------------------------
MOD_PI_2_BPSK, MOD_BPSK, MOD_QPSK, MOD_QAM16, MOD_QAM64, MOD_QAM256 = 0, 1, 2, 4, 6, 8


def bits_per_symbol(mod: int) -> int:
    return 1 if mod in (MOD_PI_2_BPSK, MOD_BPSK) else mod


def demodulate_soft(mod: int, symbols: np.ndarray, noise_vars: np.ndarray) -> np.ndarray:
    """demodulation_mapper::demodulate_soft: complex64 symbols + float32 noise variances -> int8 LLRs (Qm per symbol)."""
    sym = np.ascontiguousarray(symbols, dtype=np.complex64)
    nv = np.ascontiguousarray(noise_vars, dtype=np.float32)
    assert sym.size == nv.size
    out = np.zeros(sym.size * bits_per_symbol(mod), dtype=np.int8)
    fp = ctypes.POINTER(ctypes.c_float)
    r = lib().orc_demodulate_soft(mod, sym.size, sym.view(np.float32).ctypes.data_as(fp), nv.ctypes.data_as(fp),
                                  _p(out, ctypes.c_int8))
    if r != 0:
        raise ValueError("invalid modulation")
    return out
