"""Seeded test-vector generators shared by the parity tests (they use the CPU oracle as the checker)."""
from __future__ import annotations

import numpy as np

import oracle as O


def random_llrs(rng, n, kind="mixed"):
    """int8 LLRs in [-127, 127]. kinds: 'pm10' (reference benchmark: (rgen() & 1)*20 - 10), 'uniform',
    'mixed' (uniform with extra zeros and +-127 infinities)."""
    if kind == "pm10":
        return (rng.integers(0, 2, n) * 20 - 10).astype(np.int8)
    # valid LLRs only: [-120, 120] and +-127 (log_likelihood_ratio.h constructor asserts anything else)
    v = rng.integers(-120, 121, n).astype(np.int8)
    if kind == "mixed":
        sel = rng.random(n)
        v[sel < 0.05] = 0
        v[(sel >= 0.05) & (sel < 0.07)] = 127
        v[(sel >= 0.07) & (sel < 0.09)] = -127
    return v


def codeword_llrs(rng, bg, Z, snr_amp=2.0, noise=1.0, F=0, crc=None, cb_len=None):
    """Random message (+ optional CB CRC) -> oracle encoder -> BPSK +-amp + N(0, noise) -> quantize(x, 8.0).
    Filler positions get +127 (as the rate dematcher sets them). Returns (llr, msg_bits)."""
    K = O.BG_K[bg]
    KZ = K * Z
    msg = rng.integers(0, 2, KZ).astype(np.uint8)
    if F:
        msg[KZ - F:] = O.FILLER_BIT
    if crc is not None:
        crc_len = 16 if crc == O.CRC16 else 24
        L = KZ - F
        data = msg[:L - crc_len].copy()
        c = O.crc_bits(crc, data)
        msg[L - crc_len:L] = [(c >> (crc_len - 1 - i)) & 1 for i in range(crc_len)]
    cw = O.ldpc_encode(bg, Z, msg, cb_len)
    x = np.where(cw == 1, -snr_amp, snr_amp).astype(np.float32) + noise * rng.standard_normal(cw.size).astype(
        np.float32)
    llr = O.quantize_array(x, 8.0)
    llr[cw == O.FILLER_BIT] = 127
    return llr, msg


def msg_bits_match(packed, msg, KZ):
    bits = np.unpackbits(packed)[:KZ]
    return bool(np.all((bits == msg) | ((msg == O.FILLER_BIT) & (bits == 0))))


def modulate(bits: np.ndarray, mod: int) -> np.ndarray:
    """TS 38.211 §5.1 modulation mapper (the reference's modulation_mapper_lut_impl.cpp), test-vector generation
    only: unpacked bits -> complex64 symbols. mod: modulation_scheme value."""
    b = np.asarray(bits, dtype=np.float64).reshape(-1, 1 if mod in (0, 1) else mod)
    s = 1.0 - 2.0 * b  # (1 - 2 b)
    if mod == 1:  # BPSK §5.1.2
        z = (s[:, 0] + 1j * s[:, 0]) / np.sqrt(2)
    elif mod == 0:  # pi/2-BPSK §5.1.1: e^{j pi/2 (i mod 2)} / sqrt(2) (1 - 2b)(1 + j)
        z = (s[:, 0] + 1j * s[:, 0]) / np.sqrt(2)
        z[1::2] *= 1j
    elif mod == 2:  # QPSK §5.1.3
        z = (s[:, 0] + 1j * s[:, 1]) / np.sqrt(2)
    elif mod == 4:  # 16QAM §5.1.4
        z = (s[:, 0] * (2 - s[:, 2]) + 1j * s[:, 1] * (2 - s[:, 3])) / np.sqrt(10)
    elif mod == 6:  # 64QAM §5.1.5
        z = (s[:, 0] * (4 - s[:, 2] * (2 - s[:, 4])) + 1j * s[:, 1] * (4 - s[:, 3] * (2 - s[:, 5]))) / np.sqrt(42)
    elif mod == 8:  # 256QAM §5.1.6
        z = (s[:, 0] * (8 - s[:, 2] * (4 - s[:, 4] * (2 - s[:, 6])))
             + 1j * s[:, 1] * (8 - s[:, 3] * (4 - s[:, 5] * (2 - s[:, 7])))) / np.sqrt(170)
    else:
        raise ValueError(mod)
    return z.astype(np.complex64)


def noisy_symbols(rng, n: int, mod: int, noise_var: float = 0.05):
    """Random bits, modulated, plus complex AWGN of variance noise_var; returns (bits, symbols, noise_vars)."""
    qm = 1 if mod in (0, 1) else mod
    bits = rng.integers(0, 2, n * qm).astype(np.uint8)
    z = modulate(bits, mod)
    w = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * np.sqrt(noise_var / 2)
    nv = (noise_var * rng.uniform(0.5, 2.0, n)).astype(np.float32)
    return bits, (z + w).astype(np.complex64), nv
