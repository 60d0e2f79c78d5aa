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
