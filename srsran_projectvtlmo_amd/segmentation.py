"""Host-side PUSCH transport-block bookkeeping around the device decode path.

* segment_rx: the RX segmenter's codeblock metadata (ldpc_segmenter_impl::segment, ldpc_segmenter_impl.cpp:254-331,
  compute_rm_length :58-69, generate_cb_metadata :308-331; ldpc.h:140-193 for C, Z and the BG2 Kb rule). In srsRAN
  this runs on the host before the decoder; it stays on the host here (negligible work).
* crc_bits: the CRC of crc_calculator_generic_impl.cpp:28-133 (MSB first, zero initial state, no reflection), with
  byte tables, for host-side TB/CB CRC attachment when synthesising transmissions.
* segment_tx: TS 38.212 5.1-5.2 on the transmit side (TB CRC, codeblock segmentation with CB CRC24B, filler bits),
  producing the packed K*Z-bit messages the device encoder takes.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import numpy as np

from .channel_coding import BG_K

# TS 38.212 Table 5.3.2-1, ascending
LIFTING_SIZES = (2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44, 48,
                 52, 56, 60, 64, 72, 80, 88, 96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320,
                 352, 384)

CRC_POLYS = {"CRC24A": (0x1864CFB, 24), "CRC24B": (0x1800063, 24), "CRC16": (0x11021, 16)}
_TABLES = {}


def _table(name: str) -> np.ndarray:
    if name not in _TABLES:
        poly, order = CRC_POLYS[name]
        t = np.zeros(256, dtype=np.uint32)
        top = 1 << (order - 1)
        mask = (1 << order) - 1
        for b in range(256):
            r = b << (order - 8)
            for _ in range(8):
                r = ((r << 1) ^ poly) & mask if r & top else (r << 1) & mask
            t[b] = r
        _TABLES[name] = t
    return _TABLES[name]


def crc_bits(name: str, bits: np.ndarray) -> int:
    """CRC of an unpacked bit sequence (one bit per element), MSB first, zero initial state."""
    poly, order = CRC_POLYS[name]
    mask = (1 << order) - 1
    bits = np.asarray(bits, dtype=np.uint8)
    n8 = bits.size // 8 * 8
    crc = 0
    tab = _table(name)
    for byte in np.packbits(bits[:n8]).tolist():
        crc = ((crc << 8) ^ int(tab[((crc >> (order - 8)) ^ byte) & 0xFF])) & mask
    for b in bits[n8:].tolist():
        fb = ((crc >> (order - 1)) & 1) ^ int(b)
        crc = ((crc << 1) & mask) ^ (poly & mask if fb else 0)
    return crc


@dataclass
class cb_metadata:
    """The fields of codeblock_metadata (include/srsran/phy/upper/codeblock_metadata.h:41-79) the path uses."""
    base_graph: int
    lifting_size: int
    nof_cbs: int
    full_length: int        # 3 K Z (BG1) / 5 K Z (BG2)
    nof_filler_bits: int
    nof_crc_bits: int       # 24 when C > 1, else the TB CRC length
    rm_length: int          # E_r
    cw_offset: int
    tb_crc_bits: int


def tb_crc_length(tbs: int) -> int:
    return 16 if tbs <= 3824 else 24


def segment_rx(tbs: int, bg: int, nof_ch_symbols: int, Qm: int, nof_layers: int) -> List[cb_metadata]:
    """ldpc_segmenter_impl::segment (RX): codeblock count, lifting size, filler bits and rate-matching lengths."""
    tb_crc = tb_crc_length(tbs)
    B = tbs + tb_crc
    max_seg = 8448 if bg == 1 else 3840
    C = 1 if B <= max_seg else -(-B // (max_seg - 24))
    Bp = B + (24 * C if C > 1 else 0)
    kb = 22 if bg == 1 else (10 if B > 640 else 9 if B > 560 else 8 if B > 192 else 6)
    Z = next(z for z in LIFTING_SIZES if z * C * kb >= Bp)
    KZ = BG_K[bg] * Z
    cb_crc = 24 if C > 1 else 0
    max_info = -(-Bp // C) - cb_crc
    per_layer = nof_ch_symbols // nof_layers
    nof_short = C - (per_layer % C)
    out, off = [], 0
    for r in range(C):
        sym = per_layer // C if r < nof_short else -(-per_layer // C)
        E = sym * nof_layers * Qm
        out.append(cb_metadata(bg, Z, C, KZ * (3 if bg == 1 else 5), KZ - (max_info + cb_crc),
                               tb_crc if C == 1 else 24, E, off, tb_crc))
        off += E
    return out


def segment_tx(tb_bits: np.ndarray, metas: List[cb_metadata]) -> np.ndarray:
    """TB bits -> (C, K*Z) unpacked CB messages: TB CRC attached (CRC24A / CRC16), split into C segments of
    K*Z - F - CRC data bits (zero padding at the end), CB CRC24B when C > 1, filler bits (as 0) at the end."""
    m0 = metas[0]
    C, Z, F = m0.nof_cbs, m0.lifting_size, m0.nof_filler_bits
    KZ = BG_K[m0.base_graph] * Z
    tb_crc = crc_bits("CRC24A" if m0.tb_crc_bits == 24 else "CRC16", tb_bits)
    b = np.concatenate([tb_bits.astype(np.uint8),
                        np.array([(tb_crc >> (m0.tb_crc_bits - 1 - i)) & 1 for i in range(m0.tb_crc_bits)],
                                 np.uint8)])
    cb_crc = 24 if C > 1 else 0
    kd = KZ - F - cb_crc
    msgs = np.zeros((C, KZ), np.uint8)
    for r in range(C):
        seg = b[r * kd:(r + 1) * kd]
        msgs[r, :seg.size] = seg
        if C > 1:
            c = crc_bits("CRC24B", msgs[r, :kd])
            msgs[r, kd:kd + 24] = [(c >> (23 - i)) & 1 for i in range(24)]
    return msgs
