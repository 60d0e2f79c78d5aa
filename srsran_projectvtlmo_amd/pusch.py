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


def tb_join_launch(ctx: _lib.Context, specs: Sequence[tb_join_spec], d_msgs: int, d_cb_results: int, d_tb: int,
                   d_tb_results: int, stream: int = 0) -> None:
    """ldpc_hip_tb_join_launch: asynchronous on `stream` (0 = the context stream); all buffers are device pointers.
    d_tb_results receives one TbResult (4 bytes) per spec."""
    arr = (TbDesc * max(1, len(specs)))()
    for i, s in enumerate(specs):
        d = arr[i]
        d.msg_offset, d.tb_offset, d.msg_stride = s.msg_offset, s.tb_offset, s.msg_stride
        d.tbs, d.result_index, d.nof_cbs = s.tbs, s.result_index, s.nof_cbs
        d.cb_msg_bits, d.nof_filler_bits, d.cb_crc_bits = s.cb_msg_bits, s.nof_filler_bits, s.cb_crc_bits
    rc = ctx.lib.ldpc_hip_tb_join_launch(ctx.handle, len(specs), arr, d_msgs, d_cb_results, d_tb, d_tb_results,
                                         stream or None)
    _lib.check(ctx.handle, rc, "ldpc_hip_tb_join_launch")
