"""Python mirror of srsRAN's hardware-accelerated PUSCH decoder plugin surface, backed by the MI355X library.

Mirrors include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h:36-115 and
include/srsran/hal/hw_accelerator.h:35-57 (same method names, argument meaning, return values):

  reserve_queue / free_queue / configure_operation / enqueue_operation / dequeue_operation /
  read_operation_outputs / free_harq_context_entry / is_external_harq_supported

and the factory selection of hw_accelerator_factories.cpp:63-66 with the new acc_type "mi355x". The caller flow it
serves is pusch_decoder_hw_impl::on_end_softbits (pusch_decoder_hw_impl.cpp:132-342): configure + enqueue every
codeblock (external HARQ) or one codeblock at a time (host HARQ), then dequeue (spinning on False) and read the
outputs. The first dequeue of a staged batch launches rate dematching + decoding of all its codeblocks on the device
(ldpc_hip_dequeue); once all are dequeued the next enqueue starts a new batch.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import CbResult, DROPPED, EFULL, HwConfig, LdpcHipError, NOT_READY, OK

CRC16, CRC24B, CRC24A = 0, 1, 2  # hal::hw_dec_cb_crc_type
_MOD_BITS = {"BPSK": 1, "PI_2_BPSK": 1, "QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}


@dataclass
class hw_pusch_decoder_configuration:
    base_graph_index: int = 1
    modulation: str = "QPSK"
    nof_segments: int = 1
    rv: int = 0
    cw_length: int = 0
    lifting_size: int = 2
    Ncb: int = 0
    Nref: int = 0
    nof_segment_bits: int = 0
    nof_filler_bits: int = 0
    max_nof_ldpc_iterations: int = 6
    use_early_stop: bool = True
    new_data: bool = True
    cb_crc_len: int = 24
    cb_crc_type: int = CRC24B
    absolute_cb_id: int = 0


@dataclass
class hw_pusch_decoder_outputs:
    CRC_pass: bool = False
    nof_ldpc_iterations: int = 0


class hw_accelerator_pusch_dec:
    """Abstract interface (hw_accelerator_pusch_dec.h:83-115)."""


class hw_accelerator_pusch_dec_hip(hw_accelerator_pusch_dec):
    def __init__(self, ctx: _lib.Context):
        self.ctx = ctx
        self.cfg = {}

    def _check(self, rc, what):
        return _lib.check(self.ctx.handle, rc, what)

    def reserve_queue(self) -> None:
        self._check(self.ctx.lib.ldpc_hip_queue_reserve(self.ctx.handle), "reserve_queue")

    def free_queue(self) -> None:
        self._check(self.ctx.lib.ldpc_hip_queue_free(self.ctx.handle), "free_queue")
        self.cfg.clear()

    def configure_operation(self, config: hw_pusch_decoder_configuration, cb_index: int = 0) -> None:
        c = HwConfig()
        c.base_graph = int(config.base_graph_index)
        c.modulation_order = _MOD_BITS[config.modulation] if isinstance(config.modulation, str) else int(
            config.modulation)
        c.rv = config.rv
        c.new_data = 1 if config.new_data else 0
        c.nof_segments = config.nof_segments
        c.cw_length = config.cw_length
        c.lifting_size = config.lifting_size
        c.Ncb = config.Ncb
        c.Nref = config.Nref
        c.nof_segment_bits = config.nof_segment_bits
        c.nof_filler_bits = config.nof_filler_bits
        c.max_nof_ldpc_iterations = config.max_nof_ldpc_iterations
        c.use_early_stop = 1 if config.use_early_stop else 0
        c.cb_crc_type = int(config.cb_crc_type)
        c.cb_crc_len = config.cb_crc_len
        c.absolute_cb_id = config.absolute_cb_id
        self.cfg[cb_index] = c

    def enqueue_operation(self, data: np.ndarray, aux_data: Optional[np.ndarray] = None, cb_index: int = 0) -> bool:
        """True when the operation was accepted -- also when it is accepted as dropped (no free HARQ arena entry, or
        a retransmission whose soft data the arena no longer holds), which later reads as a CRC failure with the
        maximum number of iterations, as acc100 does (hw_accelerator_pusch_dec_acc100_impl.cpp:120-130, 179-186,
        233-247). False when the batch cannot take it now (full, or still in flight): the caller dequeues and
        enqueues it again (pusch_decoder_hw_impl.cpp:237-241)."""
        if cb_index not in self.cfg:
            raise LdpcHipError("enqueue_operation without configure_operation")
        llr = np.ascontiguousarray(data, dtype=np.int8)
        soft = None if aux_data is None or len(aux_data) == 0 else np.ascontiguousarray(aux_data, dtype=np.int8)
        rc = self.ctx.lib.ldpc_hip_enqueue(self.ctx.handle, cb_index, ctypes.byref(self.cfg[cb_index]),
                                           llr.ctypes.data if llr.size else None, llr.size,
                                           soft.ctypes.data if soft is not None else None,
                                           0 if soft is None else soft.size)
        if rc == EFULL:
            return False
        if rc in (OK, DROPPED):
            return True
        self._check(rc, "enqueue_operation")
        return True

    def dequeue_operation(self, data: np.ndarray, aux_data: Optional[np.ndarray] = None,
                          segment_index: int = 0) -> bool:
        """data: packed message buffer (uint8, modified); aux_data: soft buffer updated in place when the HARQ
        buffer is host-side. Returns False while the batch has not completed (the caller spins)."""
        if not (isinstance(data, np.ndarray) and data.dtype == np.uint8 and data.flags.c_contiguous):
            raise LdpcHipError("data must be a contiguous uint8 array")
        soft = aux_data if (aux_data is not None and len(aux_data) != 0) else None
        rc = self.ctx.lib.ldpc_hip_dequeue(self.ctx.handle, segment_index, data.ctypes.data, data.size,
                                           soft.ctypes.data if soft is not None else None,
                                           0 if soft is None else soft.size)
        if rc == NOT_READY:
            return False
        self._check(rc, "dequeue_operation")
        return True

    def read_operation_outputs(self, out: hw_pusch_decoder_outputs, cb_index: int = 0,
                               absolute_cb_id: int = 0) -> None:
        r = CbResult()
        self._check(self.ctx.lib.ldpc_hip_read_outputs(self.ctx.handle, cb_index, absolute_cb_id, ctypes.byref(r)),
                    "read_operation_outputs")
        out.CRC_pass = bool(r.crc_pass)
        out.nof_ldpc_iterations = int(r.nof_iterations)

    def free_harq_context_entry(self, absolute_cb_id: int) -> None:
        self._check(self.ctx.lib.ldpc_hip_harq_free(self.ctx.handle, absolute_cb_id), "free_harq_context_entry")

    def is_external_harq_supported(self) -> bool:
        return bool(self.ctx.lib.ldpc_hip_external_harq_supported(self.ctx.handle))


@dataclass
class hw_accelerator_pusch_dec_configuration:
    """hw_accelerator_pusch_dec_factory configuration (acc_type selects the implementation)."""
    acc_type: str = "mi355x"
    device: int = 0
    ext_softbuffer: bool = True
    nof_harq_slots: int = 1024
    max_queue_cbs: int = 162


class hw_accelerator_pusch_dec_factory:
    def __init__(self, cfg: hw_accelerator_pusch_dec_configuration):
        self.cfg = cfg

    def create(self) -> hw_accelerator_pusch_dec_hip:
        ctx = _lib.Context(self.cfg.device, max_queue_cbs=self.cfg.max_queue_cbs,
                           nof_harq_slots=self.cfg.nof_harq_slots if self.cfg.ext_softbuffer else 0)
        return hw_accelerator_pusch_dec_hip(ctx)


def create_hw_accelerator_pusch_dec_factory(cfg: hw_accelerator_pusch_dec_configuration):
    """hw_accelerator_factories.cpp:63-66: returns None for an unsupported acc_type."""
    if cfg.acc_type != "mi355x":
        return None
    return hw_accelerator_pusch_dec_factory(cfg)
