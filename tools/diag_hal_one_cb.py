#!/usr/bin/env python3
"""Diagnostic (not product): where a HAL one-codeblock TB's time goes (C4's 23 small TBs: BG2 Z=36, E = 1,248 QPSK
LLRs, CRC16, early stop) on the device work queue, through the Python HAL mirror in pusch_decoder_hw_impl's call
order (reserve -> configure -> enqueue -> dequeue spin -> read outputs -> free). Needs the diagnostic build
(make -C srsran_projectvtlmo_amd/csrc VARIANT=diagdwq FLAGS="-DLDPC_HIP_DIAG_DWQ -DLDPC_HIP_DIAG_CB"): per item the
host's submit / done-seen times and the device's claim / item / body stamps, plus the workgroup's stamps: 6 body
entry, 0 decoder prologue start (after the fused dematcher), 7 soft bits loaded, 1 prologue done, 2 lanes, 3
iterations, 4 hard decision + CRC, 5 stored.

With DIAG_DM=1 and DIAG_LIB=diagdm (the same build plus -DLDPC_HIP_DIAG_CB_DM) stamps 1-3 split the fused
dematcher instead: LLRs staged in LDS, de-interleave ranges written, its stores drained.

usage: python tools/diag_hal_one_cb.py [TBs]"""
import ctypes
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{os.environ.get('DIAG_LIB', 'diagdwq')}.so"
L = _lib.load()
from srsran_projectvtlmo_amd import hal  # noqa: E402
from tests.tb_chain import TransportBlock  # noqa: E402  (test vectors only)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
L.ldpc_hip_diag_dwq_read.restype = ctypes.c_uint32
L.ldpc_hip_diag_dwq_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
L.ldpc_hip_diag_cb_read.restype = ctypes.c_int
L.ldpc_hip_diag_cb_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]

repo = hal.create_ext_harq_buffer_context_repository(1024, 1024 * hal.HARQ_INCR, False)
cfg = hal.hw_accelerator_pusch_dec_configuration(acc_type="mi355x", ext_softbuffer=True, harq_buffer_context=repo)
acc = hal.create_hw_accelerator_pusch_dec_factory(cfg).create()
rng = np.random.default_rng(3)
tbs = [TransportBlock(rng, 256, 2, 156 * 4, "QPSK", 4) for _ in range(8)]
llrs = [tb.llrs(rng, 0, 2.5, 1.0)[0] for tb in tbs]
rec_buf = (ctypes.c_uint64 * (8 * 4096))()
cb_buf = (ctypes.c_uint64 * 8192)()
L.ldpc_hip_diag_dwq_read(rec_buf, 4096)
host_us, stamps = [], []
for k in range(n):
    tb, llr = tbs[k % len(tbs)], llrs[k % len(tbs)]
    op = hal.hw_pusch_decoder_configuration(base_graph_index=2, modulation="QPSK", nof_segments=1, rv=0,
                                            cw_length=llr.size, lifting_size=tb.Z, Ncb=tb.N,
                                            nof_filler_bits=tb.F, max_nof_ldpc_iterations=8, use_early_stop=True,
                                            new_data=True, cb_crc_len=16, cb_crc_type=hal.CRC16,
                                            absolute_cb_id=k % 64)
    msg = np.zeros((10 * tb.Z + 7) // 8, np.uint8)
    t0 = time.perf_counter()
    acc.reserve_queue()
    acc.configure_operation(op, 0)
    acc.enqueue_operation(llr, None, 0)
    while not acc.dequeue_operation(msg, None, 0):
        pass
    t1 = time.perf_counter()
    out = hal.hw_pusch_decoder_outputs()
    acc.read_operation_outputs(out, 0, k % 64)
    acc.free_queue()
    host_us.append((t1 - t0) * 1e6)
    if k % 10 == 9:
        assert L.ldpc_hip_diag_cb_read(acc.ctx.handle, cb_buf, 8192) == 0
        stamps.append(np.array(cb_buf, dtype=np.int64).reshape(1024, 8))
m = L.ldpc_hip_diag_dwq_read(rec_buf, 4096)
r = np.array(rec_buf[:8 * m], dtype=np.int64).reshape(m, 8)
print(f"HAL one-CB TB (BG2 Z=36, E=1248): {n} TBs, host reserve..dequeue p50 {np.median(host_us):.2f} us; {m} items")
if m:
    sub_seen = (r[:, 1] - r[:, 0]) / 1e3
    item = r[:, 3] * 0.01
    dev = r[:, 4] * 0.01
    for lab, v in (("submitted -> done seen", sub_seen), ("device: claim -> item in LDS", item),
                   ("device: claim -> body done", dev), ("outside the device (pickup + done)", sub_seen - dev)):
        print(f"  {lab:38s} {np.median(v):7.2f} {np.percentile(v, 10):7.2f} {np.percentile(v, 90):7.2f}")
    ph = []
    for k, st in zip(range(9, n, 10), stamps):
        if k >= m:
            continue
        wg = int(r[k, 5])
        s = st[wg]
        if not (s[6] and s[7]):
            continue
        # entry -> prologue start (the fused dematcher), prologue start -> soft bits stored, -> prologue done,
        # lanes, iterations, hd + crc, stored
        if os.environ.get("DIAG_DM"):  # LDPC_HIP_DIAG_CB_DM build: slots 1-3 are the dematcher's
            ph.append([(s[1] - s[6]) * 0.01, (s[2] - s[1]) * 0.01, (s[3] - s[2]) * 0.01, (s[0] - s[3]) * 0.01,
                       (s[7] - s[0]) * 0.01, (s[4] - s[7]) * 0.01, (s[5] - s[4]) * 0.01])
        else:
            ph.append([(s[0] - s[6]) * 0.01, (s[7] - s[0]) * 0.01, (s[1] - s[7]) * 0.01] +
                      list(np.diff(s[1:6]) * 0.01))
    if ph:
        ph = np.array(ph)
        names = (["dm: LLRs staged", "dm: ranges", "dm: stores drained", "dm end -> prologue", "prologue: soft bits "
                  "loaded", "soft loaded -> hd+crc done", "stored"] if os.environ.get("DIAG_DM") else
                 ["fused dematch", "prologue: soft bits loaded", "prologue: rest", "lanes", "iterations", "hd+crc",
                  "stored"])
        print("  body phases (us, p50): " + ", ".join(f"{a} {np.median(ph[:, i]):.2f}" for i, a in enumerate(names)))
