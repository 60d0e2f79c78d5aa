#!/usr/bin/env python3
"""GPU box: event-timed launches of the encoder (ldpc_hip_encode_launch) on device-resident messages, per graph and
batch size (the full shortened codeword, 50 back-to-back launches after 5 warm-up ones), to separate the kernel's own
time from the PDSCH plugin's PCIe and host costs. Prints one line per (BG, Z, CBs)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from srsran_projectvtlmo_amd import _lib  # noqa: E402
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402

if __name__ == "__main__":
    ctx = _lib.Context(0)
    s = torch.cuda.Stream()
    for bg, Z in ((1, 384), (2, 36), (2, 208), (1, 64)):
        K, Ns = (22, 66) if bg == 1 else (10, 50)
        for n in (1, 128):
            mb = ((K * Z + 7) // 8 + 15) // 16 * 16
            cb = ((Ns * Z + 7) // 8 + 15) // 16 * 16
            specs = [cc.cb_encode_spec(bg, Z, Ns * Z, i * mb, i * cb) for i in range(n)]
            msg = torch.randint(0, 256, (n * mb,), dtype=torch.uint8, device="cuda")
            cw = torch.zeros(n * cb, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                for _ in range(5):
                    cc.encode_launch(ctx, specs, msg.data_ptr(), cw.data_ptr(), s.cuda_stream)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(50):
                    cc.encode_launch(ctx, specs, msg.data_ptr(), cw.data_ptr(), s.cuda_stream)
                e1.record(s)
            e1.synchronize()
            print(f"BG{bg} Z={Z:3d} CBs={n:3d}: {e0.elapsed_time(e1) * 1000 / 50:7.1f} us per launch", flush=True)
    ctx.close()
