"""GPU box: the C4 slot blob (bench.hal_slot_blob) through tests/cpp/build/bench_sw with the one-CB zero-copy path
over the device work queue (default), the zero-copy path with a kernel launch per call (LDPC_HIP_DWQ=0) and the copy
path (LDPC_HIP_SYNC_ZERO_COPY=0), and through bench_hal with and without the work queue; prints one JSON object.
usage: python tools/sw_route_ab.py [reps] [threads]"""
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import bench
    from srsran_projectvtlmo_amd import _lib
    reps = sys.argv[1] if len(sys.argv) > 1 else "10"
    threads = sys.argv[2] if len(sys.argv) > 2 else "1,4,8,16"
    ctx = _lib.Context(0)
    blob = bench.hal_slot_blob(ctx)
    ctx.close()
    torch.cuda.synchronize()
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(blob)
        path = f.name
    out = {}
    try:
        for name, env in (("zero_copy", {}), ("zero_copy_no_dwq", {"LDPC_HIP_DWQ": "0"}),
                          ("copy", {"LDPC_HIP_SYNC_ZERO_COPY": "0"})):
            r = subprocess.run([str(ROOT / "tests/cpp/build/bench_sw"), path, reps, "0", threads], capture_output=True,
                               text=True, timeout=240, env={**os.environ, **env})
            out["sw_" + name] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-400:]
            print(name, "done", file=sys.stderr, flush=True)
        for name, env in (("hal", {}), ("hal_no_dwq", {"LDPC_HIP_DWQ": "0"})):
            r = subprocess.run([str(ROOT / "tests/cpp/build/bench_hal"), path, reps, "0"], capture_output=True,
                               text=True, timeout=240, env={**os.environ, **env})
            out[name] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-400:]
            print(name, "done", file=sys.stderr, flush=True)
    finally:
        os.unlink(path)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
