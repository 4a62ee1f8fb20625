#!/usr/bin/env python3
"""Timeline of the compiled fixed-slot kernel (diagnostic, not the driver's bench): per-wave
s_memrealtime stamps (EBPFEMU_TRACE=1, ebpf_debug_trace) of one launch over a BASELINE-shaped
batch, summarised as percentiles across waves (microseconds from the first wave's entry):
entry, each tile done, flush start / end; and per XCD, the last wave's end.

  python tools/trace_tiles.py [--config 5tuple|drop] [--packets N] [--launches K]
The stamps' own waits slow the kernel: read shares and spreads, not the length.
"""
import argparse
import ctypes
import json
import os
import sys

os.environ["EBPFEMU_TRACE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))


def main():
    import numpy as np
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="5tuple", choices=["5tuple", "drop"])
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--launches", type=int, default=20)
    args = ap.parse_args()

    dev = torch.device("cuda", 0)
    prog = Program(assemble(W.PROGRAMS[args.config]))
    frames = torch.from_numpy(W.frames_fixed(args.packets, 64)).to(dev)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    for _ in range(args.launches):
        prog.run(frames, n=args.packets, stride=64, counters=cnt)
    torch.cuda.synchronize()
    ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
    assert _lib.lib().ebpf_debug_trace(0, ctypes.byref(ptr), ctypes.byref(nb)) == 0 and nb.value
    host = np.zeros(nb.value // 8, dtype=np.uint64)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(host.ctypes.data_as(ctypes.c_void_p), ptr, nb, 2) == 0
    tr = host.reshape(-1, 16)
    tr = tr[tr[:, 0] != 0]
    t0 = tr[:, 0].min()
    us = lambda v: (v.astype(np.int64) - int(t0)) / 100.0  # 100 MHz
    pct = lambda v: {p: round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 100)}
    ntiles = tr[:, 15].astype(int)
    out = {"waves": int(len(tr)), "tiles_per_wave": sorted(set(ntiles.tolist())),
           "entry": pct(us(tr[:, 0]))}
    for k in range(1, int(ntiles.max()) + 1):
        sel = ntiles >= k
        out[f"tile{k}_done"] = pct(us(tr[sel, k]))
    out["flush_start"] = pct(us(tr[:, 12]))
    out["flush_end"] = pct(us(tr[:, 13]))
    out["flush_len"] = pct((tr[:, 13].astype(np.int64) - tr[:, 12].astype(np.int64)) / 100.0)
    xcc = (tr[:, 14] >> 32).astype(int)
    out["end_by_xcd"] = {int(x): round(float(us(tr[xcc == x, 13]).max()), 2) for x in sorted(set(xcc))}
    out["mean_end_by_xcd"] = {int(x): round(float(us(tr[xcc == x, 13]).mean()), 2)
                              for x in sorted(set(xcc))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
