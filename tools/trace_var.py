#!/usr/bin/env python3
"""Timeline of the compiled var kernel (offsets + lens batches: a pcap capture's layout) --
diagnostic, not the driver's bench. Per-wave s_memrealtime stamps (EBPFEMU_TRACE=1,
ebpf_debug_trace; interp.hip tile_body): entry, then for each of the wave's first five tiles the
moment its window is ready and the moment its statement is done, the end of the tile loop and the
counters' flush. Prints, in microseconds (100 MHz stamps) from the first wave's entry:
percentiles of the first window's arrival, of each tile's window wait (ready - previous done)
and compute (done - ready), of the wave's end, and the tiles per wave.

  python tools/trace_var.py [--program 5tuple] [--layout offsets|stride_lens] [--launches K]
The stamps' own waits slow the kernel a little: read shares and spreads, not the length.
The var kernels' stamps are compiled in only on request (they cost the kernel registers):
  make -C ebpf-emu_amd clean all EXTRA_HIPFLAGS=-DEBPFEMU_VAR_TRACE
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

    ap = argparse.ArgumentParser()
    ap.add_argument("--program", default="5tuple")
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--launches", type=int, default=6)
    args = ap.parse_args()

    dev = torch.device("cuda", 0)
    n = args.packets
    prog = Program(W.program(args.program))
    buf = W.frames_fixed(n, 64, 3)
    frames = torch.from_numpy(buf).to(dev)
    offs = torch.from_numpy((np.arange(n, dtype=np.int64) * 64).astype(np.uint32).view(np.int32)).to(dev)
    lens = torch.from_numpy(np.full(n, 64, dtype=np.int16)).to(dev)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    out = _lib.BatchOut()
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    out.verdict = verdict.data_ptr()
    out.counters = cnt.data_ptr()
    desc = prog.make_batch(frames, n=n, offsets=offs, lens=lens)
    kid = prog.batch_kernel(desc, out, 0)
    stream = torch.cuda.current_stream(dev)
    for _ in range(args.launches):
        prog.launch(desc, out, stream)
    torch.cuda.synchronize()
    ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
    assert _lib.lib().ebpf_debug_trace(0, ctypes.byref(ptr), ctypes.byref(nb)) == 0 and nb.value
    host = np.zeros(nb.value // 8, dtype=np.uint64)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(host.ctypes.data_as(ctypes.c_void_p), ptr, nb, 2) == 0
    ring = host.reshape(4, -1, 16)
    tr = ring[(args.launches - 1) % 4].astype(np.int64)
    tr = tr[(tr[:, 0] != 0) & (tr[:, 13] != 0)]
    t0 = int(tr[:, 0].min())
    us = lambda v: (v - t0) / 100.0  # noqa: E731 (s_memrealtime: 100 MHz)

    def pct(x):
        x = np.asarray(x, dtype=np.float64)
        return {p: round(float(np.percentile(x, p)), 3) for p in (5, 50, 95, 100)} if len(x) else {}

    tiles = tr[:, 15]
    res = {"kernel": _lib.KERNEL_NAMES[kid], "waves": int(len(tr)),
           "tiles_per_wave": pct(tiles), "entry": pct(us(tr[:, 0])),
           "first_window_ready": pct(us(tr[:, 1])), "end": pct(us(tr[:, 12])),
           "flushed": pct(us(tr[:, 13]))}
    for i in range(5):
        m = tiles > i
        if not m.any():
            break
        prev = tr[m, 0] if i == 0 else tr[m, 2 * i]
        res[f"tile{i}"] = {"wait": pct((tr[m, 1 + 2 * i] - prev) / 100.0),
                           "compute": pct((tr[m, 2 + 2 * i] - tr[m, 1 + 2 * i]) / 100.0)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
