#!/usr/bin/env python3
"""Timeline of the compiled loop kernel over config 5's batch (diagnostic, not the driver's
bench): per-wave s_memrealtime stamps of each wave's tile (EBPFEMU_TRACE=1, ebpf_debug_trace;
interp.hip tile_body) -- entry, window ready, statement done, counters flushed -- split by the
tile's packet length (long / short), as percentiles across waves in microseconds from the first
wave's entry, plus a histogram of the long tiles' entries (how many rounds of waves there were).

  python tools/trace_loop.py [--config checksum|checksum_stack] [--launches K]
The stamps' own waits slow the kernel a little: read shares and spreads, not the length.
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
    ap.add_argument("--config", default="checksum", choices=["checksum", "checksum_stack"])
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--launches", type=int, default=6)
    args = ap.parse_args()

    dev = torch.device("cuda", 0)
    prog = Program(W.program(args.config))
    buf, offs, lens = W.frames_mixed(args.packets)
    frames = torch.from_numpy(buf).to(dev)
    offsets = torch.from_numpy(offs).to(dev)
    lengths = torch.from_numpy(lens).to(dev)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    out = _lib.BatchOut()
    verdict = torch.empty(args.packets, dtype=torch.uint8, device=dev)
    out.verdict = verdict.data_ptr()
    out.counters = cnt.data_ptr()
    desc = prog.make_batch(frames, n=args.packets, offsets=offsets, lens=lengths, mem_size=2048,
                           r10=2048)
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
    tr = ring[(args.launches - 1) % 4]
    tr = tr[(tr[:, 0] != 0) & (tr[:, 13] != 0)]
    t0 = int(tr[:, 0].min())
    us = lambda v: (v.astype(np.int64) - t0) / 100.0  # 100 MHz
    pct = lambda v: {p: round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 100)} if len(v) else {}
    res = {"waves": int(len(tr)), "kernel_span_us": round(float(us(tr[:, 13]).max()), 2)}
    for name, sel in (("long", tr[:, 4] >= 512), ("short", tr[:, 4] < 512)):
        t = tr[sel]
        res[name] = {
            "waves": int(len(t)),
            "entry": pct(us(t[:, 0])),
            "prologue": pct((t[:, 1].astype(np.int64) - t[:, 0].astype(np.int64)) / 100.0),
            "statement": pct((t[:, 2].astype(np.int64) - t[:, 1].astype(np.int64)) / 100.0),
            "flush": pct((t[:, 13].astype(np.int64) - t[:, 12].astype(np.int64)) / 100.0),
            "end": pct(us(t[:, 13])),
        }
    lg = tr[tr[:, 4] >= 512]
    hist, edges = np.histogram(us(lg[:, 0]), bins=12)
    res["long_entry_histogram"] = {f"{edges[i]:.0f}-{edges[i + 1]:.0f}us": int(h) for i, h in enumerate(hist)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
