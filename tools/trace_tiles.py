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
    ap.add_argument("--no-counters", action="store_true")
    args = ap.parse_args()

    dev = torch.device("cuda", 0)
    prog = Program(assemble(W.PROGRAMS[args.config]))
    # a pool of distinct batches larger than the 256 MiB Infinity Cache, as bench.py: every launch
    # streams from HBM
    pool = []
    while sum(f.numel() for f in pool) < (512 << 20) and len(pool) < 16:
        pool.append(torch.from_numpy(W.frames_fixed(args.packets, 64, 100 + len(pool))).to(dev))
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    out = _lib.BatchOut()
    verdict = torch.empty(args.packets, dtype=torch.uint8, device=dev)
    out.verdict = verdict.data_ptr()
    out.counters = None if args.no_counters else cnt.data_ptr()
    descs = [prog.make_batch(f, n=args.packets, stride=64) for f in pool]
    stream = torch.cuda.current_stream(dev)
    for i in range(args.launches):
        prog.launch(descs[i % len(descs)], out, stream)
    torch.cuda.synchronize()
    ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
    assert _lib.lib().ebpf_debug_trace(0, ctypes.byref(ptr), ctypes.byref(nb)) == 0 and nb.value
    host = np.zeros(nb.value // 8, dtype=np.uint64)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(host.ctypes.data_as(ctypes.c_void_p), ptr, nb, 2) == 0
    ring = host.reshape(4, -1, 16)
    spans = []
    for k in range(4):
        r = ring[k][ring[k][:, 0] != 0]
        if len(r):
            spans.append((int(r[:, 0].min()), int(r[:, 13].max())))
    spans.sort()
    gaps = [round((spans[i + 1][0] - spans[i][1]) / 100.0, 2) for i in range(len(spans) - 1)]
    last = (args.launches - 1) % 4
    tr = ring[last][ring[last][:, 0] != 0]
    t0 = tr[:, 0].min()
    us = lambda v: (v.astype(np.int64) - int(t0)) / 100.0  # 100 MHz
    pct = lambda v: {p: round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 100)}
    ntiles = tr[:, 15].astype(int)
    out = {"waves": int(len(tr)), "tiles_per_wave": sorted(set(ntiles.tolist())),
           "entry": pct(us(tr[:, 0]))}
    for k in range(1, min(10, int(ntiles.max())) + 1):
        sel = (ntiles >= k) & (tr[:, k] != 0)  # (the tile-loop kernel stamps no tiles)
        if sel.any():
            out[f"tile{k}_done"] = pct(us(tr[sel, k]))
    out["flush_start"] = pct(us(tr[:, 12]))
    out["flush_end"] = pct(us(tr[:, 13]))
    out["flush_len"] = pct((tr[:, 13].astype(np.int64) - tr[:, 12].astype(np.int64)) / 100.0)
    xcc = (tr[:, 14] >> 32).astype(int)
    out["end_by_xcd"] = {int(x): round(float(us(tr[xcc == x, 13]).max()), 2) for x in sorted(set(xcc))}
    out["mean_end_by_xcd"] = {int(x): round(float(us(tr[xcc == x, 13]).mean()), 2)
                              for x in sorted(set(xcc))}
    # where the spread of the waves' end times lives: across CUs, or among the waves of a CU /
    # SIMD (HW_ID: wave [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]; XCC separately)
    hw = (tr[:, 14] & 0xFFFFFFFF).astype(np.int64)
    cu = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 50 + ((hw >> 8) & 15)
    simd = cu * 10 + ((hw >> 4) & 3)
    end = us(tr[:, 13])
    import collections
    def spread(keys):
        g = collections.defaultdict(list)
        for k, e in zip(keys, end):
            g[k].append(e)
        within = float(np.mean([max(v) - min(v) for v in g.values() if len(v) > 1]))
        means = [np.mean(v) for v in g.values()]
        return round(within, 2), round(float(np.max(means) - np.min(means)), 2), len(g)
    out["end_spread_within_cu_us, across_cu_means_us, cus"] = spread(cu)
    out["end_spread_within_simd_us, across_simd_means_us, simds"] = spread(simd)
    # the waves of a SIMD by launch order (wave slot in the hardware): mean end per rank
    order = collections.defaultdict(list)
    for k, slot, e in zip(simd, (hw & 15), end):
        order[k].append((slot, e))
    ranks = collections.defaultdict(list)
    for k, v in order.items():
        for r, (_, e) in enumerate(sorted(v)):
            ranks[r].append(e)
    out["mean_end_by_wave_rank_in_simd"] = {r: round(float(np.mean(v)), 2) for r, v in sorted(ranks.items())}
    out["wave_span_us"] = [round((b - a) / 100.0, 2) for a, b in spans]
    out["gap_to_next_launch_us"] = gaps
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
