#!/usr/bin/env python3
"""Consecutive batches on S streams (diagnostic): the 5-tuple (or --config) over 1 Mi x 64 B
frames, K launches alternating over S streams (each with its own library workspace, verdicts and
counters), timed with one event pair around all of them (stream 0 waits on the others before
the end event). Prints us per batch for S = 1, 2, 3, 4, twice each, and checks that the counters
summed over the streams equal K / 8 x the per-batch counters of a single-stream run.

  python tools/ab_streams.py [--config 5tuple] [--steps K]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="5tuple")
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    dev = torch.device("cuda", 0)
    n = 1 << 20
    prog = Program(W.program(args.config))
    prog.upload(0)
    bufs = [torch.from_numpy(W.frames_fixed(n, 64, 3 + 100 * k)).to(dev) for k in range(8)]
    descs = [prog.make_batch(b, n=n, stride=64, mem_size=1024, r10=512) for b in bufs]
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    outs, cnts, verds = [], [], []
    for s in range(4):
        v = torch.empty(n, dtype=torch.uint8, device=dev)
        c = torch.zeros(8, dtype=torch.int64, device=dev)
        o = _lib.BatchOut()
        o.verdict = v.data_ptr()
        o.counters = c.data_ptr()
        outs.append(o)
        cnts.append(c)
        verds.append(v)
    for s in range(4):  # warm every stream's workspace
        for i in range(8):
            prog.launch(descs[i], outs[s], streams[s])
    torch.cuda.synchronize()

    def run(S):
        for c in cnts:
            c.zero_()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        for s in range(1, S):
            streams[s].wait_event(e0)
        for i in range(args.steps):
            s = i % S
            prog.launch(descs[i % 8], outs[s], streams[s])
        for s in range(1, S):
            ev = torch.cuda.Event()
            ev.record(streams[s])
            streams[0].wait_event(ev)
        e1.record(streams[0])
        torch.cuda.synchronize()
        tot = sum(c.cpu() for c in cnts)
        return e0.elapsed_time(e1) * 1e3 / args.steps, [int(x) for x in tot]

    ref = None
    for rep in range(2):
        for S in (1, 2, 3, 4):
            us, tot = run(S)
            if ref is None:
                ref = tot
            ok = tot == ref
            print(f"S={S} {us:.3f} us/batch {1e-3 * n / us:.2f} Gpkt/s counters {'same' if ok else tot}",
                  flush=True)


if __name__ == "__main__":
    main()
