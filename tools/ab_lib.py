#!/usr/bin/env python3
"""A/B of two builds of the library on one box (diagnostic): the 5-tuple over 1 Mi x 64 B frames
as an offsets + lens batch (or fixed slots with --fixed), HIP-event us per batch over K launches,
with the package taken from PKGDIR (e.g. a worktree of an older commit, built in place).

  python tools/ab_lib.py PKGDIR [--fixed] [--steps K]
"""
import argparse
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pkgdir")
    ap.add_argument("--fixed", action="store_true")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--config", default="5tuple")
    args = ap.parse_args()
    sys.path.insert(0, args.pkgdir)
    import numpy as np
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    dev = torch.device("cuda", 0)
    n = 1 << 20
    prog = Program(W.program(args.config))
    prog.upload(0)
    descs = []
    keep = []
    for k in range(8):  # 8 distinct batches (> the Infinity Cache with the other buffers)
        buf = W.frames_fixed(n, 64, 3 + k)
        fr = torch.from_numpy(buf).to(dev)
        keep.append(fr)
        if args.fixed:
            descs.append(prog.make_batch(fr, n=n, stride=64, mem_size=1024, r10=512))
        else:
            off = torch.from_numpy((np.arange(n, dtype=np.int64) * 64).astype(np.uint32).view(np.int32)).to(dev)
            ln = torch.from_numpy(np.full(n, 64, dtype=np.int16)).to(dev)
            keep += [off, ln]
            descs.append(prog.make_batch(fr, n=n, offsets=off, lens=ln, mem_size=1024, r10=512))
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    out = _lib.BatchOut()
    out.verdict = verdict.data_ptr()
    out.counters = counters.data_ptr()
    stream = torch.cuda.current_stream(dev)
    for i in range(20):
        prog.launch(descs[i % 8], out, stream)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(args.steps):
        prog.launch(descs[i % 8], out, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.steps
    kid = prog.batch_kernel(descs[0], out, 0)
    print(f"{args.pkgdir} {'fixed' if args.fixed else 'offsets'} {us:.3f} us/batch kernel {_lib.KERNEL_NAMES[kid]}")


if __name__ == "__main__":
    main()
