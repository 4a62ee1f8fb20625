#!/usr/bin/env python3
"""Per-batch time of an xdp_md loop program (diagnostic, not the driver's bench): the per-byte
checksum as a standard XDP program (workloads.CHECKSUM_XDP) vs the plain checksum (CHECKSUM) on
the same 1 Mi mixed 64/1500-byte batch (config 5's frames, offsets + lens): in place (variant 6,
the program rebased, jit.cpp Compiler::xdp_rebase), or staged with EBPFEMU_XDP_STAGE=1 (the
xdp_stage copy, then variant 5). HIP events around K back-to-back batches on one stream.
  python tools/xdp_loop_bench.py [--packets N] [--steps K] [--stage]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))


def main():
    if "--stage" in sys.argv:  # (read by the library when it loads)
        os.environ["EBPFEMU_XDP_STAGE"] = "1"
    import numpy as np
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--stage", action="store_true", help="stage every xdp_md batch (A/B)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = args.packets
    buf, offs, lens = W.frames_mixed(n)
    frames = torch.from_numpy(buf).to(dev)
    kw = dict(n=n, offsets=torch.from_numpy(offs.view(np.int32)).to(dev),
              lens=torch.from_numpy(lens.view(np.int16)).to(dev), mem_size=2048, r10=2048)
    res = {}
    for name, xdp in (("checksum", False), ("checksum_xdp", True)):
        prog = Program(W.program(name))
        desc = prog.make_batch(frames, xdp_md=xdp, **kw)
        out = _lib.BatchOut()
        verdict = torch.empty(n, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(8, dtype=torch.int64, device=dev)
        out.verdict = verdict.data_ptr()
        out.counters = cnt.data_ptr()
        s = torch.cuda.current_stream(dev)
        for _ in range(3):
            prog.launch(desc, out, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.steps):
            prog.launch(desc, out, s)
        e1.record(s)
        torch.cuda.synchronize()
        res[name] = {"us_per_batch": round(e0.elapsed_time(e1) * 1e3 / args.steps, 2),
                     "kernel": _lib.KERNEL_NAMES[prog.batch_kernel(desc, out)],
                     "staged": prog.batch_staged(desc, out),
                     "verdict_crc": int(np.bitwise_xor.reduce(verdict.cpu().numpy().astype(np.uint64)))}
        prog.close()
    res["xdp_minus_plain_us"] = round(res["checksum_xdp"]["us_per_batch"] - res["checksum"]["us_per_batch"], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
