#!/usr/bin/env python3
"""End-to-end rate of the XDP path when packets start and end in host memory (the north star's
"pcap buffer or NIC ring" case): pinned host frames -> H2D copy -> interpreter kernel -> D2H copy
of the verdict bytes, chunked and pipelined over three HIP streams (copy-in, compute, copy-out)
so that the PCIe transfers of chunk i+1 / i-1 overlap the kernel of chunk i.

Prints one JSON line: end-to-end Mpkt/s, the H2D-only rate over the same chunks, and the
device-resident kernel rate, for the DESIGN.md table. Not the driver's bench (see bench.py).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="5tuple", choices=["5tuple", "drop"])
    ap.add_argument("--packets", type=int, default=16 << 20)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pcap", action="store_true",
                    help="the packets as one classic pcap capture (16-byte record headers between "
                         "the frames), through ebpf_emu.pcap.Capture: index, chunked H2D, kernel, "
                         "verdict D2H")
    args = ap.parse_args()
    if args.pcap:
        return pcap_e2e(args)

    import numpy as np
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    dev = torch.device("cuda", 0)
    n, c = args.packets, args.chunk
    assert n % c == 0
    nchunks = n // c
    one = W.frames_fixed(c, 64, 3)
    host = torch.empty(n * 64, dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    for i in range(nchunks):  # distinct chunks: re-seeded copies of the synthetic batch
        hv[i * c * 64:(i + 1) * c * 64] = np.roll(one, i * 64)
    verdict_host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    prog = Program(W.program(args.config))
    prog.upload(0)
    nbuf = 3
    dframes = [torch.empty(c * 64, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    dverd = [torch.empty(c, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    s_in, s_k, s_out = (torch.cuda.Stream(dev) for _ in range(3))
    descs = [prog.make_batch(dframes[i], n=c, stride=64) for i in range(nbuf)]
    outs = []
    for i in range(nbuf):
        o = _lib.BatchOut()
        o.verdict = dverd[i].data_ptr()
        o.counters = counters.data_ptr()
        outs.append(o)

    def run_e2e():
        ev_in = [torch.cuda.Event() for _ in range(nchunks)]
        ev_k = [torch.cuda.Event() for _ in range(nchunks)]
        ev_out = [torch.cuda.Event() for _ in range(nchunks)]
        for i in range(nchunks):
            b = i % nbuf
            with torch.cuda.stream(s_in):
                if i >= nbuf:
                    s_in.wait_event(ev_k[i - nbuf])  # buffer b free again
                dframes[b].copy_(host[i * c * 64:(i + 1) * c * 64], non_blocking=True)
                ev_in[i].record(s_in)
            s_k.wait_event(ev_in[i])
            if i >= nbuf:
                s_k.wait_event(ev_out[i - nbuf])  # verdict buffer b drained
            prog.launch(descs[b], outs[b], s_k)
            ev_k[i].record(s_k)
            with torch.cuda.stream(s_out):
                s_out.wait_event(ev_k[i])
                verdict_host[i * c:(i + 1) * c].copy_(dverd[b], non_blocking=True)
                ev_out[i].record(s_out)
        torch.cuda.synchronize(dev)

    def run_h2d():
        for i in range(nchunks):
            dframes[i % nbuf].copy_(host[i * c * 64:(i + 1) * c * 64], non_blocking=True)
        torch.cuda.synchronize(dev)

    def run_kernel():
        for i in range(nchunks):
            prog.launch(descs[i % nbuf], outs[i % nbuf], s_k)
        torch.cuda.synchronize(dev)

    res = {}
    for name, fn in (("e2e", run_e2e), ("h2d_only", run_h2d), ("kernel_only", run_kernel)):
        fn()
        best = 1e9
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
        res[name] = best
    # parity spot check of the end-to-end output against a device-resident run of chunk 0
    ref = prog.run(dframes[0].copy_(host[:c * 64]), n=c, stride=64)
    torch.cuda.synchronize(dev)
    assert torch.equal(ref.verdict.cpu(), verdict_host[:c]), "e2e verdicts differ"
    print(json.dumps({
        "config": args.config, "packets": n, "chunk": c, "frame_bytes": 64,
        "e2e_mpps": round(n / res["e2e"] / 1e6, 1),
        "e2e_GBps_h2d": round(n * 64 / res["e2e"] / 1e9, 2),
        "h2d_only_mpps": round(n / res["h2d_only"] / 1e6, 1),
        "h2d_only_GBps": round(n * 64 / res["h2d_only"] / 1e9, 2),
        "kernel_only_mpps": round(n / res["kernel_only"] / 1e6, 1),
    }))


def pcap_e2e(args):
    """End to end from a capture in host memory: the capture's bytes (frames + record headers)
    cross PCIe as they are; offsets / lengths come from ebpf_pcap_index."""
    import numpy as np
    import torch

    from ebpf_emu import Program, pcap
    from ebpf_emu import workloads as W

    n, c = args.packets, args.chunk
    one = W.frames_fixed(c, 64, 3).reshape(c, 64)
    # the capture: 24-byte header, then n records of 16 + 64 bytes (distinct rolled copies)
    rec = np.zeros((n, 80), dtype=np.uint8)
    hdr = np.frombuffer(pcap.to_bytes([bytes(64)])[24:40], dtype=np.uint8)
    rec[:, :16] = hdr
    for i in range(n // c):
        rec[i * c:(i + 1) * c, 16:] = np.roll(one, i, axis=0)
    buf = np.concatenate([np.frombuffer(pcap.to_bytes([])[:24], dtype=np.uint8), rec.reshape(-1)])
    t0 = time.perf_counter()
    cap = pcap.Capture(buf)
    t_stage = time.perf_counter() - t0
    prog = Program(W.program(args.config))
    prog.upload(0)
    cap.run(prog, packets_per_chunk=c)
    best = 1e9
    for _ in range(args.reps):
        t0 = time.perf_counter()
        verdict, counters = cap.run(prog, packets_per_chunk=c)
        best = min(best, time.perf_counter() - t0)
    # parity spot check: chunk 0's verdicts against a device-resident fixed-slot run
    dev = torch.device("cuda", 0)
    ref = prog.run(torch.from_numpy(rec[:c, 16:].reshape(-1).copy()).to(dev), n=c, stride=64)
    torch.cuda.synchronize(dev)
    assert torch.equal(ref.verdict.cpu(), verdict[:c]), "pcap verdicts differ"
    print(json.dumps({
        "config": args.config, "source": "pcap capture in pinned host memory", "packets": n,
        "chunk": c, "frame_bytes": 64, "capture_bytes": int(buf.nbytes),
        "e2e_mpps": round(n / best / 1e6, 1),
        "e2e_GBps_h2d": round(buf.nbytes / best / 1e9, 2),
        "index_and_pin_s": round(t_stage, 3),
    }))


if __name__ == "__main__":
    main()
