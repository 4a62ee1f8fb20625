#!/usr/bin/env python3
"""Where the wall clock of bench.py's timed region goes beyond the HIP-event time of its K steps.

For K in (1, 5, 20, 200) and three ways of waiting / launching:
  sync   : K launches, then torch.cuda.synchronize()
  poll   : K launches, then busy-poll the end event, then synchronize
  graph  : the K launches captured once into a HIP graph, replayed; busy-poll the end event
prints wall us per step, event us per step, and the fixed wall overhead (wall - event) per run.
Also an empty-stream round trip (event record + poll) and the host time of one launch call.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))


def main():
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    dev = torch.device("cuda", 0)
    n = 1 << 20
    prog = Program(W.program("5tuple"))
    prog.upload(0)
    batches = [torch.from_numpy(W.frames_fixed(n, 64, 3 + 100 * k)).to(dev) for k in range(8)]
    descs = [prog.make_batch(b, n=n, stride=64) for b in batches]
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    out = _lib.BatchOut()
    out.verdict = verdict.data_ptr()
    out.counters = counters.data_ptr()
    res = {}
    s = torch.cuda.Stream(dev)

    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    null = torch.cuda.current_stream(dev)

    def run(K, mode, graph=None):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        st = null if mode in ("null", "null_hipsync") else s
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(st)
        if graph is not None:
            graph.replay()
        else:
            for i in range(K):
                prog.launch(descs[i % 8], out, st)
        ev1.record(st)
        if mode in ("hipsync", "null_hipsync"):
            hip.hipStreamSynchronize(ctypes.c_void_p(st.cuda_stream))
        elif mode not in ("sync", "null"):
            while not ev1.query():
                pass
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        return (t1 - t0) * 1e6 / K, ev0.elapsed_time(ev1) * 1e3 / K

    for i in range(30):
        prog.launch(descs[i % 8], out, s)
    torch.cuda.synchronize(dev)
    for K in (1, 5, 20, 200):
        for mode in ("sync", "poll", "graph", "null", "hipsync", "null_hipsync"):
            g = None
            if mode == "graph":
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for i in range(K):
                        prog.launch(descs[i % 8], out, s)
                g.replay()
                torch.cuda.synchronize(dev)
            walls, evs = [], []
            for rep in range(7):
                w, e = run(K, mode, g)
                walls.append(w)
                evs.append(e)
            walls.sort()
            evs.sort()
            w, e = walls[3], evs[3]
            res[f"K{K}_{mode}"] = {"wall_us_per_step": round(w, 3), "event_us_per_step": round(e, 3),
                                   "fixed_us": round((w - e) * K, 2)}
            print(K, mode, res[f"K{K}_{mode}"], flush=True)
    # empty-stream round trip
    rts = []
    for _ in range(20):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e = torch.cuda.Event()
        e.record(s)
        while not e.query():
            pass
        rts.append((time.perf_counter() - t0) * 1e6)
    rts.sort()
    res["empty_roundtrip_us"] = round(rts[10], 2)
    t0 = time.perf_counter()
    for i in range(200):
        prog.launch(descs[i % 8], out, s)
    res["launch_call_us"] = round((time.perf_counter() - t0) * 1e6 / 200, 3)
    torch.cuda.synchronize(dev)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
