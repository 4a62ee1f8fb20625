#!/usr/bin/env python3
"""Where the driver-style run's fixed wall cost goes: bench.py's timed region (K steps of the
5-tuple over 1 Mi x 64 B frames on two streams) in several variants, interleaved in one process
so the box and its clocks are the same for all of them.

Variants (each: synchronize, t0, K launches, the variant's end sequence, synchronize, t1):
  cur       bench.py round 4: ev0 on stream 0, stream 1 waits on ev0 after the first launch,
            stream 0 joins stream 1 (event + wait) before the end event
  nojoin    no join: an end event on each stream; event time = the later of the two
  nowait    nojoin, and stream 1 does not wait on ev0 either
  last0     the steps' streams rotated so that step K-1 runs on stream 0 (ev0 on the first
            step's stream, the other stream waits on it after the first launch; join as cur)
  fast      nojoin with a pre-bound ctypes call per step (no per-call argument conversion)
  fastnw    fast + nowait
  last0nw   last0 without the start wait
  last0s3   last0 on three streams
Prints the median wall and event us per step and the fixed part (wall - event) x K per variant.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))


def main():
    import numpy as np
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    K = int(os.environ.get("K", "20"))
    reps = int(os.environ.get("REPS", "60"))
    modes = os.environ.get("MODES", "cur,nojoin,nowait,last0,fast,fastnw").split(",")
    S = 3 if any(m.endswith("s3") for m in modes) else 2
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 1 << 20
    prog = Program(W.program("5tuple"))
    prog.upload(0)
    batches = [torch.from_numpy(W.frames_fixed(n, 64, 3 + 100 * k)).to(dev) for k in range(8)]
    descs = [prog.make_batch(b, n=n, stride=64) for b in batches]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    ws_bytes = prog.workspace_bytes(descs[0], 0)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    sd, outs, keep = [], [], []
    for si in range(S):
        ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
        v = torch.empty(n, dtype=torch.uint8, device=dev)
        keep += [ws, v]
        row = []
        for bd in descs:
            b2 = type(bd).from_buffer_copy(bd)
            b2.workspace = ws.data_ptr()
            b2.workspace_bytes = ws_bytes
            row.append(b2)
        sd.append(row)
        o = _lib.BatchOut()
        o.verdict = v.data_ptr()
        o.counters = counters.data_ptr()
        outs.append(o)
    # a second handle on ebpf_run_batch without argtypes: arguments pre-converted once
    raw = ctypes.CDLL(_lib.LIB_PATH).ebpf_run_batch
    raw.restype = ctypes.c_int
    pre = [[(prog._h, ctypes.byref(sd[si][j]), ctypes.byref(outs[si]),
             ctypes.c_void_p(streams[si].cuda_stream)) for j in range(len(descs))]
           for si in range(S)]

    def step_slow(i, si):
        prog.launch(sd[si][i % len(descs)], outs[si], streams[si])

    def step_fast(i, si):
        a = pre[si][i % len(descs)]
        if raw(*a):
            raise RuntimeError("ebpf_run_batch")

    def run(mode):
        fast = mode.startswith("fast")
        step = step_fast if fast else step_slow
        wait = mode not in ("nowait", "fastnw", "last0nw")
        join = mode in ("cur", "last0", "last0nw", "last0s3")
        rot = mode.startswith("last0")
        SS = 3 if mode.endswith("s3") else 2
        sof = (lambda i: (K - 1 - i) % SS) if rot else (lambda i: i % SS)
        first = sof(0)
        ev0 = torch.cuda.Event(enable_timing=True)
        ends = [torch.cuda.Event(enable_timing=True) for _ in range(S)]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(streams[first])
        for i in range(K):
            if i == 1 and wait:
                for si in range(SS):
                    if si != first:
                        streams[si].wait_event(ev0)
            step(i, sof(i))
        last = sof(K - 1)
        if join:
            for si in range(SS):
                if si != last:
                    ej = torch.cuda.Event()
                    ej.record(streams[si])
                    streams[last].wait_event(ej)
            ends[0].record(streams[last])
            used = [ends[0]]
        else:
            for si in range(SS):
                ends[si].record(streams[si])
            used = ends[:SS]
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        ev = max(ev0.elapsed_time(e) for e in used) * 1e3
        return (t1 - t0) * 1e6, ev

    for i in range(40):
        step_slow(i, i % 2)
    torch.cuda.synchronize(dev)
    res = {m: [] for m in modes}
    for r in range(reps):
        for m in (modes if r % 2 == 0 else modes[::-1]):
            res[m].append(run(m))
    out = {"K": K, "reps": reps}
    for m in modes:
        w = sorted(x[0] for x in res[m])
        e = sorted(x[1] for x in res[m])
        fx = sorted(x[0] - x[1] for x in res[m])
        med = len(w) // 2
        out[m] = {"wall_us_per_step": round(w[med] / K, 3), "event_us_per_step": round(e[med] / K, 3),
                  "fixed_us": round(fx[med], 2), "wall_p25": round(w[len(w) // 4] / K, 3),
                  "mpps_median": round(n / (w[med] / K), 1)}
        print(m, out[m], flush=True)
    # host cost of one launch call, both ways (no GPU wait in between: the queue fills)
    for nm, st in (("slow", step_slow), ("fast", step_fast)):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(100):
            st(i, 0)
        out[f"launch_call_us_{nm}"] = round((time.perf_counter() - t0) * 1e6 / 100, 3)
        torch.cuda.synchronize(dev)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
