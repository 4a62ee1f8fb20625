#!/usr/bin/env python3
"""A/B of two builds of libebpfemu.so on one box: bench.py runs alternating between the in-tree
library (B) and another build (A, EBPFEMU_LIB_PATH), `rounds` times per config; prints the median
HIP-event us per batch of each and writes gpurun_out/ab_<tag>.json.
usage: tools/ab_bench.py <A.so> <tag> <rounds> <config>[:extra bench args] ...
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lib, config, extra):
    env = dict(os.environ)
    if lib:
        env["EBPFEMU_LIB_PATH"] = lib
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", config, "--cpu-seconds", "0",
           "--steps", "200", "--warmup", "20"] + extra
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    for ln in out.stdout.splitlines():
        if ln.startswith("{"):
            d = json.loads(ln)
            return d["roofline"]["kernel_avg_us"], d["ms_per_step"] * 1e3
    raise RuntimeError(out.stderr[-2000:])


def main():
    a_lib, tag, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3])
    res = {}
    for spec in sys.argv[4:]:
        config, _, extra = spec.partition(":")
        extra = extra.split() if extra else []
        ev = {"A": [], "B": []}
        for r in range(rounds):
            for k, lib in (("A", a_lib), ("B", None)):
                e, w = run(lib, config, extra)
                ev[k].append(e)
                print(spec, k, r, e, w, flush=True)
        res[spec] = {k: {"median_us": statistics.median(v), "runs": v} for k, v in ev.items()}
        print(spec, "A", res[spec]["A"]["median_us"], "B", res[spec]["B"]["median_us"], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"ab_{tag}.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
