#!/usr/bin/env python3
"""Prints value / event time per step / kernel of bench.py lines in gpurun_out/<name>.log."""
import json
import os
import sys

for name in sys.argv[1:]:
    p = os.path.join("gpurun_out", name + ".log")
    if not os.path.exists(p):
        print(name, "missing")
        continue
    lines = [l for l in open(p) if l.startswith("{")]
    if not lines:
        print(name, "no bench line")
        continue
    d = json.loads(lines[-1])
    print(f"{name:8s} {d['value']:10.2f} {d['unit']} {d['roofline']['kernel_avg_us']:9.3f} us "
          f"{d['roofline']['kernel']}")
