#!/usr/bin/env python3
"""Per-launch device time of overlapping launches, from a rocprofv3 kernel trace: with
bench.py --streams 2 consecutive batches run concurrently, so each kernel's own duration (what
`--stats` averages) is longer than the time the device spends per batch. This prints, for the
kernels whose name contains SUBSTR: the launch count, the mean per-kernel duration, the union of
their busy intervals divided by the launch count (the per-batch device time, which bench.py's
`roofline.kernel_avg_us` measures with HIP events), and how much of the busy time had two or
more of them running at once.

  python tools/rocprof_union.py gpurun_out/<dir>/run_kernel_trace.csv SUBSTR [--skip N]
(--skip: leading launches to drop -- the warmup; --count: launches to keep -- bench.py's timed
steps, before its single-stream calibration launches)
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("substr")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--count", type=int, default=0, help="launches to keep after --skip (0 = all)")
    args = ap.parse_args()
    iv = []
    for row in csv.DictReader(open(args.trace)):
        if args.substr in row.get("Kernel_Name", ""):
            iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    iv.sort()
    iv = iv[args.skip:args.skip + args.count] if args.count else iv[args.skip:]
    if not iv:
        raise SystemExit("no matching kernels")
    busy = 0
    cur_s, cur_e = iv[0]
    for s, e in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    # time with >= 2 launches running: sweep over start / end events
    ev = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv])
    depth, last, overlap = 0, ev[0][0], 0
    for t, d in ev:
        if depth >= 2:
            overlap += t - last
        depth += d
        last = t
    n = len(iv)
    print(json.dumps({
        "kernel": args.substr, "launches": n,
        "mean_kernel_us": round(sum(e - s for s, e in iv) / n / 1e3, 3),
        "union_busy_us_per_launch": round(busy / n / 1e3, 3),
        "overlapped_share_of_busy": round(overlap / busy, 4),
        "span_us": round((iv[-1][1] - iv[0][0]) / 1e3, 3),
        "span_us_per_launch": round((iv[-1][1] - iv[0][0]) / n / 1e3, 3),
    }, indent=1))


if __name__ == "__main__":
    main()
