#!/usr/bin/env python3
"""bench.py — device-resident throughput of the batched eBPF/XDP interpreter on MI355X.

Metric (BASELINE.json): Mpkt/s device-resident, 64 B frames, fixed XDP program; achieved HBM
GB/s vs peak. A "step" = one launch of the interpreter over one batch of synthetic frames
already resident in HBM (verdict byte per packet + the per-verdict counters). Default workload
= BASELINE configs[2]: the ~32-instruction IPv4 5-tuple classifier over 1 Mi x 64 B frames, the
program the ">= 10 Gpkt/s" target is quoted on. `--config drop|checksum` runs configs 2 / 5.
Batches rotate over a pool larger than the 256 MiB Infinity Cache, so every step streams its
frames from HBM. Steps alternate over two HIP streams (--streams, default 2; each stream with
its own workspace and verdict buffer, one counters array): consecutive batches overlap, the next
batch's ramp under the previous one's tail, as a NIC's queues would feed them.
`roofline.kernel_avg_us` is then the device time per batch; `kernel_single_us` one launch at a
time (measured after the timed region; `--streams 1` times that way throughout).

Multi-GPU (`bench.py --gpus N`, which starts N rank processes itself, or the same under
python -m torch.distributed.run --nproc-per-node N): one rank per GPU, each rank owns its own
shard of packets (weak scaling: per-GPU work fixed; pool batch k of rank r is seeded chunk
k*N + r); the only collective is one RCCL all-reduce of the 8 per-verdict counters per job.
value = packets of all ranks / max time. The reduced counters are checked against the oracle's
counters of those chunks (tests/golden/bench_pins.json): `parity_pinned`.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CONFIGS = {
    # name: (BASELINE configs index, description)
    "5tuple": (2, "IPv4 5-tuple header parse -> PASS/DROP (31 insns) over 1Mi x 64B frames"),
    "drop": (1, "XDP_DROP-all (3 insns) over 1Mi x 64B frames"),
    "checksum": (4, "per-byte checksum loop over 1Mi mixed 64B/1500B frames"),
    # the 5-tuple with its flow key spilled to the stack and reloaded (memory tier 0.5: the
    # stack window in registers of the compiled kernel); same frames and verdicts as 5tuple
    "stack": (2, "IPv4 5-tuple, flow key spilled to r10-16 and reloaded (38 insns) over 1Mi x 64B frames"),
    # stores into the packet's header window and an atomic on the stack (memory tier 0.5 with
    # packet-window stores; --generic: the general interpreter's tier 1)
    "tier1": (2, "XDP_TX MAC-swap reflector with packet stores and a stack atomic (17 insns) over 1Mi x 64B frames"),
    # a ~100-instruction firewall (past the tile interpreter's 62 micro-ops: the forward-program
    # compiler), same frames as 5tuple
    "acl": (2, "IPv4/IPv6 ACL firewall (97 insns) over 1Mi x 64B frames"),
    # the 5-tuple as a standard XDP program under the xdp_md calling convention (xdp.rs:16-20:
    # r1 = ctx, data / data_end read from it), same frames as 5tuple; the ctx is synthesised in
    # the kernel's window (no staging copy)
    "xdp": (2, "IPv4 5-tuple as a standard XDP program, xdp_md ctx (38 insns) over 1Mi x 64B frames"),
    # config 5 with the running sum in a stack slot (memory tier 0.5 with a loop: the loop kernel's
    # stack variant; --generic: the general interpreter's tier 1)
    "checksum_stack": (4, "per-byte checksum loop, sum kept at r10-8, over 1Mi mixed 64B/1500B frames"),
    # the 5-tuple with its L4 decision in a local function (CALL / EXIT flattened at load time onto
    # the compiled kernel; --generic: the general interpreter's frame stack), same verdicts
    "call": (2, "IPv4 5-tuple with the L4 decision as a local call (35 insns) over 1Mi x 64B frames"),
    # a NAT / router rewrite: TTL - 1 with the header checksum, ports 53/80 redirected through the
    # L4 header pointer behind the IPv4 options (a register-address store: store mode, the var
    # kernel with the header window in LDS; --generic: the general interpreter's tier 1)
    "nat": (2, "IPv4 NAT rewrite: TTL - 1 + checksum, port redirect through the L4 pointer (40 insns) "
               "over 1Mi x 64B frames"),
    # config 5 as a standard XDP program: the sum over ctx->data .. ctx->data_end (a loop program's
    # xdp_md batch: staged images, compiled with the staged ctx known -- DESIGN 3.17)
    "checksum_xdp": (4, "per-byte checksum as a standard XDP program (xdp_md ctx) over 1Mi mixed "
                        "64B/1500B frames"),
    # the same with ctx->data_end reloaded in every iteration (the loop reads the ctx: in place
    # through the loop kernels' ctx-aware refills -- DESIGN 3.17, 3.29)
    "checksum_xdp_reload": (4, "per-byte checksum as an XDP program reloading ctx->data_end every "
                               "iteration over 1Mi mixed 64B/1500B frames"),
    # a long program: a 128-rule firewall chain (workloads.acl_rules_source, 1013 insns, ~297 run
    # per packet) -- compiled past the near-branch reach (jit.cpp far mode); issue-bound, not HBM
    "acl_rules": (2, "IPv4 rule-table firewall, 128 rules (1013 insns, ~297 executed per packet) "
                     "over 1Mi x 64B frames"),
    # a payload writer: ICMP echo replies in place, and every other IPv4 frame's 4-byte trailer
    # (the frame's last bytes: r1 + r2 - 4) incremented -- register-address stores; with
    # --frame-bytes 1504 the trailer is 1500 bytes in, past the header window: store mode's
    # overflow image (jit.cpp ovf_fill, one 64-byte block per packet)
    "responder": (2, "XDP responder: ICMP echo reply in place + a 4-byte telemetry trailer "
                     "incremented at the frame's end (49 insns) over 1Mi x 64B frames"),
}
PROGRAM_OF = {"stack": "5tuple_stack", "tier1": "mac_swap_tx", "xdp": "5tuple_xdp",
              "call": "5tuple_call"}
MIXED_CONFIGS = ("checksum", "checksum_stack", "checksum_xdp", "checksum_xdp_reload")
XDP_CONFIGS = ("xdp", "checksum_xdp", "checksum_xdp_reload")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU). Without WORLD_SIZE in the environment, N > 1 "
                         "starts N rank processes itself (before any GPU call); under torchrun "
                         "it must equal WORLD_SIZE. Default: WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="5tuple")
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per batch per GPU")
    ap.add_argument("--layout", choices=["fixed", "offsets", "pcap"], default="fixed",
                    help="64-byte-frame configs: fixed slots (a NIC ring), the same frames as an "
                         "offsets + lens batch at 64-byte slots (the var kernels), or as a classic "
                         "pcap capture (24-byte file header, a 16-byte record header before each "
                         "frame: records at 8 mod 16) indexed in place by ebpf_pcap_index")
    ap.add_argument("--frame-bytes", type=int, default=64,
                    help="fixed-slot configs: bytes per frame slot (rounded up to 16; e.g. 1500)")
    ap.add_argument("--long-options", type=int, default=0,
                    help="64-byte-frame configs: every Nth frame's IPv4 IHL set to 15 (options up "
                         "to byte 74: the NAT's port store past the 64-byte header window)")
    ap.add_argument("--total-packets", type=int, default=0,
                    help="strong scaling: one global batch of this many packets (BASELINE config 4"
                         " = 100000000), sharded over the ranks in seeded 1Mi-packet chunks")
    ap.add_argument("--pool-mib", type=int, default=512, help="min bytes of distinct batches")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0=skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU this process may use (affinity, capped by the cgroup quota)")
    ap.add_argument("--cpu-seconds-1core", type=float, default=4.0,
                    help="single-thread CPU baseline budget (0 = skip)")
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams the steps alternate over (each with its own workspace and "
                         "verdict buffer): consecutive batches overlap, one's ramp under the "
                         "other's tail; 1 = one launch after another")
    ap.add_argument("--settle-ms", type=float, default=0.0,
                    help="untimed clock-settling run of the workload before the W warmup steps "
                         "(host milliseconds; reported as settle_ms)")
    ap.add_argument("--no-counters", action="store_true", help="A/B: verdicts only")
    ap.add_argument("--generic", action="store_true",
                    help="run on the general interpreter (EBPF_BATCH_GENERIC), for comparison")
    ap.add_argument("--pmc-json", default=None,
                    help="PMC summary (tools/pmc_summary.py output) of this workload: its HBM bytes"
                         " per launch (roofline.traffic) and VALU instructions (issue_roofline);"
                         " default profiles/pmc_<config>[_<slot>B].json")
    return ap.parse_args()


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK =
    LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), as torch.distributed.run would.
    The parent never touches the GPU (no HIP call before or after the spawn, no exec); rank 0
    prints the line. If a rank fails, the others are terminated (their exact PIDs). Returns the
    first nonzero exit status, else 0."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in live:  # a peer blocked in a collective would wait forever
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---- the weak-scaling pool: which seeded chunks each rank times, and the fixture that pins them --
PIN_FIXTURE = os.path.join(ROOT, "tests", "golden", "bench_pins.json")


def chunk_id(k: int, rank: int, world: int) -> int:
    """Pool batch k of rank r of W is chunk k*W + r: the ranks' pools are disjoint, and at any W
    the timed chunks are 0 .. B*W-1 (tests/golden/bench_pins.json holds their oracle counters)."""
    return k * world + rank


def chunk_seed(c: int, mixed: bool) -> int:
    """config_id of chunk c: 64-byte frames are the config-4 chunks (dist.chunk_seed); mixed
    64/1500-byte batches use 5 + 100c (chunk 0 = tests/golden/workloads.json's checksum batch)."""
    return 5 + 100 * c if mixed else 3 + 100 * c


def pin_weak(prog_name: str, mixed: bool, frame_bytes: int, n: int, world: int, pool: int,
             steps: int, cnt):
    """Expected global counters of a weak-scaling run (K steps; step i runs pool batch i mod B on
    every rank), from the committed oracle fixture -> (want u64[8], source) or (None, reason)."""
    if not os.path.exists(PIN_FIXTURE):
        return None, f"{os.path.relpath(PIN_FIXTURE, ROOT)} missing"
    with open(PIN_FIXTURE) as f:
        fx = json.load(f)
    p = fx["programs"].get(prog_name)
    if n == 1 << 20 and not mixed and frame_bytes == 1504 and p and "chunk_counters_1504" in p:
        # (1504-byte slots: every pool batch of rank r is a copy of chunk r)
        cc = p["chunk_counters_1504"]
        if world > len(cc):
            return None, f"{world} ranks exceed the fixture's {len(cc)} 1504-byte chunks"
        want = [0] * 8
        for r in range(world):
            for j in range(8):
                want[j] += steps * cc[r][j]
        want = [w & ((1 << 64) - 1) for w in want]
        return want, (f"{os.path.relpath(PIN_FIXTURE, ROOT)}: counters == the oracle's counters of "
                      f"the 1504-byte chunks r over {steps} steps x {world} ranks")
    if n != 1 << 20 or (not mixed and frame_bytes != 64):
        return None, "no fixture for this batch shape (pinned: 1 Mi packets of 64 B or mixed)"
    if p is None or p["frames"] != ("mixed" if mixed else "fixed64"):
        return None, f"no fixture for program {prog_name}"
    cc = p["chunk_counters"]
    if pool * world > len(cc):
        return None, f"pool of {pool} x {world} ranks exceeds the fixture's {len(cc)} chunks"
    want = [0] * 8
    for i in range(steps):
        for r in range(world):
            row = cc[chunk_id(i % pool, r, world)]
            for j in range(8):
                want[j] += row[j]
    want = [w & ((1 << 64) - 1) for w in want]
    src = (f"{os.path.relpath(PIN_FIXTURE, ROOT)}: counters == the oracle's counters of chunks "
           f"k*{world}+r over {steps} steps x {world} ranks")
    return want, src


def stub_rank(args, world, rank):
    """EBPFEMU_BENCH_STUB=1 (CPU test of the launcher, no GPU): every rank takes the counters of
    its own pool chunks from the fixture instead of running kernels, then the same gloo
    reduction, max-over-ranks time and pin check as a real run; rank 0 prints the line."""
    import torch
    import torch.distributed as dist

    if os.environ.get("EBPFEMU_BENCH_STUB_FAIL") == str(rank):  # (test: a rank that dies)
        sys.exit(3)
    dist.init_process_group("gloo")
    prog_name = PROGRAM_OF.get(args.config, args.config)
    mixed = args.config in MIXED_CONFIGS
    if args.total_packets:
        return stub_rank_strong(args, world, rank)
    with open(PIN_FIXTURE) as f:
        cc = json.load(f)["programs"][prog_name]["chunk_counters"]
    # (the pool size bench's loop below reaches for 1 Mi packets per batch)
    pool = 1 if mixed else min(16, -(-args.pool_mib // 64))
    t0 = time.perf_counter()
    mine = [0] * 8
    for i in range(args.steps):
        row = cc[chunk_id(i % pool, rank, world)]
        mine = [a + b for a, b in zip(mine, row)]
    counters = torch.tensor([m - (1 << 64) if m >= 1 << 63 else m for m in mine],
                            dtype=torch.int64)
    dist.all_reduce(counters)
    elapsed = torch.tensor([time.perf_counter() - t0 + 1e-6], dtype=torch.float64)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    cnt = [int(c) & ((1 << 64) - 1) for c in counters.tolist()]
    want, src = pin_weak(prog_name, mixed, 64, 1 << 20, world, pool, args.steps, cnt)
    assert cnt == want, ("counters differ from the fixture", cnt, want)
    if rank == 0:
        n = 1 << 20
        print(json.dumps({"metric": "stub", "value": n * world * args.steps / float(elapsed) / 1e6,
                          "unit": "Mpkt/s", "n_gpus": world, "steps": args.steps,
                          "counters": {"drop": cnt[1], "pass": cnt[2], "insns_retired": cnt[7]},
                          "parity_pinned": src, "stub": True}), flush=True)
    dist.destroy_process_group()


def stub_rank_strong(args, world, rank):
    """The stub for --total-packets (BASELINE config 4, strong scaling): rank r takes the counters
    of its contiguous shard of the global batch's seeded chunks (dist.shard_chunks) from
    tests/golden/config4.json, then the same gloo reduction, max-over-ranks time and the config-4
    pin as a real run."""
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "ebpf-emu_amd"))
    from ebpf_emu import dist as D

    with open(os.path.join(ROOT, "tests", "golden", "config4.json")) as f:
        g4 = json.load(f)
    assert args.config == "5tuple" and g4["total_packets"] == args.total_packets
    sizes = D.chunk_sizes(args.total_packets, D.CHUNK)
    mine = D.shard_chunks(len(sizes), world, rank)
    t0 = time.perf_counter()
    own = [0] * 8
    for _ in range(args.steps):
        for k in mine:
            own = [a + b for a, b in zip(own, g4["chunk_counters"][k])]
    counters = torch.tensor([m - (1 << 64) if m >= 1 << 63 else m for m in own],
                            dtype=torch.int64)
    dist.all_reduce(counters)
    elapsed = torch.tensor([time.perf_counter() - t0 + 1e-6], dtype=torch.float64)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    cnt = [int(c) & ((1 << 64) - 1) for c in counters.tolist()]
    want = [(c * args.steps) & ((1 << 64) - 1) for c in g4["counters"]]
    assert cnt == want, ("config-4 counters differ from tests/golden/config4.json", cnt, want)
    if rank == 0:
        print(json.dumps({"metric": "stub", "value": args.total_packets * args.steps /
                          float(elapsed) / 1e6, "unit": "Mpkt/s", "n_gpus": world,
                          "steps": args.steps, "scaling": "strong",
                          "packets_per_rank": [sum(sizes[k] for k in D.shard_chunks(len(sizes), world, r))
                                               for r in range(world)],
                          "counters": {"drop": cnt[1], "pass": cnt[2], "insns_retired": cnt[7]},
                          "parity_pinned": "tests/golden/config4.json: counters == steps x fixture",
                          "stub": True}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if (args.gpus or 1) > 1:
            sys.exit(launch_ranks(args.gpus))
    elif args.gpus is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("EBPFEMU_BENCH_STUB") == "1":
        return stub_rank(args, world, rank)

    import numpy as np
    import torch
    import torch.distributed as dist

    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    # EBPFEMU_BENCH_DIST=1: the process-group path (RCCL init, barriers, counter all-reduce, max
    # over ranks) even for one rank, to exercise it on a one-GPU box. EBPFEMU_BENCH_BACKEND=gloo
    # rehearses N ranks on one GPU (ranks share device LOCAL_RANK mod count; RCCL refuses two
    # ranks on one device): the plumbing and the pins, not a scaling number.
    use_dist = world > 1 or os.environ.get("EBPFEMU_BENCH_DIST") == "1"
    backend = os.environ.get("EBPFEMU_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    if use_dist:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    def all_reduce(t, op=None):
        op = op or dist.ReduceOp.SUM
        if backend == "nccl":
            dist.all_reduce(t, op=op)
        else:
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)

    cfg_idx, desc = CONFIGS[args.config]
    if args.total_packets:
        desc = desc.replace("1Mi x 64B frames", f"a {args.total_packets}-packet global batch of "
                            "64B frames (seeded 1Mi-packet chunks)")
        cfg_idx = 3 if args.config == "5tuple" else cfg_idx
    if args.frame_bytes != 64 and args.config != "checksum":
        desc = desc.replace("64B frames", f"{(max(64, args.frame_bytes) + 15) // 16 * 16}B frame slots")
    if args.long_options:
        desc += f" (every {args.long_options}th frame with IHL 15)"
    if args.layout != "fixed":
        desc += " (offsets + lens batch)" if args.layout == "offsets" else \
            " (a pcap capture indexed in place: offsets + lens into the capture)"
        assert not args.total_packets and args.config not in MIXED_CONFIGS
    n = args.packets
    img = W.program(PROGRAM_OF.get(args.config, args.config))
    prog = Program(img)
    prog.upload(local)

    # ---- synthetic device-resident batches ----
    from ebpf_emu import dist as D

    mixed = args.config in MIXED_CONFIGS
    fb = (max(64, args.frame_bytes) + 15) // 16 * 16  # fixed slots: 16-byte aligned, >= 64
    batches = []
    pool_bytes = 0
    if args.total_packets:
        # strong scaling: this rank's contiguous shard of a global batch of seeded chunks
        assert not mixed, "--total-packets is defined for the 64-byte-frame configs"
        sizes = D.chunk_sizes(args.total_packets, D.CHUNK)
        mine = D.shard_chunks(len(sizes), world, rank)
        n = sum(sizes[k] for k in mine)
        # (the chunks tests/golden/config4.json pins: dist.chunk_frames, one seed formula)
        buf = np.concatenate([D.chunk_frames(k, sizes[k]) for k in mine])
        batches.append(dict(frames=torch.from_numpy(buf).to(dev)))
        algo_bytes = n * (64 + 1)
        floor_bytes = n * (64 + 1)
        pool_bytes = buf.nbytes
    k = 0
    while not args.total_packets:
        # weak scaling: a pool of distinct batches per rank (pool batch k of rank r is seeded
        # chunk k*W + r, chunk_id), larger than the Infinity Cache so that every step streams from
        # HBM; tests/golden/bench_pins.json holds the oracle's counters of every such chunk
        cid = chunk_seed(chunk_id(k, rank, world), mixed)
        if mixed:
            buf, offs, lens = W.frames_mixed(n, config_id=cid)
            batches.append(dict(frames=torch.from_numpy(buf).to(dev),
                                offsets=torch.from_numpy(offs.view(np.int32)).to(dev),
                                lens=torch.from_numpy(lens.view(np.int16)).to(dev)))
            algo_bytes = int(lens.astype(np.int64).sum()) + n * (4 + 2 + 1)
            floor_bytes = line_floor_bytes(offs.astype(np.int64), lens.astype(np.int64)) + n * (4 + 2 + 1)
        elif fb == 64 or k == 0:
            buf = W.frames_fixed(n, fb, cid)
            if args.long_options:
                v = buf.reshape(n, fb)
                v[::args.long_options, 14] = (v[::args.long_options, 14] & 0xF0) | 0x0F
            batches.append(dict(frames=torch.from_numpy(buf).to(dev)))
            if args.layout == "offsets":  # the same frames through u32 offsets + u16 lengths
                batches[-1]["offsets"] = torch.from_numpy(
                    (np.arange(n, dtype=np.int64) * fb).astype(np.uint32).view(np.int32)).to(dev)
                batches[-1]["lens"] = torch.from_numpy(np.full(n, fb, dtype=np.int16)).to(dev)
            elif args.layout == "pcap":  # the same frames as a capture, indexed in place
                cap = pcap_capture(buf.reshape(n, fb))
                from ebpf_emu import pcap as PC

                offs, lens, _ = PC.index(cap)
                assert len(offs) == n and (lens == fb).all()
                batches[-1] = dict(frames=torch.from_numpy(cap).to(dev),
                                   offsets=torch.from_numpy(offs.view(np.int32)).to(dev),
                                   lens=torch.from_numpy(lens.view(np.int16)).to(dev))
            # a header program's algorithmic bytes are its packet's 64-byte header
            # window + the verdict byte (+ offset and length) = 65 B per 64-byte frame. The floor
            # is what HBM must move for them: the 128-byte lines the bytes the launch reads touch
            # (on fixed slots only the 16-byte chunks the program's loads reach, jit.cpp
            # window_chunks: 16 for drop-all, all 64 with a register-address load)
            wb = prog.window_bytes if args.layout == "fixed" and not args.generic else 64
            meta = 6 if args.layout != "fixed" else 0
            algo_bytes = n * (64 + 1 + meta)
            # (a capture's records: 16-byte record headers between the frames)
            st = np.arange(n, dtype=np.int64) * ((fb + 16) if args.layout == "pcap" else fb) + \
                (40 if args.layout == "pcap" else 0)
            floor_bytes = line_floor_bytes(st, np.full(n, wb, dtype=np.int64)) + n * (1 + meta)
            if args.config == "responder" and fb > 64:  # (+ the 4-byte trailer at the frame's end:
                algo_bytes += n * 4                      #  its 128-byte line, past the window)
                floor_bytes += n * 128
        else:  # large slots: copies of the first batch at other addresses (host RNG is slow)
            batches.append(dict(frames=batches[0]["frames"].clone()))
        # (the bytes a launch touches decide whether the pool outgrows the Infinity Cache)
        pool_bytes += buf.nbytes if mixed else n * 64
        k += 1
        if pool_bytes >= args.pool_mib * (1 << 20) or k >= 16:
            break
    mem_size, r10 = (2048, 2048) if mixed or fb > 1024 else (1024, 512)
    verdict = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    counters = torch.zeros(8, dtype=torch.int64, device=dev)

    from ebpf_emu import _lib

    descs = []
    for b in batches:
        if mixed:
            bd = prog.make_batch(b["frames"], n=n, offsets=b["offsets"], lens=b["lens"],
                                 mem_size=mem_size, r10=r10, generic=args.generic,
                                 xdp_md=args.config in XDP_CONFIGS)
        else:
            bd = prog.make_batch(b["frames"], n=n, stride=fb, offsets=b.get("offsets"),
                                 lens=b.get("lens"), mem_size=mem_size, r10=r10,
                                 generic=args.generic, xdp_md=args.config in XDP_CONFIGS)
        descs.append(bd)
    # S streams (--streams): step i runs on stream i mod S with that stream's own workspace
    # (counter shards, zeroed once) and verdict buffer; every launch adds into the one counters
    # array (the library's fold is an atomic add). Stream 0 is the current stream.
    S = max(1, args.streams)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    ws_bytes = max(prog.workspace_bytes(bd, local) for bd in descs)
    verdicts = [verdict] + [torch.empty_like(verdict) for _ in range(S - 1)]
    workspaces, sdescs, outs = [], [], []
    for si in range(S):
        ws = torch.zeros(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        workspaces.append(ws)
        row = []
        for bd in descs:
            b2 = type(bd).from_buffer_copy(bd)
            b2.workspace = ws.data_ptr()
            b2.workspace_bytes = ws_bytes
            row.append(b2)
        sdescs.append(row)
        o = _lib.BatchOut()
        o.verdict = verdicts[si].data_ptr()
        o.counters = None if args.no_counters else counters.data_ptr()
        outs.append(o)
    out = outs[0]
    stream = streams[0]

    # step i of k runs on stream (k-1-i) mod S (the timed region's order, below)
    def sof(i, k):
        return (k - 1 - i) % S

    def step(i, k=None):
        si = sof(i, k if k is not None else S)
        prog.launch(sdescs[si][i % len(descs)], outs[si], streams[si])

    if args.settle_ms > 0:  # untimed: the GPU's clocks up to their steady state
        ts, i = time.perf_counter(), 0
        while (time.perf_counter() - ts) * 1e3 < args.settle_ms:
            step(i)
            i += 1
            if i % 64 == 0:  # keep the queue short (enqueue is faster than a batch)
                torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)

    def region(k):
        """k steps bracketed by an event pair: the start event on the first step's stream, the
        other streams wait on it after the first launch; the last step's stream joins the others
        before the end event. Returns (start event, end event, host seconds to enqueue)."""
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        first = sof(0, k)
        ts = time.perf_counter()
        e0.record(streams[first])
        for i in range(k):
            if i == 1:  # (after the first launch: its enqueue is the first thing the GPU waits for)
                for si in range(S):
                    if si != first:
                        streams[si].wait_event(e0)
            step(i, k)
        te = time.perf_counter() - ts
        last = sof(k - 1, k)
        for si in range(S):  # the last step's stream joins the others before the end event
            if si != last:
                ej = torch.cuda.Event()
                ej.record(streams[si])
                streams[last].wait_event(ej)
        e1.record(streams[last])
        return e0, e1, te

    # warmup: the timed region's own sequence (events, cross-stream waits and joins) untimed, so
    # its first-use costs land here -- the first cross-stream wait of a process stalled the next
    # launch by 130-210 us in about half of the driver-style runs (rocprof kernel traces,
    # profiles/r05_first_wait_stall.log), 7 us per step over 20 steps
    if args.warmup:
        region(args.warmup)
    torch.cuda.synchronize(dev)
    counters.zero_()

    # ---- timed region: barrier + sync on both sides, K steps, max over ranks ----
    # HIP events on the launch streams: one pair around the K back-to-back batches (a batch =
    # every launch of one ebpf_run_batch), so the per-batch time includes the dispatch gaps
    # between launches but no event packets between them. The wall clock adds one host -> GPU ->
    # host round trip (the first launch's latency and the completion signal: ~13 us measured for
    # an empty stream, tools/timing_probe.py). Step i runs on stream (K-1-i) mod S: consecutive
    # steps alternate and the last one runs on stream 0; with the last step on another stream the
    # end join waits on that stream's completion signal from stream 0's queue, which measured
    # 11 us more per run (tools/fixed_cost_ab.py "cur" vs "last0": profiles/r05_fixed_cost_ab.json)
    if use_dist:
        dist.barrier()
    K = args.steps
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0, ev1, t_enq = region(K)
    if use_dist:  # the one exchange step: per-verdict counters, RCCL / xGMI
        all_reduce(counters)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if use_dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        all_reduce(tt, dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kern_avg_ms = ev0.elapsed_time(ev1) / args.steps

    cnt = [int(c) & ((1 << 64) - 1) for c in counters.cpu().tolist()]
    total_pkts = (args.total_packets or n * world) * args.steps
    if not args.no_counters:
        assert sum(cnt[:7]) == total_pkts, (cnt, total_pkts)  # every packet: exactly one verdict
    pinned = None
    if args.total_packets and args.config == "5tuple" and not args.no_counters:
        # parity of the benched workload: the global counters of the K steps equal K times the
        # oracle's counters of the same chunks (tests/golden/config4.json), checked after timing
        gp = os.path.join(ROOT, "tests", "golden", "config4.json")
        if os.path.exists(gp):
            with open(gp) as f:
                g4 = json.load(f)
            if g4["total_packets"] == args.total_packets and g4["chunk"] == D.CHUNK:
                want = [(c * args.steps) & ((1 << 64) - 1) for c in g4["counters"]]
                assert cnt == want, ("config-4 counters differ from tests/golden/config4.json",
                                     cnt, want)
                pinned = "tests/golden/config4.json: counters == steps x fixture"
    pin_note = None
    if args.long_options:
        pin_note = "frames modified by --long-options: no fixture"
    elif not args.total_packets and not args.no_counters:
        # parity of the timed weak-scaling work at any rank count: the global counters of the K
        # steps equal the oracle's counters of the chunks every rank timed (checked after timing)
        want, src = pin_weak(PROGRAM_OF.get(args.config, args.config), mixed, fb, n, world,
                             len(batches), args.steps, cnt)
        if want is None:
            pin_note = src
        else:
            assert cnt == want, ("timed counters differ from the oracle's fixture", src, cnt, want)
            pinned = src
    mpps = total_pkts / elapsed / 1e6
    # the device's rate: the algorithmic bytes of a step over the HIP-event time per step (with
    # S > 1 streams consecutive launches overlap, so this is the time between batches, not one
    # kernel's duration), and the same bytes over the wall-clock step time that `value` uses
    achieved_gbs = algo_bytes / (kern_avg_ms * 1e-3) / 1e9
    floor_gbs = floor_bytes / (kern_avg_ms * 1e-3) / 1e9
    wall_gbs = algo_bytes * args.steps / elapsed / 1e9
    # one launch at a time, after the timed region (not part of `value`): the kernel's own
    # duration, which rocprof's per-kernel average of a --streams 1 run reports
    single_ms = kern_avg_ms
    if S > 1:
        c0 = torch.cuda.Event(enable_timing=True)
        c1 = torch.cuda.Event(enable_timing=True)
        kc = max(8, min(args.steps, 50))
        torch.cuda.synchronize(dev)
        c0.record(stream)
        for i in range(kc):
            prog.launch(sdescs[0][i % len(descs)], outs[0], stream)
        c1.record(stream)
        torch.cuda.synchronize(dev)
        single_ms = c0.elapsed_time(c1) / kc

    # PMC of the same workload (FETCH_SIZE doubled + WRITE_SIZE, MI355X guide HBM section;
    # SQ_INSTS_VALU), collected by tools/pmc.sh into the committed summary
    traffic = None
    issue = None
    suffix = (("" if mixed or fb == 64 else f"_{fb}B") + ("" if args.layout == "fixed" else f"_{args.layout}")
              + ("_generic" if args.generic else ""))
    pj = args.pmc_json or os.path.join(ROOT, "profiles", f"pmc_{args.config}{suffix}.json")
    pmc_note = None
    if os.path.exists(pj) and not args.total_packets and n == 1 << 20:
        with open(pj) as f:
            pmc = json.load(f)
        # a summary profiled on another build of the kernel does not describe this run: refuse
        # it when its kernel time differs from this run's by more than 10 % (PMC passes serialize
        # the launches: compared with one launch at a time)
        prof_us = pmc.get("kernel_avg_us_profiled")
        if not prof_us or abs(prof_us - single_ms * 1e3) > 0.10 * single_ms * 1e3:
            pmc_note = (f"{os.path.relpath(pj, ROOT)} not attached: profiled at {prof_us} us vs "
                        f"{single_ms * 1e3:.2f} us in this run")
            pmc = {}
        traffic = pmc.get("hbm_bytes_per_launch")
        valu = pmc.get("avg", {}).get("SQ_INSTS_VALU")
        if valu:
            # instruction-issue roofline: wave64 VALU instructions per second of the dominant
            # kernel vs 256 CUs x 4 SIMDs x one wave64 VALU op per 2 cycles x 2.4 GHz
            ceil = 256 * 4 * 2.4e9 / 2
            per_s = valu / (pmc["kernel_avg_us_profiled"] * 1e-6)
            issue = {"valu_wave_insts_per_launch": int(valu),
                     "valu_wave_insts_per_s": round(per_s, 1),
                     "valu_lane_ops_per_s": round(per_s * 64, 1),
                     "ceiling_wave_insts_per_s": ceil,
                     "frac": round(per_s / ceil, 4),
                     "ebpf_lane_insts_per_s": None,
                     "source": os.path.relpath(pj, ROOT)}

    kid = prog.batch_kernel(descs[0], out, local)
    kernel_name = _lib.KERNEL_NAMES[kid]
    if kid == _lib.EBPF_KERNEL_JIT_LOOP:  # (the loop program's kernel: plain or deep)
        kernel_name = prog.jit_loop_kernel() + " (compiled loop program)"
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, img, batches[0], mixed, n, mem_size, r10)

    if issue is not None:
        issue["ebpf_lane_insts_per_s"] = round(cnt[7] / (kern_avg_ms * 1e-3 * args.steps), 1)
    if rank == 0:
        line = {
            "metric": "Mpkt/s device-resident, 64B frames, fixed XDP prog; achieved HBM GB/s vs peak",
            "value": round(mpps, 2),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "strong" if args.total_packets else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded Ethernet/IPv4 frames, device-resident, pool > Infinity Cache)",
            "config": {
                "workload": desc,
                "baseline_config": cfg_idx,
                "packets_per_step_per_gpu": n,
                "global_batch": args.total_packets or n * world,
                "frame_bytes": "64/1500 mixed" if mixed else fb,
                "program_insns": len(prog),
                "mem_size": mem_size,
                "pool_batches": len(batches),
                "parallelism": f"dp{world} (packet shards, counters all-reduced over RCCL)",
                "streams": S,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                # the wall-clock view of the same launches (value's time base): GB/s and fraction
                "achieved_wall": round(wall_gbs, 2),
                "frac_wall": round(wall_gbs / HBM_PEAK_GBS, 5),
                "algo_bytes_per_launch": algo_bytes,
                # the HBM line floor of those bytes (128-byte lines touched: a 64-byte window in
                # a 1504-byte slot straddles two lines in one case of four) and its fraction;
                # the PMC traffic per launch over the same time (null without a PMC summary)
                "floor_bytes_per_launch": floor_bytes,
                "floor_bytes_per_packet": round(floor_bytes / max(n, 1), 2),
                "frac_floor": round(floor_gbs / HBM_PEAK_GBS, 5),
                "frac_traffic": (round(traffic / (kern_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                                 if traffic else None),
                # HIP-event time per step over the timed region: one event pair around the K
                # launches (each one whole batch; with counters, its last workgroup folds the
                # per-shard sums into them). With S > 1 streams the launches overlap: rocprof's
                # union of kernel busy intervals per launch (tools/rocprof_union.py) agrees with
                # this, its per-kernel average is longer
                "kernel_avg_us": round(kern_avg_ms * 1e3, 3),
                "streams": S,
                # one launch at a time (S = 1: the timed region itself); rocprof's per-kernel
                # average of a --streams 1 run
                "kernel_single_us": round(single_ms * 1e3, 3),
                "frac_single": round(algo_bytes / (single_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                "kernel": kernel_name,
            },
            "issue_roofline": issue,
            "counters": {"drop": cnt[1], "pass": cnt[2], "other": cnt[5], "faults": cnt[6],
                         "insns_retired": cnt[7]},
            "ebpf_insns_per_s": round(cnt[7] / elapsed, 1),
            # device-resident rate from the HIP-event time of the K steps (no host launch / sync)
            "value_device": round((args.total_packets or n * world) / (kern_avg_ms * 1e-3) / 1e6, 2),
            "host_enqueue_us_per_step": round(t_enq / args.steps * 1e6, 3),
            # the wall clock's fixed part: one host -> GPU -> host round trip around the K steps
            # (first launch's latency + completion signal), which value spreads over K steps
            "wall_fixed_us": round((elapsed - kern_avg_ms * 1e-3 * args.steps) * 1e6, 2),
            "pmc_note": pmc_note,
            "parity_pinned": pinned,
            "pin_note": pin_note,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


def pcap_capture(frames):
    """A classic little-endian pcap capture (pcap.to_bytes's format, ebpf_emu/pcap.py) of the rows
    of `frames` (u8[n][L]), built with numpy: 24-byte file header, then per frame a 16-byte record
    header (ts = the record index, incl_len = orig_len = L) and the frame."""
    import struct

    import numpy as np

    n, L = frames.shape
    rec = np.zeros((n, 16 + L), dtype=np.uint8)
    hdr = rec[:, :16].view(np.uint32)
    hdr[:, 0] = np.arange(n, dtype=np.uint32)
    hdr[:, 2] = L
    hdr[:, 3] = L
    rec[:, 16:] = frames
    head = np.frombuffer(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1), dtype=np.uint8)
    return np.concatenate([head, rec.reshape(-1)])


def line_floor_bytes(starts, lengths, line=128):
    """Bytes of the distinct 128-byte HBM lines that byte ranges [start, start + length) touch
    (the MI355X L2 line: a read of any byte of a line moves the line)."""
    import numpy as np

    starts = np.asarray(starts, dtype=np.int64)
    lengths = np.asarray(lengths, dtype=np.int64)
    keep = lengths > 0
    a = starts[keep] // line
    b = (starts[keep] + lengths[keep] - 1) // line
    span = b - a + 1
    idx = np.repeat(a, span) + (np.arange(int(span.sum())) - np.repeat(np.cumsum(span) - span, span))
    return int(np.unique(idx).size) * line


def host_cpus():
    """CPUs this process may use: its affinity set, capped by a cgroup v2 CPU quota (on the GPU
    box os.cpu_count() / nproc show the whole machine, while the box's share is smaller)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, img, batch0, mixed, n, mem_size, r10):
    """The C oracle ("port" of the reference semantics) on host cores over a bounded sample:
    every usable core (static contiguous partitions, std::thread-style pthreads inside
    or_run_batch), then one core."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    usable, affinity, quota = host_cpus()
    threads = args.cpu_threads or usable
    op = oracle.Program(img)
    frames = batch0["frames"].cpu().numpy()
    indexed = "offsets" in batch0  # (mixed frames, or the offsets / pcap layouts)
    if indexed:
        offs = batch0["offsets"].cpu().numpy().view(np.uint32)
        lens = batch0["lens"].cpu().numpy().view(np.uint16)
    stride = (max(64, args.frame_bytes) + 15) // 16 * 16

    def rate(nthreads, seconds):
        kw = dict(mem_size=mem_size, r10=r10, threads=nthreads,
                  xdp_md=args.config in XDP_CONFIGS)
        # chunks sized to ~0.2 s of work so the time budget is met closely
        chunk = max(4096, min(n, int((1 << 14 if mixed else 1 << 20) * nthreads / 8)))
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            lo = done % n
            hi = min(n, lo + chunk)
            if indexed:
                op.run_batch(frames, hi - lo, offsets=offs[lo:hi], lens=lens[lo:hi], **kw)
            else:
                op.run_batch(frames[lo * stride:hi * stride], hi - lo, stride=stride, **kw)
            done += hi - lo
        dt = time.perf_counter() - t0
        return done / dt / 1e6, done, dt

    v, done, dt = rate(threads, args.cpu_seconds)
    out = {"value": round(v, 3), "unit": "Mpkt/s", "cores": threads, "kind": "port",
           "sample": f"{done} packets of the same workload ({'mixed' if mixed else '64B'} frames), "
                     f"{dt:.1f} s, C oracle (oracle/ebpf_oracle.c) with {threads} threads",
           "nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpus": quota,
           "cpu_model": cpu_model()}
    if args.cpu_seconds_1core > 0:
        v1, done1, dt1 = rate(1, args.cpu_seconds_1core)
        out["value_1core"] = round(v1, 3)
        out["sample_1core"] = f"{done1} packets, {dt1:.1f} s, one thread"
    return out


if __name__ == "__main__":
    main()
