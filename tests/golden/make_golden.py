"""Generates the golden fixtures in this directory (committed; re-run only on purpose).

The Rust reference cannot run here, so expected outputs come from the C oracle, and every
fuzz vector is cross-checked against the independent Python restatement before it is written.
  fuzz_vectors.json : 160 random programs x up to 8 packets -> status, r0, regs, CRC32(memory)
  workloads.json    : BASELINE configs 2/3/5 at full size (1,048,576 packets) -> counters,
                      CRC32 of the verdict array, first 256 verdicts
  config4.json      : BASELINE config 4, the 5-tuple over a 100,000,000-packet global batch of
                      seeded 1 Mi-packet chunks (chunk k: ebpf_emu.dist.chunk_frames(k, size), the
                      one definition bench.py --total-packets also builds its shards with) ->
                      per-chunk counters and verdict CRC32s, and the global counters
  bench_pins.json   : bench.py's weak-scaling pools at any rank count -> per-chunk counters of
                      every 1 Mi-packet chunk a pool can hold, for each bench program (so that the
                      default bench line pins its timed counters at N = 1..8)
Usage: python tests/golden/make_golden.py [config4 | bench_pins | bench_pins_add NAME... |
       bench_pins_add_1504]
"""
import json
import os
import random
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ebpf-emu_amd"), os.path.dirname(HERE)]

import numpy as np  # noqa: E402

import oracle  # noqa: E402
import pyref  # noqa: E402
from ebpf_emu import workloads as W  # noqa: E402
from fuzzgen import gen_packet, gen_program  # noqa: E402

MAX_STEPS = 2000


def fuzz_vectors():
    rng = random.Random(0xC0FFEE)
    out = []
    while len(out) < 160:
        img = gen_program(rng)
        try:
            op = oracle.Program(img)
        except oracle.OracleDecodeError:
            continue
        pkts = [gen_packet(rng) for _ in range(rng.randrange(1, 9))]
        exp = []
        for p in pkts:
            st, regs, mem, steps = op.run_full(p, 1024, 512, MAX_STEPS)
            pst, pregs, pmem, psteps = pyref.run_full(img, p, 1024, 512, MAX_STEPS)
            assert (st, steps) == (pst, psteps) and (st != 0 or (regs, mem) == (pregs, pmem))
            e = {"status": st, "steps": steps}
            if st == 0:
                e.update(r0=f"{regs[0]:x}", regs=[f"{r:x}" for r in regs], mem_crc32=zlib.crc32(mem))
            exp.append(e)
        out.append({"prog": img.hex(), "pkts": [p.hex() for p in pkts], "expect": exp})
    return {"generator": "tests/fuzzgen.py seed 0xC0FFEE", "mem_size": 1024, "r10": 512,
            "max_steps": MAX_STEPS, "vectors": out}


def workloads():
    n = 1 << 20
    res = {}
    for name, cid, layout in (("drop", 2, "fixed"), ("5tuple", 3, "fixed"), ("checksum", 5, "mixed")):
        p = oracle.Program(W.program(name))
        if layout == "fixed":
            buf = W.frames_fixed(n, 64, cid)
            r0, st, cnt = p.run_batch(buf, n, stride=64, threads=os.cpu_count())
            mem, r10 = 1024, 512
        else:
            buf, offs, lens = W.frames_mixed(n, config_id=cid)
            mem, r10 = 2048, 2048
            r0, st, cnt = p.run_batch(buf, n, offsets=offs, lens=lens, mem_size=mem, r10=r10,
                                      threads=os.cpu_count())
        verdict = np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8)
        res[name] = {"config_id": cid, "layout": layout, "n": n, "mem_size": mem, "r10": r10,
                     "program": W.program(name).hex(), "counters": [int(c) for c in cnt],
                     "verdict_crc32": zlib.crc32(verdict.tobytes()),
                     "verdict_head": verdict[:256].tolist()}
        print(name, res[name]["counters"])
    return res


def _config4_chunk(args):
    from ebpf_emu import dist as D

    k, size = args
    p = oracle.Program(W.program("5tuple"))
    buf = D.chunk_frames(k, size)
    r0, st, cnt = p.run_batch(buf, size, stride=64, threads=1)
    verdict = np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8)
    return [int(c) for c in cnt], zlib.crc32(verdict.tobytes())


def config4(total=100_000_000):
    from multiprocessing import Pool

    from ebpf_emu import dist as D

    chunk = D.CHUNK
    sizes = D.chunk_sizes(total, chunk)
    with Pool(max(1, min(8, os.cpu_count() or 1) - 1)) as pool:
        per = pool.map(_config4_chunk, list(enumerate(sizes)))
    tot = [sum(c[i] for c, _ in per) for i in range(8)]
    assert sum(tot[:7]) == total
    return {"program": W.program("5tuple").hex(), "total_packets": total, "chunk": chunk,
            "seed": "chunk k: ebpf_emu.dist.chunk_frames(k, size) = workloads.frames_fixed(size, "
                    "64, config_id=dist.chunk_seed(k) = 3 + 100 * k)",
            "mem_size": 1024, "r10": 512, "chunk_sizes": sizes,
            "chunk_counters": [c for c, _ in per], "chunk_verdict_crc32": [v for _, v in per],
            "counters": tot}


# bench.py's weak-scaling pool: rank r of W, pool batch k -> chunk k*W + r (bench.chunk_id), so
# the chunks of any rank count are 0 .. B*W-1. 64-byte chunks: dist.chunk_frames(c) (seed 3 + 100c,
# the config-4 chunks); mixed chunks: workloads.frames_mixed(1Mi, config_id=5 + 100c).
PIN_CHUNKS_64 = 128  # 16 pool batches x 8 ranks
PIN_CHUNKS_MIXED = 16  # 2 pool batches x 8 ranks (a 1 Mi mixed batch is ~840 MB: one per rank)
PIN_PROGRAMS_64 = ("5tuple", "drop", "5tuple_stack", "mac_swap_tx", "acl", "5tuple_xdp",
                   "5tuple_call", "nat", "acl_rules", "responder")
PIN_PROGRAMS_MIXED = ("checksum", "checksum_stack", "checksum_xdp", "checksum_xdp_reload")
XDP_PROGRAMS = ("5tuple_xdp", "checksum_xdp", "checksum_xdp_reload")
# 1504-byte slots (bench.py --frame-bytes 1504: rank r's pool is copies of chunk r,
# workloads.frames_fixed(1Mi, 1504, config_id=3 + 100r), mem_size = r10 = 2048)
PIN_CHUNKS_1504 = 8
PIN_PROGRAMS_1504 = ("responder",)


def _pin_chunk(args):
    from ebpf_emu import dist as D

    kind, c = args
    out = {}
    if kind == "64":
        buf = D.chunk_frames(c, D.CHUNK)
        for name in PIN_PROGRAMS_64:
            p = oracle.Program(W.program(name))
            _, _, cnt = p.run_batch(buf, D.CHUNK, stride=64, mem_size=1024, r10=512, threads=1,
                                    xdp_md=name == "5tuple_xdp")
            out[name] = [int(x) for x in cnt]
    else:
        buf, offs, lens = W.frames_mixed(D.CHUNK, config_id=5 + 100 * c)
        for name in PIN_PROGRAMS_MIXED:
            p = oracle.Program(W.program(name))
            _, _, cnt = p.run_batch(buf, D.CHUNK, offsets=offs, lens=lens, mem_size=2048,
                                    r10=2048, threads=1, xdp_md=name in XDP_PROGRAMS)
            out[name] = [int(x) for x in cnt]
    return kind, c, out


def _pin_chunk_1504(c):
    buf = W.frames_fixed(1 << 20, 1504, 3 + 100 * c)
    out = {}
    for name in PIN_PROGRAMS_1504:
        p = oracle.Program(W.program(name))
        _, _, cnt = p.run_batch(buf, 1 << 20, stride=1504, mem_size=2048, r10=2048, threads=1)
        out[name] = [int(x) for x in cnt]
    return c, out


def bench_pins_add_1504():
    """Adds the 1504-byte chunks' counters (chunk_counters_1504) of PIN_PROGRAMS_1504."""
    from multiprocessing import Pool

    path = os.path.join(HERE, "bench_pins.json")
    with open(path) as f:
        pins = json.load(f)
    with Pool(4) as pool:  # (a 1504-byte chunk is 1.5 GB)
        res = sorted(pool.map(_pin_chunk_1504, range(PIN_CHUNKS_1504)))
    for name in PIN_PROGRAMS_1504:
        e = pins["programs"][name]
        e["chunk_counters_1504"] = [o[name] for _, o in res]
        e["frames_1504"] = "workloads.frames_fixed(1Mi, 1504, config_id=3 + 100*r), mem_size = r10 = 2048"
        for cnt in e["chunk_counters_1504"]:
            assert sum(cnt[:7]) == 1 << 20
    with open(path, "w") as f:
        json.dump(pins, f, indent=0)


def bench_pins_add(names):
    """Adds programs' chunk counters to the committed bench_pins.json (same chunks): names from
    PIN_PROGRAMS_MIXED get the mixed chunks, the rest the 64-byte chunks."""
    from multiprocessing import Pool

    global PIN_PROGRAMS_64, PIN_PROGRAMS_MIXED
    path = os.path.join(HERE, "bench_pins.json")
    with open(path) as f:
        pins = json.load(f)
    mixed_names = tuple(n for n in names if n in PIN_PROGRAMS_MIXED)
    PIN_PROGRAMS_64 = tuple(n for n in names if n not in PIN_PROGRAMS_MIXED)
    PIN_PROGRAMS_MIXED = mixed_names
    jobs = ([("64", c) for c in range(PIN_CHUNKS_64)] if PIN_PROGRAMS_64 else []) + \
        ([("mixed", c) for c in range(PIN_CHUNKS_MIXED)] if mixed_names else [])
    with Pool(max(1, min(8, os.cpu_count() or 1) - 1)) as pool:
        res = pool.map(_pin_chunk, jobs)
    for name in names:
        mixed = name in mixed_names
        rows = sorted((c, o[name]) for kind, c, o in res if (kind == "mixed") == mixed)
        pins["programs"][name] = {"frames": "mixed" if mixed else "fixed64",
                                  "xdp_md": name in XDP_PROGRAMS,
                                  "program": W.program(name).hex(),
                                  "mem_size": 2048 if mixed else 1024,
                                  "r10": 2048 if mixed else 512,
                                  "chunk_counters": [cnt for _, cnt in rows]}
    with open(path, "w") as f:
        json.dump(pins, f, indent=0)


def bench_pins():
    from multiprocessing import Pool

    from ebpf_emu import dist as D

    jobs = [("64", c) for c in range(PIN_CHUNKS_64)] + [("mixed", c) for c in range(PIN_CHUNKS_MIXED)]
    with Pool(max(1, min(8, os.cpu_count() or 1) - 1)) as pool:
        res = pool.map(_pin_chunk, jobs)
    progs = {}
    for name in PIN_PROGRAMS_64 + PIN_PROGRAMS_MIXED:
        mixed = name in PIN_PROGRAMS_MIXED
        rows = sorted((c, o[name]) for kind, c, o in res if (kind == "mixed") == mixed)
        for _, cnt in rows:
            assert sum(cnt[:7]) == D.CHUNK
        progs[name] = {"frames": "mixed" if mixed else "fixed64",
                       "xdp_md": name in XDP_PROGRAMS,
                       "program": W.program(name).hex(),
                       "mem_size": 2048 if mixed else 1024, "r10": 2048 if mixed else 512,
                       "chunk_counters": [cnt for _, cnt in rows]}
    return {"chunk": D.CHUNK,
            "chunk_of": "rank r of W, pool batch k -> chunk k*W + r",
            "seed_fixed64": "dist.chunk_frames(c, 1Mi) = workloads.frames_fixed(1Mi, 64, "
                            "config_id=3 + 100*c)",
            "seed_mixed": "workloads.frames_mixed(1Mi, config_id=5 + 100*c)",
            "programs": progs}


if __name__ == "__main__":
    if sys.argv[1:2] == ["bench_pins_add"]:
        bench_pins_add(sys.argv[2:])
        sys.exit(0)
    if sys.argv[1:] == ["bench_pins_add_1504"]:
        bench_pins_add_1504()
        sys.exit(0)
    if sys.argv[1:] == ["bench_pins"]:
        with open(os.path.join(HERE, "bench_pins.json"), "w") as f:
            json.dump(bench_pins(), f, indent=0)
        sys.exit(0)
    if sys.argv[1:] == ["config4"]:
        with open(os.path.join(HERE, "config4.json"), "w") as f:
            json.dump(config4(), f, indent=0)
        sys.exit(0)
    with open(os.path.join(HERE, "fuzz_vectors.json"), "w") as f:
        json.dump(fuzz_vectors(), f, indent=0)
    with open(os.path.join(HERE, "workloads.json"), "w") as f:
        json.dump(workloads(), f, indent=1)
