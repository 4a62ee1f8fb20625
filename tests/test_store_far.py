"""Store mode past byte 128: the overflow image in 64-byte blocks (jit.cpp ovf_fill / ovf_ensure).

The reference writes any image byte in place (emu.rs:354-372, mmu.rs:7-12). Round 5's compiled
store mode held image bytes [64, 128) in a per-packet overflow image and deoptimized a lane
storing past it; a payload rewrite of a 1500-byte frame ran on the general interpreter. The
overflow image now covers image bytes [64, E), E = min(mem_size rounded up to 64, 2048), kept per
64-byte block: a block is filled from the packet (zeros at or past LEN) by the lane's first store
into it, or by a load spanning it and a filled block; loads of filled blocks read the image,
others the packet. A lane deoptimizes only for a store ending past E or past the stack window's
start (r10 - k, held in registers), or a constant-address load of a block it filled.

CPU: the responder workload is store mode and proven deopt-free for mem_size <= 2048 (its
trailer store is bounded by the packet's length, jit.cpp store_mode_no_deopt len_bound); the
workspace holds (E - 64) bytes of overflow image per packet. GPU: random programs storing and
loading through pointers 0 .. ~1500 bytes in (fuzzgen.gen_far_store_program) on 1504-byte slots
and on unaligned offsets + lens batches of up to 1500-byte packets == the general interpreter ==
the oracle; the responder over crafted ICMP / IPv4 / other frames with zero lanes deoptimized (no
deopt pass at all on fixed slots)."""
import random
import struct
import zlib

import numpy as np
import pytest

MEM = 2048
R10 = 2048
STEPS = 1 << 22


def test_responder_store_mode_proof():
    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    p = Program(W.program("responder"))
    assert p.store_mode and p.store_mode_no_deopt
    assert p.compile()
    p.close()


def test_overflow_workspace_size():
    """(E - 64) bytes of overflow image per packet: 960 at mem_size 1024, 1984 at 2048 and past."""
    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    p = Program(W.program("nat"))
    fr = torch.zeros(64 * 1000, dtype=torch.uint8)
    sizes = {}
    for mem in (1024, 2048, 4096):
        b = p.make_batch(fr, n=1000, stride=64, mem_size=mem, r10=mem)
        sizes[mem] = p.workspace_bytes(b, 0)
    assert sizes[2048] - sizes[1024] == 1000 * (1984 - 960)
    assert sizes[4096] == sizes[2048]
    p.close()


def _ipv4(rng, n, proto, ihl=5, icmp_type=None):
    p = bytearray(rng.getrandbits(8) for _ in range(n))
    if n >= 14:
        p[12:14] = b"\x08\x00"
    if n >= 15:
        p[14] = 0x40 | ihl
    if n >= 24:
        p[23] = proto
    l4 = 14 + 4 * ihl
    if icmp_type is not None and n > l4:
        p[l4] = icmp_type
    return bytes(p)


def _responder_packets(rng, n):
    out = []
    for _ in range(n):
        ln = rng.choice([0, 20, 41, 42, 60, 64, 65, 100, 127, 128, 129, 200, 600, 1000, 1400,
                         1499, 1500, 1504])
        k = rng.random()
        if k < 0.35:
            out.append(_ipv4(rng, ln, 1, rng.choice([5, 5, 6, 15, 4]), rng.choice([8, 8, 0, 3])))
        elif k < 0.8:
            out.append(_ipv4(rng, ln, rng.choice([6, 17]), rng.choice([5, 5, 9])))
        else:
            out.append(bytes(rng.getrandbits(8) for _ in range(ln)))
    return out


def _fixed(pkts, stride, dev):
    import torch

    buf = np.zeros(len(pkts) * stride, dtype=np.uint8)
    for i, p in enumerate(pkts):
        q = p[:stride].ljust(stride, b"\0")
        buf[i * stride:(i + 1) * stride] = np.frombuffer(q, dtype=np.uint8)
    return torch.from_numpy(buf).to(dev)


def _batch(pkts, dev, layout):
    """-> (frames, kwargs, the packets as the kernel sees them)"""
    if layout == "fixed1504":
        pk = [p[:1504].ljust(1504, b"\0") for p in pkts]
        return _fixed(pk, 1504, dev), dict(n=len(pk), stride=1504), pk
    from test_gpu_parity import _stage

    frames, kw = _stage(pkts, dev, offsets_layout=True, misalign=3)
    return frames, kw, pkts


def _run_checked(oracle_mod, img, pkts, dev, layout, expect_no_deopt=None, tag=""):
    import torch

    from ebpf_emu import Program, _lib

    prog = Program(img)
    frames, kw, pk = _batch(pkts, dev, layout)
    b = prog.make_batch(frames, mem_size=MEM, r10=R10, **kw)
    kid = prog.batch_kernel(b)
    ws = torch.zeros(prog.workspace_bytes(b, 0), dtype=torch.uint8, device=dev)
    b = prog.make_batch(frames, mem_size=MEM, r10=R10, workspace=ws, **kw)
    out = _lib.BatchOut()
    n = len(pk)
    r0 = torch.empty(n, dtype=torch.int64, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    ws[8:12] = 0xFF
    out.r0, out.status, out.counters = r0.data_ptr(), st.data_ptr(), cnt.data_ptr()
    prog.launch(b, out, torch.cuda.current_stream())
    torch.cuda.synchronize()
    w = ws[:12].cpu().numpy().view(np.uint32)
    assert w[0] == 0, (tag, "the deopt list was left non-empty", w)
    if expect_no_deopt is not None:
        # no lane deoptimized: the pass either not launched (0xFFFFFFFF kept: a proven program on
        # a batch whose longest packet the host knows) or re-ran nothing
        assert w[2] == (0xFFFFFFFF if expect_no_deopt == "no pass" else 0), (tag, w)
    gcnt = torch.zeros(8, dtype=torch.int64, device=dev)
    gen = prog.run(frames, r0=True, status=True, generic=True, counters=gcnt, mem_size=MEM,
                   r10=R10, **kw)
    torch.cuda.synchronize()
    assert torch.equal(st, gen.status), (tag, img.hex())
    ok = st == 0
    assert torch.equal(r0[ok], gen.r0[ok]), (tag, img.hex())
    assert torch.equal(cnt, gcnt), (tag, cnt, gcnt)
    op = oracle_mod.Program(img)
    stn, r0n = st.cpu().numpy(), r0.cpu().numpy().view(np.uint64)
    for i in range(n):
        s, o0, _ = op.run_packet(pk[i], MEM, R10, STEPS)
        assert stn[i] == s, (tag, i, len(pk[i]), img.hex())
        if s == 0:
            assert int(r0n[i]) == o0, (tag, i, len(pk[i]), img.hex())
    prog.close()
    return kid, w


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed1504", "offsets_mis3"])
def test_far_store_fuzz(cuda, oracle_mod, layout):
    """Random store-mode programs through pointers up to ~1500 bytes in: the var tile loop's
    store mode (its overflow image in 64-byte blocks) + its deopt pass == the general interpreter
    == the oracle; stores at offsets 128..1500 included, the route asserted."""
    from ebpf_emu import Program, _lib
    from fuzzgen import gen_far_store_program

    rng = random.Random(zlib.crc32(b"far" + layout.encode()))
    done = 0
    for it in range(14):
        img = gen_far_store_program(rng)
        try:
            oracle_mod.Program(img)
            p = Program(img)
        except Exception:
            continue
        sm = p.store_mode
        p.close()
        if not sm:
            continue
        lens = [0, 14, 60, 64, 65, 127, 128, 200, 700, 1000, 1400, 1499, 1500]
        pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice(lens))) for _ in range(150)]
        kid, _ = _run_checked(oracle_mod, img, pkts, cuda, layout, tag=f"{layout} {it}")
        assert kid in (_lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK), (layout, it, kid)
        done += 1
    assert done >= 6, done


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["fixed1504", "offsets_mis3"])
def test_responder_vs_oracle(cuda, oracle_mod, layout):
    """The responder workload: ICMP echo replies behind IPv4 options and telemetry trailers up
    to byte 1503 written in place on the compiled store mode, no lane deoptimized and no deopt
    pass (proven); every output == the general interpreter == the oracle."""
    from ebpf_emu import _lib
    from ebpf_emu import workloads as W

    rng = random.Random(7 + len(layout))
    pkts = _responder_packets(rng, 3000)
    # (fixed slots: every packet 1504 bytes, below the stack window at 2048 - 4 -- no pass; with
    # lengths the host cannot bound LEN below mem_size = r10, so the pass runs and re-runs none)
    kid, w = _run_checked(oracle_mod, W.program("responder"), pkts, cuda, layout,
                          expect_no_deopt="no pass" if layout == "fixed1504" else "empty pass",
                          tag=layout)
    assert kid in (_lib.EBPF_KERNEL_JIT_VARL_STACK, _lib.EBPF_KERNEL_JIT_STACK)


@pytest.mark.gpu
def test_responder_full_batch_pinned(cuda):
    """bench.py --config responder --frame-bytes 1504's chunk 0 on the GPU: counters == the
    committed oracle fixture (tests/golden/bench_pins.json chunk_counters_1504)."""
    import json
    import os

    import torch

    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    with open(os.path.join(os.path.dirname(__file__), "golden", "bench_pins.json")) as f:
        pin = json.load(f)["programs"]["responder"]
    n = 1 << 20
    buf = W.frames_fixed(n, 1504, 3)
    prog = Program(W.program("responder"))
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    fr = torch.from_numpy(buf).to(cuda)
    prog.run(fr, n=n, stride=1504, mem_size=2048, r10=2048, counters=cnt)
    torch.cuda.synchronize()
    assert [int(x) for x in cnt.cpu().numpy().view(np.uint64)] == pin["chunk_counters_1504"][0]
    prog.close()
