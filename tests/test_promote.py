"""Stack-slot promotion (host.cpp promote_slots, jit.cpp promo_guard / all_loads_proven): a loop
program that keeps its accumulator in an 8-byte stack slot (`ldxdw rT, [r10-8]; add rT, rD;
stxdw [r10-8], rT`, config 5 with a spilled sum: workloads.CHECKSUM_STACK) runs -- for production
batches (verdict, r0, status, counters) -- as a tier-0 loop program with the slot in a free
register, on the loop kernels' byte machinery (counted passes, the byte-sum idiom, cooperative
sums). Reference: emu.rs:341-349 / 354-372 (the slot's loads and stores), emu.rs:452-458 (steps).

CPU: which programs are promoted and that the promoted code carries the byte-sum idiom.
GPU: the production outputs of promoted batches (route EBPF_KERNEL_JIT_LOOP) against the general
interpreter and the oracle, on every var layout, with packets long enough to reach the slots
(LEN > r10 - k: those lanes deoptimize to the general interpreter) and step budgets that bind;
batches asking for the final registers keep the stack loop kernel (EBPF_KERNEL_JIT_LOOP_STACK).
r0 is compared where the packet completes: a faulted packet's r0 is not a reference output (the
reference panics), and the folded accumulator (`nop; add rS, rD; nop`) leaves it elsewhere.
"""
import random
import zlib

import numpy as np
import pytest

from fuzzgen import gen_slot_loop_program


def test_promotion_applies(product_lib):
    from ebpf_emu import Program
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble
    from test_stack_tier import STACK_SUM

    for img in (W.program("checksum_stack"), assemble(STACK_SUM)):
        p = Program(img)
        assert p.compile() and p.promoted
        a = p.jit_asm(4)
        assert "promotion guard" in a and "v_sad_u8" in a  # (the byte-sum idiom)
        p.close()
    for name in ("checksum", "5tuple_stack", "mac_swap_tx"):  # (no slot loop to promote)
        p = Program(W.program(name))
        assert p.compile() and not p.promoted, name
        p.close()
    rng = random.Random(9)
    n = 0
    for _ in range(40):
        p = Program(gen_slot_loop_program(rng))
        assert p.compile()
        n += p.promoted
        p.close()
    assert 10 <= n < 40, n


LAYOUTS = ["offsets16", "offsets_mis3", "stride_lens", "xdp_offsets"]


def _prod(img, pkts, dev, layout, generic=False, max_steps=20000, mem_size=2048, r10=1024):
    import torch

    from ebpf_emu import Program
    from test_gpu_parity import _stage
    from test_stack_tier import VAR_LAYOUTS

    lay = dict(VAR_LAYOUTS[layout])
    xdp = lay.pop("xdp", False)
    frames, kw = _stage(pkts, dev, **lay)
    prog = Program(img)
    b = prog.make_batch(frames, max_steps=max_steps, generic=generic, xdp_md=xdp, mem_size=mem_size,
                        r10=r10, **kw)
    kernel = prog.batch_kernel(b, None, dev.index or 0)
    cnt = torch.zeros(8, dtype=torch.int64, device=dev)
    res = prog.run(frames, max_steps=max_steps, r0=True, status=True, counters=cnt, generic=generic,
                   xdp_md=xdp, mem_size=mem_size, r10=r10, **kw)
    torch.cuda.synchronize()
    out = dict(status=res.status.cpu().numpy(), r0=res.r0.cpu().numpy().view(np.uint64),
               verdict=res.verdict.cpu().numpy(), counters=cnt.cpu().numpy().view(np.uint64),
               kernel=kernel)
    prog.close()
    return out, xdp


def _oracle(oracle_mod, img, pkts, xdp, mem_size, r10, max_steps):
    import struct

    op = oracle_mod.Program(img)
    st, r0 = [], []
    cnt = np.zeros(8, dtype=np.uint64)
    for p in pkts:
        im = struct.pack("<II", 8, 8 + len(p)) + p if xdp else p
        s, regs, _m, steps = op.run_full(im, mem_size, r10, max_steps)
        st.append(s)
        r0.append(regs[0] if s == 0 else 0)
        cnt[(regs[0] if regs[0] < 5 else 5) if s == 0 else 6] += 1
        cnt[7] += steps
    return np.array(st, dtype=np.uint8), np.array(r0, dtype=np.uint64), cnt


@pytest.mark.gpu
@pytest.mark.parametrize("layout", LAYOUTS)
def test_promoted_vs_oracle(cuda, oracle_mod, layout):
    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble
    from test_stack_tier import STACK_SUM

    rng = random.Random(zlib.crc32(b"promote" + layout.encode()))
    progs = [W.program("checksum_stack"), assemble(STACK_SUM)]
    progs += [gen_slot_loop_program(rng) for _ in range(14)]
    n_prom = 0
    for it, img in enumerate(progs):
        p = Program(img)
        prom = p.compile() and p.promoted
        p.close()
        # lengths around r10 - k = 1016 (r10 = 1024): the long ones deoptimize
        lens = [0, 1, 7, 60, 64, 100, 500, 1000, 1010, 1016, 1017, 1020, 1500, 2000]
        pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice(lens))) for _ in range(150)]
        for steps in ((20000, 41) if it % 3 == 0 else (20000,)):
            got, xdp = _prod(img, pkts, cuda, layout, max_steps=steps)
            if prom:
                assert got["kernel"] == _lib.EBPF_KERNEL_JIT_LOOP, (layout, it)
                n_prom += 1
            ref, _ = _prod(img, pkts, cuda, layout, generic=True, max_steps=steps)
            for key in ("status", "verdict", "counters"):
                assert np.array_equal(got[key], ref[key]), (key, layout, it, steps, img.hex())
            # r0 of a packet that faulted (ST_STEPS here) is not an output of the reference, which
            # panics there; the promoted program's folded accumulator leaves it elsewhere
            okr = got["status"] == 0
            assert np.array_equal(got["r0"][okr], ref["r0"][okr]), (layout, it, steps, img.hex())
            st, r0, cnt = _oracle(oracle_mod, img, pkts, xdp, 2048, 1024, steps)
            assert np.array_equal(got["status"], st), (layout, it, steps)
            ok = st == 0
            assert np.array_equal(got["r0"][ok], r0[ok]), (layout, it, steps)
            assert list(got["counters"]) == list(cnt), (layout, it, steps)
    assert n_prom >= 8, n_prom


@pytest.mark.gpu
def test_promoted_checksum_full_size(cuda, oracle_mod):
    """Config 5 with the sum in a stack slot at full size (the bench's batch: 1 Mi mixed frames,
    chunk 0 of the pinned pool): counters equal the pinned fixture's; with the registers asked
    for, the batch runs the stack loop kernel with the same verdicts."""
    import json
    import os

    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "golden", "bench_pins.json")) as f:
        want = json.load(f)["programs"]["checksum_stack"]["chunk_counters"][0]
    n = 1 << 20
    buf, offs, lens = W.frames_mixed(n, config_id=5)
    fr = torch.from_numpy(buf).to(cuda)
    o = torch.from_numpy(offs.view(np.int32)).to(cuda)
    ln = torch.from_numpy(lens.view(np.int16)).to(cuda)
    prog = Program(W.program("checksum_stack"))
    b = prog.make_batch(fr, n=n, offsets=o, lens=ln, mem_size=2048, r10=2048)
    assert prog.batch_kernel(b, None, 0) == _lib.EBPF_KERNEL_JIT_LOOP
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    res = prog.run(fr, n=n, offsets=o, lens=ln, mem_size=2048, r10=2048, counters=cnt)
    torch.cuda.synchronize()
    assert list(cnt.cpu().numpy().view(np.uint64)) == want
    v1 = res.verdict.cpu().numpy()
    sub = 4096
    res2 = prog.run(fr, n=sub, offsets=o, lens=ln, mem_size=2048, r10=2048, regs=True)
    torch.cuda.synchronize()
    assert np.array_equal(res2.verdict.cpu().numpy(), v1[:sub])
    prog.close()
