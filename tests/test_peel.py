"""Loop-invariant bound loads peeled at load time (host.cpp peel_invariant_loads).

A loop that tests its bound at the top and reloads it every iteration (an XDP program re-reading
ctx->data_end) is rewritten, for every kernel but the general interpreter, into a one-block loop
with the test at the bottom and two nops retiring the `ja` and the reload. The reference runs the
original program step by step (emu.rs:452-458), so the rewrite must leave the registers exactly as
each original step does: the tests below compare every output -- registers of faulted and
budget-stopped lanes included -- with the general interpreter (which runs the original micro-ops)
and with the oracle, over load widths, conditions (64- and 32-bit), narrow reloads that keep the
bound's high bytes, and binding and non-binding step budgets.

CPU: which shapes are peeled (the compiled loop takes the counted-loop byte passes)."""
import random

import numpy as np
import pytest

from ebpf_emu.asm import assemble

W_NAME = {1: "b", 2: "h", 4: "w", 8: "dw"}


def _src(width, op, k, hi=False, wide_body=False):
    pre = "lddw r4, 0x1234567800000000\n" if hi else ""
    body = ("mov r6, r1\nadd r6, r3\nldxb r5, [r6+0]\nadd r0, r5\n" if not wide_body else
            "mov r6, r1\nadd r6, r3\nldxb r5, [r6+0]\nmov r7, r5\nlsh r7, 3\nxor r0, r7\nadd r0, r5\n")
    return f"""
    {pre}mov r3, 0
    mov r0, 0
loop:
    ldx{W_NAME[width]} r4, [r1+{k}]
    {op} r3, r4, done
    {body}    add r3, 1
    ja loop
done:
    exit
"""


def test_peel_shapes_compile_to_counted_loops():
    """Which loops are peeled (two micro-ops more: the nops' second and the back edge), and that
    the XDP checksum reloading ctx->data_end then gets the counted loop's byte passes (v_sad_u8)
    in its xdp_md copies, as the checksum with its test at the bottom does."""
    import re

    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    def uops(img):
        p = Program(img)
        assert p.compile()
        m = re.search(r"; compiled eBPF loop program: (\d+) micro-ops", p.jit_asm(2))
        p.close()
        return int(m.group(1))

    assert uops(assemble(_src(1, "jge", 14))) == 13  # (11 instructions)
    assert uops(assemble(_src(4, "jne", 12, hi=True))) == 14  # (+ lddw)
    # not peeled: the body writes the bound's base / the bound; a jump into the loop
    assert uops(assemble(_src(1, "jge", 14).replace("add r3, 1", "add r3, 1\nadd r1, 0"))) == 12
    assert uops(assemble(_src(1, "jge", 14).replace("add r3, 1", "add r3, 1\nmov r4, 9"))) == 12
    assert uops(assemble(_src(1, "jset", 14))) == 11  # (no negated jset)
    for name, sums in (("checksum_xdp_reload", True), ("checksum_xdp", True)):
        p = Program(W.program(name))
        assert p.compile()
        for v in (5, 6):
            assert ("v_sad_u8" in p.jit_asm(v)) == sums, (name, v)
        p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 2, 4, 8])
def test_peeled_loops_vs_interpreter_and_oracle(cuda, oracle_mod, width):
    import torch

    from ebpf_emu import Program

    rng = random.Random(77 + width)
    n = 200
    stride = 128
    pk = []
    for i in range(n):
        ln = rng.choice([0, 3, 20, 64, 100, 128])
        b = bytearray(rng.getrandbits(8) for _ in range(ln))
        pk.append(bytes(b))
    buf = np.zeros(n * stride, dtype=np.uint8)
    for i, b in enumerate(pk):
        buf[i * stride:i * stride + len(b)] = np.frombuffer(b, dtype=np.uint8)
    fr = torch.from_numpy(buf).to(cuda)
    lens = torch.tensor([len(b) for b in pk], dtype=torch.int16, device=cuda)
    ops = ["jge", "jgt", "jeq", "jne", "jge32", "jgt32"]
    done = 0
    for op in ops:
        for hi in (False, True):
            if hi and width == 8:
                continue
            for wide in (False, True):
                k = rng.choice([0, 4, 12, 14, 30, 56])
                img = assemble(_src(width, op, k, hi=hi, wide_body=wide))
                prog = Program(img)
                assert prog.compile()
                for steps in (1 << 22, 700, 37):
                    kw = dict(n=n, stride=stride, lens=lens, mem_size=1024, r10=512, max_steps=steps,
                              r0=True, status=True, regs=True)
                    got = prog.run(fr, **kw)
                    gen = prog.run(fr, generic=True, **kw)
                    torch.cuda.synchronize()
                    tag = f"w{width} {op} hi={hi} wide={wide} k={k} steps={steps}"
                    for key in ("status", "r0", "regs"):
                        assert torch.equal(getattr(got, key), getattr(gen, key)), (tag, key)
                    st = got.status.cpu().numpy()
                    regs = got.regs.cpu().numpy().view(np.uint64).reshape(n, -1)
                    op_ = oracle_mod.Program(img)
                    for i in range(0, n, 7):
                        ost, oregs, _, _ = op_.run_full(pk[i], 1024, 512, steps)
                        assert st[i] == ost, (tag, i)
                        if ost == 0:  # (a stopped lane's registers: against the interpreter above)
                            assert [int(v) for v in regs[i][:11]] == oregs, (tag, i)
                    done += 1
                prog.close()
    assert done >= 30
