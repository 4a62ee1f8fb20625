"""The fixed-slot kernel's occupancy variant (ebpf_tile_jit_fixed_occ, EBPF_KERNEL_JIT_FIXED_OCC).

Issue-bound programs -- a rule chain retiring hundreds of steps per packet for the same 64 bytes
of HBM -- ran on ebpf_tile_jit_fixed at 4 waves per SIMD (two window buffers per wave, 102
VGPRs), too few to hide the min-pc scheme's exec / vcc dependency chains. The variant holds one
window buffer per wave (the next tile is claimed and DMA'd when the current one is done,
gen_tile.py jit_statement_loop(single=True)) and compiles the program without the preloaded
window (only v[0:55]), so 3 workgroups of 8 waves fit a CU: 6 waves per SIMD.
Every forward program takes it (jit.cpp occ_wanted; programs of >= 96 micro-ops only until late in
round 6) when its code fits the registers (occ_regs_ok) and the batch is not xdp_md; programs of
>= 256 micro-ops its 12-wave form (ebpf_tile_jit_fixed_occw, same kernel id). The reference runs
every program through one step() (emu.rs:452-458): outputs must not change, only the kernel.

CPU: which programs get the variant's code, and that the code names only the statement's
registers. GPU: the route, and every output == the general interpreter == the oracle, including
partial last tiles and a grid capped so waves re-enter the statement (511 tiles per entry)."""
import os
import random
import re

import numpy as np
import pytest

OCC = "occ=1"
NOT_HERE = "(not this program's kernel)"


def _occ_body(text):
    """The occupancy statements' compiled code (None if the program has none there): the 8-wave
    form's (ebpf_tile_jit_fixed_occ) or, for programs of >= launch.h kOccWideUops micro-ops, the
    12-wave form's (ebpf_tile_jit_fixed_occw)."""
    for m in re.finditer(r"; JIT N=(\d+) [^\n]*occ=1[^\n]*\n", text):
        n = m.group(1)
        head = text[m.end():text.index(f".Ldone{n}:", m.end())]
        if NOT_HERE in head or "needs more registers" in head:
            continue
        if "out of line" in head:  # far mode: behind the kernel's code
            k = text.index(f".Lbody{n}:")
            return text[k:text.index("\n.Lfunc_end", k)]
        return head
    return None


def test_occ_routing():
    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    for name, want in (("acl_rules", True), ("acl", True), ("5tuple", True), ("drop", True),
                       ("nat", False), ("5tuple_stack", False)):
        p = Program(W.program(name))
        assert p.compile(), name
        assert (_occ_body(p.jit_asm(1)) is not None) == want, name
        p.close()


def test_occ_code_in_its_registers():
    """Every VGPR the variant's code names is one its statement owns (v[0:55])."""
    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    for name in ("acl_rules", "acl"):
        p = Program(W.program(name))
        p.compile()
        b = _occ_body(p.jit_asm(1))
        regs = set()
        for m in re.finditer(r"(?<![\w.])v\[(\d+):(\d+)\]|(?<![\w.])v(\d+)\b", b):
            regs |= ({int(m.group(3))} if m.group(3)
                     else set(range(int(m.group(1)), int(m.group(2)) + 1)))
        assert regs and max(regs) <= 55, (name, sorted(regs))
        assert "ds_read_b128 v[64" not in b  # (no preloaded window)
        p.close()


def test_pending_masks_in_rule_chains():
    """jit.cpp pm_assign: in the fixed-slot statements (marker pm=1, s[72:79] clobbered), a
    rule chain's lanes park in SGPR masks -- every rule's entry takes exec from its mask, no LPC
    compare re-admits lanes -- and the code names no SGPR past s79."""
    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    p = Program(W.program("acl_rules"))
    p.compile()
    b = _occ_body(p.jit_asm(1))
    # (a rule's entry: its mask -- or, its region holding only register work, the region's
    # survivors in s[72:73], jit.cpp cm_assign; its tests then one v_cmpx each)
    entries = len(re.findall(r"^s_or_saveexec_b64 (s\[7[2-9]:7[3-9]\]), \1$", b, re.M))
    entries += len(re.findall(r"^s_mov_b64 exec, s\[72:73\]$", b, re.M))
    assert entries >= 128, entries  # (one per rule, in each copy)
    assert len(re.findall(r"^v_cmpx_", b, re.M)) >= 256
    assert not re.search(r"^v_cmpx_eq_u32 vcc, \d+, v28$", b, re.M)
    sg = [int(x) for x in re.findall(r"(?<![\w.])s\[?(\d+)", b)]
    assert max(sg) <= 79, max(sg)
    p.close()


def _frames(rng, n):
    from ebpf_emu import workloads as W

    buf = W.frames_fixed(n, 64, rng.randrange(1 << 30))
    return buf


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["acl_rules", "acl"])
@pytest.mark.parametrize("n", [64, 4096 + 17, 100_000])
def test_occ_vs_oracle(cuda, oracle_mod, name, n):
    import torch

    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W

    rng = random.Random(n * 7 + len(name))
    img = W.program(name)
    buf = _frames(rng, n)
    prog = Program(img)
    fr = torch.from_numpy(buf).to(cuda)
    k = prog.batch_kernel(prog.make_batch(fr, n=n, stride=64))
    assert _lib.KERNEL_NAMES[k].startswith("ebpf_tile_jit_fixed_occ"), _lib.KERNEL_NAMES[k]
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    res = prog.run(fr, n=n, stride=64, r0=True, status=True, counters=cnt)
    torch.cuda.synchronize()
    r0, st, ocnt = oracle_mod.Program(img).run_batch(buf, n, stride=64, threads=8)
    assert np.array_equal(res.status.cpu().numpy(), st)
    assert np.array_equal(res.r0.cpu().numpy().view(np.uint64), r0)
    assert np.array_equal(cnt.cpu().numpy().view(np.uint64), ocnt)
    v = res.verdict.cpu().numpy()
    assert np.array_equal(v, np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8))
    # every register, against the general interpreter
    full = prog.run(fr, n=n, stride=64, r0=True, status=True, regs=True)
    gen = prog.run(fr, n=n, stride=64, r0=True, status=True, regs=True, generic=True)
    torch.cuda.synchronize()
    assert torch.equal(full.regs, gen.regs) and torch.equal(full.status, gen.status)
    prog.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["acl", "acl_rules"])  # (the 8- and the 12-wave form)
def test_occ_statement_reentry(cuda, oracle_mod, name):
    """A grid capped to 2 workgroups (EBPFEMU_FIXED_WGS): each wave runs > 511 tiles, so it
    re-enters the statement with its next tile's window already in flight (first = 0)."""
    import subprocess
    import sys

    code = (
        "import sys, numpy as np, torch\n"
        f"sys.path[:0] = {[os.path.join(os.path.dirname(__file__), '..', 'ebpf-emu_amd'), os.path.join(os.path.dirname(__file__), '..', 'oracle')]!r}\n"
        "import oracle\n"
        "from ebpf_emu import Program, _lib, workloads as W\n"
        "n = 16 * 600 * 64 + 5\n"
        "buf = W.frames_fixed(n, 64, 11)\n"
        f"img = W.program({name!r})\n"
        "p = Program(img)\n"
        "fr = torch.from_numpy(buf).cuda()\n"
        "assert _lib.KERNEL_NAMES[p.batch_kernel(p.make_batch(fr, n=n, stride=64))].startswith('ebpf_tile_jit_fixed_occ')\n"
        "cnt = torch.zeros(8, dtype=torch.int64, device='cuda')\n"
        "res = p.run(fr, n=n, stride=64, r0=True, status=True, counters=cnt)\n"
        "torch.cuda.synchronize()\n"
        "r0, st, oc = oracle.Program(img).run_batch(buf, n, stride=64, threads=8)\n"
        "assert np.array_equal(res.status.cpu().numpy(), st)\n"
        "assert np.array_equal(res.r0.cpu().numpy().view(np.uint64), r0)\n"
        "assert np.array_equal(cnt.cpu().numpy().view(np.uint64), oc)\n"
        "print('ok')\n")
    # (2 workgroups of 8 waves / 1 of 12: > 511 tiles per wave either way)
    env = dict(os.environ, EBPFEMU_FIXED_WGS="2" if name == "acl" else "1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr[-3000:]


@pytest.mark.gpu
def test_occ_fuzz_long_programs(cuda, oracle_mod):
    """Random forward programs of 100-900 instructions on fixed slots: those the variant takes
    == the oracle (the others take ebpf_tile_jit_fixed)."""
    from fuzzgen import gen_long_program
    from test_gpu_jit import _run, _same, _vs_oracle

    rng = random.Random(606)
    took = 0
    for it in range(6):
        img = gen_long_program(rng, rng.randrange(100, 900))
        pkts = [bytes(rng.getrandbits(8) for _ in range(64)) for _ in range(rng.choice([64, 130]))]
        from test_big_programs import _kernel

        name = _kernel(img, cuda, "fixed", pkts)
        took += name.startswith("ebpf_tile_jit_fixed_occ")
        got = _run(img, pkts, cuda, fixed_stride=64)
        ref = _run(img, pkts, cuda, fixed_stride=64, no_jit=True)
        _same(got, ref, f"occ fuzz {it}")
        _vs_oracle(oracle_mod, img, pkts, got, tag=f"occ fuzz {it}")
    assert took >= 3
