"""The C-ABI library: loads without a GPU, exports every symbol include/*.h declares, and its
loader (the product decoder) agrees with the oracle's decoder field for field."""
import ctypes
import glob
import os
import random
import re

import pytest

from fuzzgen import gen_program

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(ebpf_\w+)\s*\(", text))
    return sorted(names)


def test_exports_every_declared_symbol(product_lib):
    from ebpf_emu import _lib

    decl = declared_functions()
    assert len(decl) >= 12
    for name in decl:
        assert hasattr(product_lib, name), name
    assert sorted(_lib.EXPORTS) == decl
    assert b"gfx950" in product_lib.ebpf_version()


def test_loader_matches_oracle_decoder(product_lib, oracle_mod):
    from ebpf_emu import ins

    rng = random.Random(7)
    n_ok = n_rej = 0
    for it in range(1500):
        img = gen_program(rng, valid_only=(it % 3 != 0))
        try:
            ref = oracle_mod.Program(img).decoded()
            rerr = None
        except oracle_mod.OracleDecodeError as e:
            ref, rerr = None, (e.code, e.word)
        try:
            got = [(i.imm, i.imm64, i.off, int(i.src), int(i.dst), i.opcode) for i in ins.decode_image(img)]
            gerr = None
        except ins.DecodeError as e:
            got, gerr = None, (e.code, e.word)
        assert rerr == gerr, img.hex()
        if rerr is None:
            assert got == ref, img.hex()
            n_ok += 1
        else:
            n_rej += 1
    assert n_ok > 500 and n_rej > 50


def test_tier_selection(product_lib):
    from ebpf_emu.asm import assemble
    from ebpf_emu.ins import load_image

    def tier(src):
        h = load_image(assemble(src))
        t = product_lib.ebpf_prog_tier(h)
        product_lib.ebpf_prog_free(h)
        return t

    assert tier("ldxb r0, [r1+0]\nexit") == 0
    assert tier("stb [r10-1], 1\nexit") == 1
    assert tier("lock add [r10-8], r1\nexit") == 1
    assert tier("call +0\nexit") == 1


def test_forward_only_selection(product_lib):
    """The forward-jump fast path: tier 0, every jump target after the jump, <= 256 micro-ops."""
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble
    from ebpf_emu.ins import load_image

    def fwd(img):
        h = load_image(img)
        t = product_lib.ebpf_prog_forward_only(h)
        product_lib.ebpf_prog_free(h)
        return t

    assert fwd(W.program("5tuple")) == 1
    assert fwd(W.program("drop")) == 1
    assert fwd(W.program("checksum")) == 0                      # loops
    assert fwd(assemble("ja +0\nexit")) == 1                   # target = next insn
    assert fwd(assemble("ja -1\nexit")) == 0                   # jump to itself
    assert fwd(assemble("jeq r1, 0, +5\nexit")) == 1           # target past the end
    assert fwd(assemble("stb [r10-1], 1\nexit")) == 0          # tier 1
    assert fwd(assemble("mov r0, 0\n" * 4095 + "exit")) == 1   # EBPF_MAX_COMPILED_UOPS
    assert fwd(assemble("mov r0, 0\n" * 4096 + "exit")) == 0
    assert product_lib.ebpf_prog_forward_only(None) == -1


def test_invalid_arguments_fail_before_any_device_call(product_lib):
    from ebpf_emu import _lib
    from ebpf_emu.asm import assemble
    from ebpf_emu.ins import load_image

    h = load_image(assemble("mov r0, 1\nexit"))
    b = _lib.Batch()
    product_lib.ebpf_batch_init(ctypes.byref(b))
    assert (b.mem_size, b.r10, b.max_steps) == (1024, 512, 1 << 22)
    out = _lib.BatchOut()
    assert product_lib.ebpf_run_batch(h, None, ctypes.byref(out), None) == _lib.EBPF_EINVAL
    # no packet layout (stride 0, no offsets / lens)
    assert product_lib.ebpf_run_batch(h, ctypes.byref(b), ctypes.byref(out), None) == _lib.EBPF_EINVAL
    b.stride = 64  # (n = 0: a valid batch returns before touching a device)
    assert product_lib.ebpf_run_batch(h, ctypes.byref(b), ctypes.byref(out), None) == _lib.EBPF_OK
    b.mem_size = 12  # any image length is valid (Mmu.memory is a Vec<u8>, mmu.rs:2-4)
    assert product_lib.ebpf_run_batch(h, ctypes.byref(b), ctypes.byref(out), None) == _lib.EBPF_OK
    b.mem_size = (1 << 24) + 1
    assert product_lib.ebpf_run_batch(h, ctypes.byref(b), ctypes.byref(out), None) == _lib.EBPF_EINVAL
    b.mem_size = 1024
    b.init_fp_len = 65  # deeper than EBPF_MAX_CALL_DEPTH
    b.init_fp = 8
    assert product_lib.ebpf_run_batch(h, ctypes.byref(b), ctypes.byref(out), None) == _lib.EBPF_EINVAL
    b.init_fp_len = 1
    b.init_fp = None  # a depth without a stack
    assert product_lib.ebpf_run_batch(h, ctypes.byref(b), ctypes.byref(out), None) == _lib.EBPF_EINVAL
    b.init_fp_len = 0
    b.max_steps = 0
    assert product_lib.ebpf_run_batch(h, ctypes.byref(b), ctypes.byref(out), None) == _lib.EBPF_EINVAL
    product_lib.ebpf_prog_free(h)
    assert product_lib.ebpf_strerror(_lib.EBPF_ELEN) == b"invalid hex format for u64"


def test_load_hex_matches_reference_parser(product_lib):
    from ebpf_emu import _lib

    h = ctypes.c_void_p()
    bad = ctypes.c_size_t()
    assert product_lib.ebpf_prog_load_hex(b"  b7 00 00 00 2a 00 00 00  95 00 00 00 00 00 00 00 \n",
                                          ctypes.byref(h), ctypes.byref(bad)) == 0
    assert product_lib.ebpf_prog_len(h) == 2
    product_lib.ebpf_prog_free(h)
    assert product_lib.ebpf_prog_load_hex(b"b7 00 17", ctypes.byref(h), ctypes.byref(bad)) == _lib.EBPF_ELEN
    assert product_lib.ebpf_prog_load_hex(b"zz00000000000000", ctypes.byref(h), ctypes.byref(bad)) == _lib.EBPF_EHEX
