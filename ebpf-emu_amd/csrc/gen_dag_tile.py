#!/usr/bin/env python3
"""Generates dag_tile.inc: the self-contained gfx950 interpreter of one tile (64 packets, one per
lane) for the forward-only fast path (dag_tile_kernel in interp.hip), as ONE inline-asm statement.

It does everything between the header-window DMA and the per-packet outputs:
  * the register file r0..r10 (main.rs:28-31 layout, or the caller's init_regs) in VGPRs;
  * the lowest-parked-pc loop over the micro-ops (uop.h DUop, asm half), dispatched with
    s_setpc into fixed 128-byte handler slots (dag_asm.h ids), exec narrowed to the lanes parked
    at the pc, results committed under that exec;
  * every micro-op kind of a tier-0 program: the ALU (incl. MUL, DIV/MOD by a bit-serial divider,
    NEG, the reference's ARSH with its overflow fault), END, the canonical jumps, LDX with the
    mmu.rs bounds checks (per-lane faults), reads inside the LDS header window and past it
    (global loads of only the dwords that hold packet bytes), static faults;
  * at exit: r0 out, and the whole register file to regs_out when the caller asked for it.
There is no register file in LDS, so the LDS left per wave is the header window.

Operands (interp.hip dag_tile_asm): live "+s" (pc set), lpc/nst/st "+v" (lane pc, retired steps,
status), r0l/r0h "=&v"; prog, mem, r10l, r10h, initp, rflag "s"; win, swz, len, base, raddr,
vok "v". Fixed (clobbered) registers are the maps SG/VG below. Only SALU/VALU/DS/SMEM, VGPR index
mode and plain global loads/stores on VGPR addresses: no readlane, DPP, trans, SDWA, M0 or
VALU-written SGPRs feeding VMEM, so no gfx950 software wait states are needed inside.

  python3 gen_dag_tile.py > dag_tile.inc
"""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
IDS = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (H_\w+) (\d+)",
                                                      open(os.path.join(HERE, "dag_asm.h")).read())}
SLOT = 128
VB = 16  # first VGPR of the fixed block (the register file); see interp.hip's clobber list

# status codes (include/ebpf_emu.h)
ST_MEM, ST_MEM_UB, ST_INSN, ST_ARITH = 1, 2, 3, 4

M = {
    # DUop asm half, dword i in s[64 + i] (uop.h)
    "HOFF": "s64", "DST2": "s65", "SRC2": "s66", "NPC": "s67", "X": "s68", "A0": "s69",
    "KML": "s70", "KMH": "s71", "NBIT": "s[72:73]", "TBIT": "s[74:75]",
    "IMM": "s[76:77]", "IMML": "s76", "IMMH": "s77", "WID": "s78", "END": "s79",
    "W0": "s80", "W1": "s81", "W2": "s82", "W3": "s83", "W4": "s84", "W5": "s85",
    "SLOTB": "s[88:89]", "SLOTBL": "s88", "SLOTBH": "s89", "EXEC0": "s[90:91]",
    "T0": "s[92:93]", "T1": "s[94:95]", "P": "s96", "T2": "s97", "JT": "s[98:99]", "JTL": "s98",
    "JTH": "s99", "T3": "s62", "MEMW": "s63", "T4": "s[56:57]", "T5": "s[58:59]", "MODE": "s60",
    "CNT": "s61", "T7": "s[54:55]", "T8": "s[52:53]",
    # VGPRs
    "RF0": f"v{VB}", "RF1": f"v{VB + 1}",
    "A": f"v[{VB + 22}:{VB + 23}]", "AL": f"v{VB + 22}", "AH": f"v{VB + 23}",
    "S": f"v[{VB + 24}:{VB + 25}]", "SL": f"v{VB + 24}", "SH": f"v{VB + 25}",
    "R": f"v[{VB + 26}:{VB + 27}]", "RL": f"v{VB + 26}", "RH": f"v{VB + 27}",
}
for i in range(20):
    M[f"t{i}"] = f"v{VB + 28 + i}"
for i in range(0, 20, 2):
    M[f"T{i}{i + 1}"] = f"v[{VB + 28 + i}:{VB + 29 + i}]"
M.update({"WD0": M["t13"], "WD1": M["t14"], "WD2": M["t15"], "SHF": M["t16"], "LENM": M["t17"]})
NVGPR = 48  # v[VB : VB + 48]
SGPRS = list(range(52, 64)) + list(range(64, 100))


def F(text):
    """Substitute {NAME} register names (the asm's own %[..] operands and %= are untouched)."""
    return re.sub(r"\{(\w+)\}", lambda m: M[m.group(1)], text)


READ_A = "s_set_gpr_idx_on {DST2}, gpr_idx(SRC0)\nv_mov_b32 {AL}, {RF0}\nv_mov_b32 {AH}, {RF1}\ns_set_gpr_idx_off"
READ_S = "s_set_gpr_idx_on {SRC2}, gpr_idx(SRC0)\nv_mov_b32 {SL}, {RF0}\nv_mov_b32 {SH}, {RF1}\ns_set_gpr_idx_off"


def WRITE(lo, hi):
    return f"s_set_gpr_idx_on {{DST2}}, gpr_idx(DST)\nv_mov_b32 {{RF0}}, {lo}\nv_mov_b32 {{RF1}}, {hi}\ns_set_gpr_idx_off"


TAIL_N = """v_mov_b32 %[lpc], {NPC}
v_add_u32 %[nst], 1, %[nst]
s_or_b64 %[live], %[live], {NBIT}
s_branch .Lloop%="""
TAIL_W = WRITE("{RL}", "{RH}") + "\n" + TAIL_N
TAIL_W32 = WRITE("{RL}", "0") + "\n" + TAIL_N
JTAIL = """v_mov_b32 {t0}, {X}
v_mov_b32 {t1}, {NPC}
v_cndmask_b32 %[lpc], {t1}, {t0}, vcc
v_add_u32 %[nst], 1, %[nst]
s_cmp_lg_u64 vcc, 0
s_cselect_b64 {T0}, {TBIT}, 0
s_andn2_b64 {T1}, exec, vcc
s_cselect_b64 {T1}, {NBIT}, 0
s_or_b64 %[live], %[live], {T0}
s_or_b64 %[live], %[live], {T1}
s_branch .Lloop%="""
WAIT = "s_waitcnt lgkmcnt(0)"


def fault_split(tag, status):
    """vcc = faulting lanes among the active ones: they stop with `status`; exec continues
    with the others (back to the loop when there are none)."""
    return f"""s_mov_b64 {{T4}}, exec
s_and_b64 exec, {{T4}}, vcc
s_cbranch_scc0 .Lnf_{tag}%=
v_mov_b32 %[st], {status}
v_mov_b32 %[lpc], -1
.Lnf_{tag}%=:
s_andn2_b64 exec, {{T4}}, vcc
s_cbranch_scc0 .Lloop%="""


def alu64(op, reg):
    if reg:
        return f"{READ_A}\n{READ_S}\n{op} {{RL}}, {{SL}}, {{AL}}\n{op} {{RH}}, {{SH}}, {{AH}}\n{TAIL_W}"
    return f"{READ_A}\n{op} {{RL}}, {{IMML}}, {{AL}}\n{op} {{RH}}, {{IMMH}}, {{AH}}\n{TAIL_W}"


def alu32(body, reg=False, a=True):
    pre = (READ_A + "\n" if a else "") + (READ_S + "\n" if reg else "")
    return f"{pre}{body}\n{TAIL_W32}"


def jump(cmp, reg, pre=""):
    return f"{READ_A}\n" + (READ_S + "\n" if reg else "") + f"{pre}{cmp}\n{JTAIL}"


def mul64(reg):
    bl, bh = ("{SL}", "{SH}") if reg else ("{IMML}", "{IMMH}")
    pre = READ_A + "\n" + (READ_S + "\n" if reg else "")
    return pre + f"""v_mul_lo_u32 {{RL}}, {{AL}}, {bl}
v_mul_hi_u32 {{t0}}, {{AL}}, {bl}
v_mul_lo_u32 {{t1}}, {{AL}}, {bh}
v_mul_lo_u32 {{t2}}, {{AH}}, {bl}
v_add3_u32 {{RH}}, {{t0}}, {{t1}}, {{t2}}
{TAIL_W}"""


def divmod_setup(mod, w64, reg):
    """Dividend -> T45, divisor -> T67, original dividend -> T1011 (the result of a division by
    zero for MOD); MODE = 1 for MOD. 32-bit forms: zero-extended low words (Q6)."""
    bl, bh = ("{SL}", "{SH}") if reg else ("{IMML}", "{IMMH}")
    pre = READ_A + "\n" + (READ_S + "\n" if reg else "")
    ah = "{AH}" if w64 else "0"
    bh = bh if w64 else "0"
    return pre + f"""v_mov_b32 {{t4}}, {{AL}}
v_mov_b32 {{t5}}, {ah}
v_mov_b32 {{t6}}, {bl}
v_mov_b32 {{t7}}, {bh}
v_mov_b32 {{t10}}, {{AL}}
v_mov_b32 {{t11}}, {ah}
s_mov_b32 {{MODE}}, {1 if mod else 0}
s_branch .Ldivmod%="""


def arsh64(reg):
    sh = "{SL}" if reg else "{IMML}"
    pre = READ_A + "\n" + (READ_S + "\n" if reg else "")
    tag = "arsh64r" if reg else "arsh64i"
    return pre + f"""v_lshrrev_b64 {{T01}}, {sh}, {{A}}
v_sub_u32_e64 {{t2}}, 64, {sh}
v_lshlrev_b64 {{T23}}, {{t2}}, {{A}}
v_or_b32 {{t0}}, {{t0}}, {{t2}}
v_or_b32 {{t1}}, {{t1}}, {{t3}}
v_sub_co_u32_e64 {{t4}}, {{T5}}, 0, {{t0}}
v_subb_co_u32_e64 {{t5}}, {{T5}}, 0, {{t1}}, {{T5}}
v_cmp_gt_i32 vcc, 0, {{AH}}
v_cndmask_b32 {{RL}}, {{t0}}, {{t4}}, vcc
v_cndmask_b32 {{RH}}, {{t1}}, {{t5}}, vcc
v_cmp_eq_u32_e64 {{T0}}, 0, {{t0}}
s_mov_b32 {{T3}}, 0x80000000
v_cmp_eq_u32_e64 {{T1}}, {{T3}}, {{t1}}
s_and_b64 {{T0}}, {{T0}}, {{T1}}
s_and_b64 vcc, vcc, {{T0}}
{fault_split(tag, ST_ARITH)}
{TAIL_W}"""


def arsh32(reg):
    sh = "{SL}" if reg else "{IMML}"
    pre = READ_A + "\n" + (READ_S + "\n" if reg else "")
    return pre + f"""v_alignbit_b32 {{t0}}, {{AL}}, {{AL}}, {sh}
v_sub_u32 {{t1}}, 0, {{t0}}
v_cmp_gt_i32 vcc, 0, {{AL}}
v_cndmask_b32 {{RL}}, {{t0}}, {{t1}}, vcc
{TAIL_W32}"""


H = {
    "H_SLOW": f"v_mov_b32 %[st], {ST_INSN}\nv_mov_b32 %[lpc], -1\ns_branch .Lloop%=",
    "H_EXIT": "v_mov_b32 %[lpc], -1\nv_add_u32 %[nst], 1, %[nst]\ns_branch .Lloop%=",
    "H_FAULT": "v_mov_b32 %[st], {IMML}\nv_mov_b32 %[lpc], -1\ns_branch .Lloop%=",
    "H_MOV64_IMM": WRITE("{IMML}", "{IMMH}") + "\n" + TAIL_N,
    "H_MOV64_REG": f"{READ_S}\n" + WRITE("{SL}", "{SH}") + "\n" + TAIL_N,
    "H_ADD64_IMM": f"{READ_A}\nv_lshl_add_u64 {{R}}, {{A}}, 0, {{IMM}}\n{TAIL_W}",
    "H_ADD64_REG": f"{READ_A}\n{READ_S}\nv_lshl_add_u64 {{R}}, {{A}}, 0, {{S}}\n{TAIL_W}",
    "H_SUB64_REG": f"{READ_A}\n{READ_S}\nv_sub_co_u32 {{RL}}, vcc, {{AL}}, {{SL}}\nv_subb_co_u32 {{RH}}, vcc, {{AH}}, {{SH}}, vcc\n{TAIL_W}",
    "H_AND64_IMM": alu64("v_and_b32", False), "H_AND64_REG": alu64("v_and_b32", True),
    "H_OR64_IMM": alu64("v_or_b32", False), "H_OR64_REG": alu64("v_or_b32", True),
    "H_XOR64_IMM": alu64("v_xor_b32", False), "H_XOR64_REG": alu64("v_xor_b32", True),
    # the hardware uses bits [5:0] / [4:0] of the shift count: the reference's masks (Q20)
    "H_LSH64_IMM": f"{READ_A}\nv_lshlrev_b64 {{R}}, {{IMML}}, {{A}}\n{TAIL_W}",
    "H_LSH64_REG": f"{READ_A}\n{READ_S}\nv_lshlrev_b64 {{R}}, {{SL}}, {{A}}\n{TAIL_W}",
    "H_RSH64_IMM": f"{READ_A}\nv_lshrrev_b64 {{R}}, {{IMML}}, {{A}}\n{TAIL_W}",
    "H_RSH64_REG": f"{READ_A}\n{READ_S}\nv_lshrrev_b64 {{R}}, {{SL}}, {{A}}\n{TAIL_W}",
    "H_MOV32_IMM": WRITE("{IMML}", "0") + "\n" + TAIL_N,
    "H_MOV32_REG": f"{READ_S}\n" + WRITE("{SL}", "0") + "\n" + TAIL_N,
    "H_ADD32_IMM": alu32("v_add_u32 {RL}, {IMML}, {AL}"),
    "H_ADD32_REG": alu32("v_add_u32 {RL}, {SL}, {AL}", reg=True),
    "H_SUB32_REG": alu32("v_sub_u32 {RL}, {AL}, {SL}", reg=True),
    "H_AND32_IMM": alu32("v_and_b32 {RL}, {IMML}, {AL}"),
    "H_AND32_REG": alu32("v_and_b32 {RL}, {SL}, {AL}", reg=True),
    "H_OR32_IMM": alu32("v_or_b32 {RL}, {IMML}, {AL}"),
    "H_OR32_REG": alu32("v_or_b32 {RL}, {SL}, {AL}", reg=True),
    "H_XOR32_IMM": alu32("v_xor_b32 {RL}, {IMML}, {AL}"),
    "H_XOR32_REG": alu32("v_xor_b32 {RL}, {SL}, {AL}", reg=True),
    "H_LSH32_IMM": alu32("v_lshlrev_b32 {RL}, {IMML}, {AL}"),
    "H_LSH32_REG": alu32("v_lshlrev_b32 {RL}, {SL}, {AL}", reg=True),
    "H_RSH32_IMM": alu32("v_lshrrev_b32 {RL}, {IMML}, {AL}"),
    "H_RSH32_REG": alu32("v_lshrrev_b32 {RL}, {SL}, {AL}", reg=True),
    "H_ZX16": alu32("v_and_b32 {RL}, 0xffff, {AL}"),
    "H_ZX32": alu32("v_mov_b32 {RL}, {AL}"),
    "H_NOP": TAIL_N,
    # v_perm_b32 selector bytes: 0..3 pick bytes of src1, 0x0c gives 0x00
    "H_BSWAP16": alu32("s_mov_b32 {T3}, 0x0c0c0001\nv_perm_b32 {RL}, {AL}, {AL}, {T3}"),
    "H_BSWAP32": alu32("s_mov_b32 {T3}, 0x00010203\nv_perm_b32 {RL}, {AL}, {AL}, {T3}"),
    "H_BSWAP64": f"""{READ_A}
s_mov_b32 {{T3}}, 0x00010203
v_perm_b32 {{RL}}, {{AH}}, {{AH}}, {{T3}}
v_perm_b32 {{RH}}, {{AL}}, {{AL}}, {{T3}}
{TAIL_W}""",
    "H_MUL64_IMM": mul64(False), "H_MUL64_REG": mul64(True),
    "H_MUL32_IMM": alu32("v_mul_lo_u32 {RL}, {AL}, {IMML}"),
    "H_MUL32_REG": alu32("v_mul_lo_u32 {RL}, {AL}, {SL}", reg=True),
    "H_NEG64": f"{READ_A}\nv_sub_co_u32 {{RL}}, vcc, 0, {{AL}}\nv_subb_co_u32 {{RH}}, vcc, 0, {{AH}}, vcc\n{TAIL_W}",
    "H_NEG32": alu32("v_sub_u32 {RL}, 0, {AL}"),
    "H_ARSH64_IMM": arsh64(False), "H_ARSH64_REG": arsh64(True),
    "H_ARSH32_IMM": arsh32(False), "H_ARSH32_REG": arsh32(True),
    "H_DIV64_IMM": divmod_setup(False, True, False), "H_DIV64_REG": divmod_setup(False, True, True),
    "H_MOD64_IMM": divmod_setup(True, True, False), "H_MOD64_REG": divmod_setup(True, True, True),
    "H_DIV32_IMM": divmod_setup(False, False, False), "H_DIV32_REG": divmod_setup(False, False, True),
    "H_MOD32_IMM": divmod_setup(True, False, False), "H_MOD32_REG": divmod_setup(True, False, True),
    "H_JA": "v_mov_b32 %[lpc], {X}\nv_add_u32 %[nst], 1, %[nst]\ns_or_b64 %[live], %[live], {TBIT}\ns_branch .Lloop%=",
    # jumps: vcc = condition over the active lanes; x / npc, tbit / nbit already canonical
    "H_JEQ_IMM": jump("v_cmp_eq_u64 vcc, {IMM}, {A}", False),
    "H_JEQ_REG": jump("v_cmp_eq_u64 vcc, {S}, {A}", True),
    "H_JGT_IMM": jump("v_cmp_lt_i64 vcc, {IMM}, {A}", False),   # k < A
    "H_JGT_REG": jump("v_cmp_lt_i64 vcc, {S}, {A}", True),
    "H_JLT_IMM": jump("v_cmp_gt_i64 vcc, {IMM}, {A}", False),   # k > A
    "H_JLT_REG": jump("v_cmp_gt_i64 vcc, {S}, {A}", True),
    "H_JSET_IMM": jump("v_cmp_ne_u32 vcc, 0, {t0}", False,
                       "v_and_b32 {t0}, {IMML}, {AL}\nv_and_b32 {t1}, {IMMH}, {AH}\nv_or_b32 {t0}, {t0}, {t1}\n"),
    "H_JSET_REG": jump("v_cmp_ne_u32 vcc, 0, {t0}", True,
                       "v_and_b32 {t0}, {SL}, {AL}\nv_and_b32 {t1}, {SH}, {AH}\nv_or_b32 {t0}, {t0}, {t1}\n"),
    # JMP32: signed compares of the low words == compares of the sign-extended words (Q3)
    "H_JEQ32_IMM": jump("v_cmp_eq_u32 vcc, {IMML}, {AL}", False),
    "H_JEQ32_REG": jump("v_cmp_eq_u32 vcc, {SL}, {AL}", True),
    "H_JGT32_IMM": jump("v_cmp_lt_i32 vcc, {IMML}, {AL}", False),
    "H_JGT32_REG": jump("v_cmp_lt_i32 vcc, {SL}, {AL}", True),
    "H_JLT32_IMM": jump("v_cmp_gt_i32 vcc, {IMML}, {AL}", False),
    "H_JLT32_REG": jump("v_cmp_gt_i32 vcc, {SL}, {AL}", True),
    "H_JSET32_IMM": jump("v_cmp_ne_u32 vcc, 0, {t0}", False, "v_and_b32 {t0}, {IMML}, {AL}\n"),
    "H_JSET32_REG": jump("v_cmp_ne_u32 vcc, 0, {t0}", True, "v_and_b32 {t0}, {SL}, {AL}\n"),
    "H_LDXK": "s_branch .Lldxk%=",
    "H_LDXK_FAR": "s_branch .Lldxkfar%=",
    "H_LDX": "s_branch .Lldx%=",
}


def window_addr(dst, b):
    """LDS address of window dword b (VGPR, a multiple of 4) of this lane: the 16-byte chunk
    (b & 0x30) is XOR-swizzled per lane (interp.hip win_off)."""
    return f"""v_and_b32 {{t18}}, 48, {b}
v_xor_b32 {{t18}}, {{t18}}, %[swz]
v_and_b32 {{t19}}, 15, {b}
v_add3_u32 {dst}, %[win], {{t18}}, {{t19}}"""


def window_tail(a0, shift):
    """{WD0..2} = the three dwords at (a0 & ~3) (LDS reads or global loads in flight), byte
    shift in `shift`; mask to the access width (k), zero the bytes at or past len (the zeroed
    image, main.rs:16), merge into the old dst value (upper bytes kept, Q1) and commit."""
    return f"""v_sub_u32_e64 {{LENM}}, %[len], {a0}
v_cmp_lt_u32 vcc, {a0}, %[len]
v_cndmask_b32 {{LENM}}, 0, {{LENM}}, vcc
v_min_u32 {{LENM}}, 8, {{LENM}}
v_lshlrev_b32 {{LENM}}, 3, {{LENM}}
v_sub_u32 {{LENM}}, 64, {{LENM}}
{READ_A}
{WAIT}
v_alignbyte_b32 {{RL}}, {{WD1}}, {{WD0}}, {shift}
v_alignbyte_b32 {{RH}}, {{WD2}}, {{WD1}}, {shift}
v_and_b32 {{RL}}, {{KML}}, {{RL}}
v_and_b32 {{RH}}, {{KMH}}, {{RH}}
v_lshlrev_b64 {{R}}, {{LENM}}, {{R}}
v_lshrrev_b64 {{R}}, {{LENM}}, {{R}}
v_cndmask_b32 {{RL}}, 0, {{RL}}, vcc
v_cndmask_b32 {{RH}}, 0, {{RH}}, vcc
v_bfi_b32 {{RL}}, {{KML}}, {{RL}}, {{AL}}
v_bfi_b32 {{RH}}, {{KMH}}, {{RH}}, {{AH}}
{TAIL_W}"""


def far_read(a0v, tag):
    """Current exec = lanes reading packet bytes outside the window (a0v < len): {WD0..2} =
    the dwords at (a0 & ~3) + 0/4/8, each loaded only if it holds a packet byte (pkt_read in
    interp.hip: no access leaves the page of a valid byte), else 0."""
    return f"""v_and_b32 {{t10}}, -4, {a0v}
v_mov_b32 {{t11}}, 0
v_lshl_add_u64 {{T89}}, %[base], 0, {{T1011}}
global_load_dword {{WD0}}, {{T89}}, off
v_mov_b32 {{WD1}}, 0
v_mov_b32 {{WD2}}, 0
s_mov_b64 {{T8}}, exec
v_add_u32 {{t12}}, 4, {{t10}}
v_cmp_lt_u32 vcc, {{t12}}, %[len]
s_and_b64 exec, {{T8}}, vcc
s_cbranch_scc0 .Lfa_{tag}%=
global_load_dword {{WD1}}, {{T89}}, off offset:4
.Lfa_{tag}%=:
s_mov_b64 exec, {{T8}}
v_add_u32 {{t12}}, 8, {{t10}}
v_cmp_lt_u32 vcc, {{t12}}, %[len]
s_and_b64 exec, {{T8}}, vcc
s_cbranch_scc0 .Lfb_{tag}%=
global_load_dword {{WD2}}, {{T89}}, off offset:8
.Lfb_{tag}%=:
s_mov_b64 exec, {{T8}}
s_waitcnt vmcnt(0)"""


# LDXK: constant address a0 = A0 inside the window, end = END; window dword i at chunk bits
# W[2i] (xor'ed with the lane swizzle), byte-in-chunk W[2i + 1]
LDXK = f""".Lldxk%=:
s_cmp_gt_u32 {{END}}, %[mem]
s_cbranch_scc1 .Lkfault%=
v_xor_b32 {{WD0}}, {{W0}}, %[swz]
v_add3_u32 {{WD0}}, %[win], {{WD0}}, {{W1}}
v_xor_b32 {{WD1}}, {{W2}}, %[swz]
v_add3_u32 {{WD1}}, %[win], {{WD1}}, {{W3}}
v_xor_b32 {{WD2}}, {{W4}}, %[swz]
v_add3_u32 {{WD2}}, %[win], {{WD2}}, {{W5}}
ds_read_b32 {{WD0}}, {{WD0}}
ds_read_b32 {{WD1}}, {{WD1}}
ds_read_b32 {{WD2}}, {{WD2}}
s_and_b32 {{T3}}, {{A0}}, 3
{window_tail("{A0}", "{T3}")}
.Lkfault%=:
s_cmp_ge_u32 {{A0}}, %[mem]
s_cselect_b32 {{T3}}, {ST_MEM}, {ST_MEM_UB}
v_mov_b32 %[st], {{T3}}
v_mov_b32 %[lpc], -1
s_branch .Lloop%="""

# LDXK outside the window: a0 < 2^32 (the host faults larger constants statically)
LDXK_FAR = f""".Lldxkfar%=:
s_cmp_gt_u32 {{END}}, %[mem]
s_cbranch_scc1 .Lkfault%=
v_mov_b32 {{t7}}, {{A0}}
v_mov_b32 {{WD0}}, 0
v_mov_b32 {{WD1}}, 0
v_mov_b32 {{WD2}}, 0
s_mov_b64 {{T7}}, exec
v_cmp_lt_u32 vcc, {{A0}}, %[len]
s_and_b64 exec, {{T7}}, vcc
s_cbranch_scc0 .Lkf_none%=
{far_read("{t7}", "kf")}
.Lkf_none%=:
s_mov_b64 exec, {{T7}}
s_and_b32 {{T3}}, {{A0}}, 3
{window_tail("{A0}", "{T3}")}"""

# LDX: address = S + sext(off) (IMM), mmu.rs bounds per lane: signed overflow or addr >= mem ->
# ST_MEM, addr + width > mem -> ST_MEM_UB (emu.rs:344, mmu.rs:13-30); then the window (addr +
# width <= 64), or the packet bytes past it, or zeros past the packet
LDX = f""".Lldx%=:
{READ_S}
v_lshl_add_u64 {{T01}}, {{S}}, 0, {{IMM}}
v_xor_b32 {{t2}}, {{SH}}, {{t1}}
v_xor_b32 {{t3}}, {{IMMH}}, {{t1}}
v_and_b32 {{t2}}, {{t2}}, {{t3}}
v_cmp_gt_i32_e64 {{T0}}, 0, {{t2}}
v_cmp_ne_u32_e64 {{T1}}, 0, {{t1}}
s_or_b64 {{T0}}, {{T0}}, {{T1}}
v_cmp_le_u32_e64 {{T1}}, %[mem], {{t0}}
s_or_b64 {{T0}}, {{T0}}, {{T1}}
v_add_u32 {{t4}}, {{WID}}, {{t0}}
v_cmp_lt_u32_e64 {{T1}}, %[mem], {{t4}}
s_andn2_b64 {{T1}}, {{T1}}, {{T0}}
s_or_b64 vcc, {{T0}}, {{T1}}
v_cndmask_b32_e64 {{t5}}, {ST_MEM_UB}, {ST_MEM}, {{T0}}
{fault_split("ldx", "{t5}")}
v_cmp_lt_u32_e64 {{T1}}, 64, {{t4}}
v_cndmask_b32_e64 {{t6}}, {{t0}}, 0, {{T1}}
v_and_b32 {{t6}}, -4, {{t6}}
{window_addr("{WD0}", "{t6}")}
v_add_u32 {{t7}}, 4, {{t6}}
v_min_u32 {{t7}}, 60, {{t7}}
{window_addr("{WD1}", "{t7}")}
v_add_u32 {{t7}}, 8, {{t6}}
v_min_u32 {{t7}}, 60, {{t7}}
{window_addr("{WD2}", "{t7}")}
ds_read_b32 {{WD0}}, {{WD0}}
ds_read_b32 {{WD1}}, {{WD1}}
ds_read_b32 {{WD2}}, {{WD2}}
v_cmp_lt_u32_e64 {{T0}}, {{t0}}, %[len]
s_and_b64 {{T7}}, {{T1}}, {{T0}}
s_cbranch_scc0 .Lldx_near%=
{WAIT}
s_mov_b64 {{T5}}, exec
s_mov_b64 exec, {{T7}}
{far_read("{t0}", "ldx")}
s_mov_b64 exec, {{T5}}
.Lldx_near%=:
v_and_b32 {{SHF}}, 3, {{t0}}
{window_tail("{t0}", "{SHF}")}"""

# bit-serial restoring division: T45 dividend, T67 divisor -> T01 quotient, T23 remainder;
# division by zero: DIV -> 0, MOD -> dividend (T1011) (emu.rs:90-100,126-135, Q5)
DIVMOD = """.Ldivmod%=:
v_mov_b32 {t0}, 0
v_mov_b32 {t1}, 0
v_mov_b32 {t2}, 0
v_mov_b32 {t3}, 0
s_mov_b32 {CNT}, 64
.Ldivloop%=:
v_lshlrev_b64 {T23}, 1, {T23}
v_lshrrev_b32 {t8}, 31, {t5}
v_or_b32 {t2}, {t2}, {t8}
v_lshlrev_b64 {T45}, 1, {T45}
v_lshlrev_b64 {T01}, 1, {T01}
v_cmp_ge_u64 vcc, {T23}, {T67}
v_sub_co_u32_e64 {t8}, {T5}, {t2}, {t6}
v_subb_co_u32_e64 {t9}, {T5}, {t3}, {t7}, {T5}
v_cndmask_b32 {t2}, {t2}, {t8}, vcc
v_cndmask_b32 {t3}, {t3}, {t9}, vcc
v_cndmask_b32_e64 {t8}, 0, 1, vcc
v_or_b32 {t0}, {t0}, {t8}
s_sub_u32 {CNT}, {CNT}, 1
s_cmp_lg_u32 {CNT}, 0
s_cbranch_scc1 .Ldivloop%=
v_cmp_eq_u64 vcc, 0, {T67}
s_cmp_eq_u32 {MODE}, 0
s_cbranch_scc0 .Lmodres%=
v_cndmask_b32_e64 {RL}, {t0}, 0, vcc
v_cndmask_b32_e64 {RH}, {t1}, 0, vcc
s_branch .Ldivend%=
.Lmodres%=:
v_cndmask_b32 {RL}, {t2}, {t10}, vcc
v_cndmask_b32 {RH}, {t3}, {t11}, vcc
.Ldivend%=:
""" + TAIL_W

INIT = "\n".join([
    "s_cmp_lg_u64 %[initp], 0",
    "s_cbranch_scc1 .Linitc%=",
] + [f"v_mov_b32 v{VB + i}, 0" for i in range(22) if i not in (4, 20, 21)] + [
    f"v_mov_b32 v{VB + 4}, %[len]",
    f"v_mov_b32 v{VB + 20}, %[r10l]",
    f"v_mov_b32 v{VB + 21}, %[r10h]",
    "s_branch .Linitd%=",
    ".Linitc%=:",
    "s_load_dwordx16 s[64:79], %[initp], 0x0",   # r0..r7: exactly the caller's 88 bytes
    "s_load_dwordx4 s[80:83], %[initp], 0x40",
    "s_load_dwordx2 s[84:85], %[initp], 0x50",
    WAIT,
] + [f"v_mov_b32 v{VB + i}, s{64 + i}" for i in range(22)] + [".Linitd%="":"])

PROLOGUE = INIT + """
s_mov_b64 {EXEC0}, exec
s_min_u32 {MEMW}, %[mem], 64
s_getpc_b64 {SLOTB}
.Lpc%=:
s_add_u32 {SLOTBL}, {SLOTBL}, .Lslots%=-.Lpc%=
s_addc_u32 {SLOTBH}, {SLOTBH}, 0
.Lloop%=:
s_mov_b64 exec, {EXEC0}
s_ff1_i32_b64 {P}, %[live]
s_cmp_lt_i32 {P}, 0
s_cbranch_scc1 .Ldone%=
s_bitset0_b64 %[live], {P}
s_lshl_b32 {T2}, {P}, 8
s_load_dwordx16 s[64:79], %[prog], {T2}
s_add_u32 {T2}, {T2}, 64
s_load_dwordx8 s[80:87], %[prog], {T2}
v_cmp_eq_u32 vcc, {P}, %[lpc]
s_mov_b64 exec, vcc
s_waitcnt lgkmcnt(0)
s_add_u32 {JTL}, {SLOTBL}, {HOFF}
s_addc_u32 {JTH}, {SLOTBH}, 0
s_setpc_b64 {JT}
.p2align 7
.Lslots%=:"""

EPILOGUE = f""".Ldone%=:
v_mov_b32 %[r0l], {{RF0}}
v_mov_b32 %[r0h], {{RF1}}
s_cmp_eq_u32 %[rflag], 0
s_cbranch_scc1 .Lend%=
v_cmp_ne_u32 vcc, 0, %[vok]
s_and_saveexec_b64 {{T4}}, vcc
""" + "\n".join(f"global_store_dwordx2 %[raddr], v[{VB + 2 * r}:{VB + 2 * r + 1}], off offset:{8 * r}"
                for r in range(11)) + """
s_waitcnt vmcnt(0)
s_mov_b64 exec, {T4}
.Lend%=:"""


# handlers longer than a 128-byte slot (the assembler's .org refuses an overfull slot)
OUT_OF_LINE = {"H_ARSH64_IMM", "H_ARSH64_REG"}


def main():
    names = [n for n, i in sorted(IDS.items(), key=lambda kv: kv[1]) if n != "H_COUNT"]
    assert [IDS[n] for n in names] == list(range(len(names))), "handler ids must be dense"
    missing = [n for n in names if n not in H]
    assert not missing, missing
    parts = [PROLOGUE]
    bodies = []
    for n in names:  # a handler too long for its slot runs out of line behind a trampoline
        code = H[n]
        if n in OUT_OF_LINE:
            bodies.append(f".L{n.lower()}%=:\n" + code)
            code = f"s_branch .L{n.lower()}%="
        parts.append(f"; {n}\n.org .Lslots%=+{IDS[n] * SLOT}\n" + code)
    parts.append(f".org .Lslots%=+{IDS['H_COUNT'] * SLOT}")
    parts += bodies + [LDXK, LDXK_FAR, LDX, DIVMOD, EPILOGUE]
    text = F("\n".join(parts))
    assert "{" not in text, "unsubstituted register name"
    out = ["// GENERATED by gen_dag_tile.py from dag_asm.h -- do not edit. One inline-asm statement.",
           "// clang-format off"]
    for line in text.splitlines():
        out.append('"' + line.replace("\\", "\\\\").replace('"', '\\"') + '\\n"')
    out.append("// clang-format on")
    print("\n".join(out))


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "--clobbers":
        print(", ".join(f'"s{s}"' for s in SGPRS) + ", " +
              ", ".join(f'"v{v}"' for v in range(VB, VB + NVGPR)))
    else:
        main()
