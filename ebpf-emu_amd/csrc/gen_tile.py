#!/usr/bin/env python3
"""Generates tile.inc + tile_ids.h: the gfx950 interpreter of one tile (64 packets, one per lane)
of a forward-only tier-0 program, as ONE inline-asm statement (tile_kernel in interp.hip).

What the statement does, between the C++ header-window DMA and the counter ballots:
  * prologue: per-lane packet address / length (FIXED stride layout, or the LDS metadata the
    C++ prologue DMA'd), validity, the main.rs:14-31 register layout (or the caller's
    init_regs), the ST_BADPKT check (main.rs:20-21), the pc set;
  * the interpreter: the lowest pc with a parked lane runs next ("min-pc" re-convergence,
    forward jumps only, so each pc runs at most once per tile). Dispatch = one s_load_dwordx16
    of the micro-op (uop.h TUop, 64 bytes) + s_setpc into fixed 256-byte handler slots;
    exec is narrowed to the lanes parked at the pc (v_cmpx) and results are committed under it;
  * basic-block chaining: a micro-op whose successor is not a block start (no jump lands there)
    has a chained form that loads its successor and jumps straight to it, skipping the pc-set
    update and the min-pc search; only block-ending micro-ops touch the pc set;
  * register file r0..r10 in v[0:21], accessed IN PLACE under s_set_gpr_idx (the dst/src
    register is scalar: dst2/src2 of the micro-op);
  * every tier-0 micro-op kind (ALU incl. MUL, DIV/MOD by a bit-serial divider, NEG, the
    reference's ARSH with its overflow fault; END; canonical jumps; LDX with the mmu.rs bounds
    checks, reads in the LDS header window and past it; static faults);
  * epilogue: verdict / r0 / status / final registers stored for the valid lanes; outputs the
    lane's counter bucket (0..4 r0, 5 other, 6 fault, 7 not a packet) and retired steps.
The DONE sentinel: bit 63 of the pc set is always set and micro-op 63 is the DONE handler, so
the min-pc search needs no empty-set test (programs of <= 63 micro-ops).

Only SALU/VALU/DS/SMEM, VGPR index mode and plain global loads/stores on VGPR addresses: no
readlane, DPP, trans, SDWA or VALU-written SGPRs feeding VMEM, so no gfx950 software wait states
are needed inside (MI355X guide §5.7 item 2); M0 is saved on entry and restored on exit.

  python3 gen_tile.py           # writes tile.inc and tile_ids.h next to this file
  python3 gen_tile.py --clobbers
"""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
IDS_OLD = {m.group(1): int(m.group(2)) for m in re.finditer(
    r"#define (H_\w+) (\d+)", open(os.path.join(HERE, "dag_asm.h")).read())}
SLOT = 256

# status codes (include/ebpf_emu.h)
ST_MEM, ST_MEM_UB, ST_INSN, ST_ARITH, ST_BADPKT = 1, 2, 3, 4, 7

NVGPR = 56  # v[0:55] belong to the statement (clobbered)
# s[33:70] belong to the statement: within the 72 SGPRs of 8 waves per SIMD, and clear of s32 (the
# ABI stack pointer). The micro-op is s[36:51] (s_load_dwordx16 needs a 4-aligned destination).
UB = 36


def u(i, n=1):
    return f"s{UB + i}" if n == 1 else f"s[{UB + i}:{UB + i + n - 1}]"


M = {
    # TUop, dword i in s[UB + i] (uop.h)
    "HOFF": u(0), "DST2": u(1), "SRC2": u(2), "NPC": u(3), "X": u(4), "A0": u(5),
    "KML": u(6), "KMH": u(7), "NBIT": u(8, 2), "TBIT": u(10, 2),
    "IMM": u(12, 2), "IMML": u(12), "IMMH": u(13), "WID": u(14), "END": u(15),
    "UOP": u(0, 16),
    # LDXK: byte offsets of the window dwords (a0 & ~3) + 0/4/8 (clamped to 60), the end address,
    # the bit shift of a one-dword access; steps to take back on a fault (REMK for LDXK, REMX for
    # LDX and ARSH64); BLEN: the length of the basic block this micro-op starts (retired steps)
    "W0": u(2), "W1": u(10), "W2": u(11), "KEND": u(4), "KSHIFT": u(12), "REMK": u(14),
    "REMX": u(5), "BLEN": u(15),
    # divider: its mode lives in the (dead after dispatch) handler offset
    "MODE": u(0),
    # prologue / epilogue scratch inside the micro-op registers
    "KFR": u(0, 2), "KST": u(2, 2), "KSTL": u(2), "KSTH": u(3), "KN": u(4, 2),
    "KOFF": u(6, 2), "KLEN": u(8, 2), "KINIT": u(10, 2), "KR10": u(12, 2),
    "KR10L": u(12), "KR10H": u(13), "KFRL": u(0), "KFRH": u(1), "KNL": u(4), "KNH": u(5),
    "EV": u(0, 2), "ER0": u(2, 2), "EST": u(4, 2), "ERG": u(6, 2),
    "KMEM": "s33", "T3": "s34", "CNT": "s34", "M0S": "s35",
    "LIVE": "s[52:53]", "PROG": "s[54:55]", "PROGL": "s54", "PROGH": "s55",
    "SLOTB": "s[56:57]", "SLOTBL": "s56", "SLOTBH": "s57", "VM": "s[58:59]",
    "T0": "s[60:61]", "T1": "s[62:63]", "T4": "s[64:65]", "T5": "s[66:67]", "T7": "s[68:69]",
    "T0L": "s60", "T0H": "s61", "T1L": "s62", "T1H": "s63", "T5L": "s66", "T5H": "s67",
    "T7L": "s68", "T7H": "s69",
    "PCOFF": "s70",
    # loop mode: the step budget (max_steps, clamped to 32 bits)
    "MAXS": "s71",
    # the jump target and the dispatcher's pc use temporaries dead at that point
    "JT": "s[60:61]", "JTL": "s60", "JTH": "s61", "P": "s62",
    # every wave of the kernel is full: the statement runs with exec = all 64 lanes
    "EXEC0": "-1",
    # VGPRs: the register file r_i = v[2i : 2i+1] is v[0:21]
    "RF": "v[0:1]", "RF0": "v0", "RF1": "v1",
    "A": "v[54:55]", "AL": "v54", "AH": "v55",
    # loop mode: the packet offset of this lane's 64-byte LDS window (refilled on demand)
    "WB": "v22",
    "S": "v[24:25]", "SL": "v24", "SH": "v25",
    "R": "v[26:27]", "RL": "v26", "RH": "v27",
    "LPC": "v28", "NST": "v29", "ST": "v30", "LEN": "v31",
    "BASE": "v[32:33]", "BASEL": "v32", "BASEH": "v33", "WIN": "v34", "SWZ": "v35",
}
for i in range(20):
    M[f"t{i}"] = f"v{36 + i}"
for i in range(0, 20, 2):
    M[f"T{i}{i + 1}"] = f"v[{36 + i}:{37 + i}]"
M.update({"WD0": M["t13"], "WD1": M["t14"], "WD2": M["t15"], "SHF": M["t16"], "LENM": M["t17"]})
SGPRS = list(range(33, 72))


def F(text):
    """Substitute {NAME} register names (the asm's own %[..] operands and %= are untouched)."""
    return re.sub(r"\{(\w+)\}", lambda m: M[m.group(1)], text)


def on(modes, idx="{DST2}"):
    return f"s_set_gpr_idx_on {idx}, gpr_idx({modes})"


OFF = "s_set_gpr_idx_off"
READ_A = f"{on('SRC0')}\nv_mov_b64 {{A}}, {{RF}}\n{OFF}"
READ_S = f"{on('SRC0', '{SRC2}')}\nv_mov_b64 {{S}}, {{RF}}\n{OFF}"
WRITE_R = f"{on('DST')}\nv_mov_b64 {{RF}}, {{R}}\n{OFF}"
WRITE_R32 = f"{on('DST')}\nv_mov_b32 {{RF0}}, {{RL}}\nv_mov_b32 {{RF1}}, 0\n{OFF}"
STEP = ""  # steps are counted per basic block at dispatch (BLEN); faults take back REM

# Find the lowest parked pc (bit 63 = the DONE sentinel), fetch its micro-op, narrow exec to the
# lanes parked there, jump to its handler.
DISPATCH = """s_mov_b64 exec, {EXEC0}
s_ff1_i32_b64 {P}, {LIVE}
s_bitset0_b64 {LIVE}, {P}
s_lshl_b32 {PCOFF}, {P}, 6
s_load_dwordx16 {UOP}, {PROG}, {PCOFF}
v_cmpx_eq_u32 vcc, {P}, {LPC}
s_waitcnt lgkmcnt(0)
v_add_u32 {NST}, {BLEN}, {NST}
.if %[loops]
v_cmp_lt_u32 vcc, {MAXS}, {NST}
s_cbranch_vccnz .Lbudget%=
.endif
s_add_u32 {JTL}, {SLOTBL}, {HOFF}
s_addc_u32 {JTH}, {SLOTBH}, 0
s_setpc_b64 {JT}"""

# Chained successor: same lanes, next micro-op.
CHAIN = """s_add_u32 {PCOFF}, {PCOFF}, 64
s_load_dwordx16 {UOP}, {PROG}, {PCOFF}
s_waitcnt lgkmcnt(0)
s_add_u32 {JTL}, {SLOTBL}, {HOFF}
s_addc_u32 {JTH}, {SLOTBH}, 0
s_setpc_b64 {JT}"""

# Block end of a non-jump: park the lanes at npc.
END_N = "v_mov_b32 {LPC}, {NPC}\ns_or_b64 {LIVE}, {LIVE}, {NBIT}\n" + DISPATCH

# Block end of a conditional jump: vcc = taken lanes among the active ones.
JTAIL = """v_mov_b32 {t0}, {X}
v_mov_b32 {t1}, {NPC}
v_cndmask_b32 {LPC}, {t1}, {t0}, vcc
s_cmp_lg_u64 vcc, 0
s_cselect_b64 {T0}, {TBIT}, 0
s_andn2_b64 {T1}, exec, vcc
s_cselect_b64 {T1}, {NBIT}, 0
s_or_b64 {LIVE}, {LIVE}, {T0}
s_or_b64 {LIVE}, {LIVE}, {T1}
""" + DISPATCH


def fault_split(tag, status, rem):
    """vcc = faulting lanes among the active ones: they stop with `status` (the steps of their
    block from this micro-op on, `rem`, are not retired); exec continues with the others (to the
    dispatcher when there are none)."""
    return f"""s_mov_b64 {{T4}}, exec
s_and_b64 exec, {{T4}}, vcc
s_cbranch_scc0 .Lnf_{tag}%=
v_mov_b32 {{ST}}, {status}
v_mov_b32 {{LPC}}, -1
v_subrev_u32 {{NST}}, {rem}, {{NST}}
.Lnf_{tag}%=:
s_andn2_b64 exec, {{T4}}, vcc
s_cbranch_scc0 .Ldisp%="""


# ---- handler bodies (without their tail): ALU-like kinds get a chained and a block-end form ----
def inplace64(op):
    return f"{on('SRC1,DST')}\n{op} {{RF0}}, {{IMML}}, {{RF0}}\n{op} {{RF1}}, {{IMMH}}, {{RF1}}\n{OFF}"


def inplace64r(op):
    return f"{READ_S}\n{on('SRC1,DST')}\n{op} {{RF0}}, {{SL}}, {{RF0}}\n{op} {{RF1}}, {{SH}}, {{RF1}}\n{OFF}"


def inplace32(op, reg=False):
    b = "{SL}" if reg else "{IMML}"
    pre = READ_S + "\n" if reg else ""
    return f"{pre}{on('SRC1,DST')}\n{op} {{RF0}}, {b}, {{RF0}}\nv_mov_b32 {{RF1}}, 0\n{OFF}"


def mul64(reg):
    bl, bh = ("{SL}", "{SH}") if reg else ("{IMML}", "{IMMH}")
    pre = READ_A + "\n" + (READ_S + "\n" if reg else "")
    return pre + f"""v_mul_lo_u32 {{RL}}, {{AL}}, {bl}
v_mul_hi_u32 {{t0}}, {{AL}}, {bl}
v_mul_lo_u32 {{t1}}, {{AL}}, {bh}
v_mul_lo_u32 {{t2}}, {{AH}}, {bl}
v_add3_u32 {{RH}}, {{t0}}, {{t1}}, {{t2}}
{WRITE_R}"""


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
{fault_split(tag, ST_ARITH, "{REMX}")}
{WRITE_R}"""


def arsh32(reg):
    sh = "{SL}" if reg else "{IMML}"
    pre = READ_A + "\n" + (READ_S + "\n" if reg else "")
    return pre + f"""v_alignbit_b32 {{t0}}, {{AL}}, {{AL}}, {sh}
v_sub_u32 {{t1}}, 0, {{t0}}
v_cmp_gt_i32 vcc, 0, {{AL}}
v_cndmask_b32 {{RL}}, {{t0}}, {{t1}}, vcc
{WRITE_R32}"""


def divmod_setup(mod, w64, reg):
    """Dividend -> T45, divisor -> T67, original dividend -> T1011 (the result of a division by
    zero for MOD); MODE = 1 for MOD. 32-bit forms: zero-extended low words (Q6). The divider
    (out of line) writes dst and returns through MODE bit 1 (chained) to the right tail."""
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
s_mov_b32 {{MODE}}, {1 if mod else 0}"""


def jump(cmp, reg, pre=""):
    return (READ_S + "\n" if reg else "") + f"{pre}{cmp}"


# name -> (body, kind): kind "alu" (chained + end forms), "jump" (end form, JTAIL), "term"
# (complete: ends itself), "ool" (body jumps out of line; the out-of-line code ends with the
# form's tail)
H = {
    "H_EXIT": ("v_mov_b32 {LPC}, -1\n" + STEP + "\n" + DISPATCH, "term"),
    "H_FAULT": ("v_mov_b32 {ST}, {IMML}\nv_mov_b32 {LPC}, -1\nv_subrev_u32 {NST}, 1, {NST}\n" + DISPATCH, "term"),
    "H_SLOW": (f"v_mov_b32 {{ST}}, {ST_INSN}\nv_mov_b32 {{LPC}}, -1\nv_subrev_u32 {{NST}}, 1, {{NST}}\n" + DISPATCH, "term"),
    "H_MOV64_IMM": (f"{on('DST')}\nv_mov_b32 {{RF0}}, {{IMML}}\nv_mov_b32 {{RF1}}, {{IMMH}}\n{OFF}", "alu"),
    "H_MOV64_REG": (f"{READ_S}\n{on('DST')}\nv_mov_b64 {{RF}}, {{S}}\n{OFF}", "alu"),
    "H_ADD64_IMM": (f"{on('SRC0,DST')}\nv_lshl_add_u64 {{RF}}, {{RF}}, 0, {{IMM}}\n{OFF}", "alu"),
    "H_ADD64_REG": (f"{READ_S}\n{on('SRC0,DST')}\nv_lshl_add_u64 {{RF}}, {{RF}}, 0, {{S}}\n{OFF}", "alu"),
    "H_SUB64_REG": (f"{READ_S}\n{on('SRC0,DST')}\nv_sub_co_u32 {{RF0}}, vcc, {{RF0}}, {{SL}}\n"
                    f"v_subb_co_u32 {{RF1}}, vcc, {{RF1}}, {{SH}}, vcc\n{OFF}", "alu"),
    "H_AND64_IMM": (inplace64("v_and_b32"), "alu"), "H_AND64_REG": (inplace64r("v_and_b32"), "alu"),
    "H_OR64_IMM": (inplace64("v_or_b32"), "alu"), "H_OR64_REG": (inplace64r("v_or_b32"), "alu"),
    "H_XOR64_IMM": (inplace64("v_xor_b32"), "alu"), "H_XOR64_REG": (inplace64r("v_xor_b32"), "alu"),
    # the hardware uses bits [5:0] / [4:0] of the shift count: the reference's masks (Q20)
    "H_LSH64_IMM": (f"{on('SRC1,DST')}\nv_lshlrev_b64 {{RF}}, {{IMML}}, {{RF}}\n{OFF}", "alu"),
    "H_LSH64_REG": (f"{READ_S}\n{on('SRC1,DST')}\nv_lshlrev_b64 {{RF}}, {{SL}}, {{RF}}\n{OFF}", "alu"),
    "H_RSH64_IMM": (f"{on('SRC1,DST')}\nv_lshrrev_b64 {{RF}}, {{IMML}}, {{RF}}\n{OFF}", "alu"),
    "H_RSH64_REG": (f"{READ_S}\n{on('SRC1,DST')}\nv_lshrrev_b64 {{RF}}, {{SL}}, {{RF}}\n{OFF}", "alu"),
    "H_MOV32_IMM": (f"{on('DST')}\nv_mov_b32 {{RF0}}, {{IMML}}\nv_mov_b32 {{RF1}}, 0\n{OFF}", "alu"),
    "H_MOV32_REG": (f"{READ_S}\n{on('DST')}\nv_mov_b32 {{RF0}}, {{SL}}\nv_mov_b32 {{RF1}}, 0\n{OFF}", "alu"),
    "H_ADD32_IMM": (inplace32("v_add_u32"), "alu"),
    "H_ADD32_REG": (inplace32("v_add_u32", True), "alu"),
    "H_SUB32_REG": (inplace32("v_subrev_u32", True), "alu"),  # dst - src
    "H_AND32_IMM": (inplace32("v_and_b32"), "alu"),
    "H_AND32_REG": (inplace32("v_and_b32", True), "alu"),
    "H_OR32_IMM": (inplace32("v_or_b32"), "alu"),
    "H_OR32_REG": (inplace32("v_or_b32", True), "alu"),
    "H_XOR32_IMM": (inplace32("v_xor_b32"), "alu"),
    "H_XOR32_REG": (inplace32("v_xor_b32", True), "alu"),
    "H_LSH32_IMM": (inplace32("v_lshlrev_b32"), "alu"),
    "H_LSH32_REG": (inplace32("v_lshlrev_b32", True), "alu"),
    "H_RSH32_IMM": (inplace32("v_lshrrev_b32"), "alu"),
    "H_RSH32_REG": (inplace32("v_lshrrev_b32", True), "alu"),
    "H_ZX16": (f"{on('SRC1,DST')}\nv_and_b32 {{RF0}}, 0xffff, {{RF0}}\nv_mov_b32 {{RF1}}, 0\n{OFF}", "alu"),
    "H_ZX32": (f"{on('DST')}\nv_mov_b32 {{RF1}}, 0\n{OFF}", "alu"),
    "H_NOP": ("", "alu"),
    # v_perm_b32 selector bytes: 0..3 pick bytes of src1, 0x0c gives 0x00
    "H_BSWAP16": (f"s_mov_b32 {{T3}}, 0x0c0c0001\n{on('SRC0,SRC1,DST')}\n"
                  f"v_perm_b32 {{RF0}}, {{RF0}}, {{RF0}}, {{T3}}\nv_mov_b32 {{RF1}}, 0\n{OFF}", "alu"),
    "H_BSWAP32": (f"s_mov_b32 {{T3}}, 0x00010203\n{on('SRC0,SRC1,DST')}\n"
                  f"v_perm_b32 {{RF0}}, {{RF0}}, {{RF0}}, {{T3}}\nv_mov_b32 {{RF1}}, 0\n{OFF}", "alu"),
    "H_BSWAP64": (f"""{READ_A}
s_mov_b32 {{T3}}, 0x00010203
v_perm_b32 {{RL}}, {{AH}}, {{AH}}, {{T3}}
v_perm_b32 {{RH}}, {{AL}}, {{AL}}, {{T3}}
{WRITE_R}""", "alu"),
    "H_MUL64_IMM": (mul64(False), "alu"), "H_MUL64_REG": (mul64(True), "alu"),
    "H_MUL32_IMM": (f"{READ_A}\nv_mul_lo_u32 {{RL}}, {{AL}}, {{IMML}}\n{WRITE_R32}", "alu"),
    "H_MUL32_REG": (f"{READ_A}\n{READ_S}\nv_mul_lo_u32 {{RL}}, {{AL}}, {{SL}}\n{WRITE_R32}", "alu"),
    "H_NEG64": (f"{on('SRC0,SRC1,DST')}\nv_sub_co_u32 {{RF0}}, vcc, 0, {{RF0}}\n"
                f"v_subb_co_u32 {{RF1}}, vcc, 0, {{RF1}}, vcc\n{OFF}", "alu"),
    "H_NEG32": (f"{on('SRC1,DST')}\nv_sub_u32 {{RF0}}, 0, {{RF0}}\nv_mov_b32 {{RF1}}, 0\n{OFF}", "alu"),
    "H_ARSH64_IMM": (arsh64(False), "alu"), "H_ARSH64_REG": (arsh64(True), "alu"),
    "H_ARSH32_IMM": (arsh32(False), "alu"), "H_ARSH32_REG": (arsh32(True), "alu"),
    "H_DIV64_IMM": (divmod_setup(False, True, False), "div"),
    "H_DIV64_REG": (divmod_setup(False, True, True), "div"),
    "H_MOD64_IMM": (divmod_setup(True, True, False), "div"),
    "H_MOD64_REG": (divmod_setup(True, True, True), "div"),
    "H_DIV32_IMM": (divmod_setup(False, False, False), "div"),
    "H_DIV32_REG": (divmod_setup(False, False, True), "div"),
    "H_MOD32_IMM": (divmod_setup(True, False, False), "div"),
    "H_MOD32_REG": (divmod_setup(True, False, True), "div"),
    "H_JA": ("v_mov_b32 {LPC}, {X}\n" + STEP + "\ns_or_b64 {LIVE}, {LIVE}, {TBIT}\n" + DISPATCH, "term"),
    # jumps: vcc = condition over the active lanes; x / npc, tbit / nbit already canonical
    "H_JEQ_IMM": (jump(f"{on('SRC1')}\nv_cmp_eq_u64 vcc, {{IMM}}, {{RF}}\n{OFF}", False), "jump"),
    "H_JEQ_REG": (jump(f"{on('SRC1')}\nv_cmp_eq_u64 vcc, {{S}}, {{RF}}\n{OFF}", True), "jump"),
    "H_JGT_IMM": (jump(f"{on('SRC1')}\nv_cmp_lt_i64 vcc, {{IMM}}, {{RF}}\n{OFF}", False), "jump"),  # k < A
    "H_JGT_REG": (jump(f"{on('SRC1')}\nv_cmp_lt_i64 vcc, {{S}}, {{RF}}\n{OFF}", True), "jump"),
    "H_JLT_IMM": (jump(f"{on('SRC1')}\nv_cmp_gt_i64 vcc, {{IMM}}, {{RF}}\n{OFF}", False), "jump"),  # k > A
    "H_JLT_REG": (jump(f"{on('SRC1')}\nv_cmp_gt_i64 vcc, {{S}}, {{RF}}\n{OFF}", True), "jump"),
    "H_JSET_IMM": (jump("v_cmp_ne_u32 vcc, 0, {t0}", False,
                        f"{on('SRC1')}\nv_and_b32 {{t0}}, {{IMML}}, {{RF0}}\nv_and_b32 {{t1}}, {{IMMH}}, {{RF1}}\n{OFF}\n"
                        "v_or_b32 {t0}, {t0}, {t1}\n"), "jump"),
    "H_JSET_REG": (jump("v_cmp_ne_u32 vcc, 0, {t0}", True,
                        f"{on('SRC1')}\nv_and_b32 {{t0}}, {{SL}}, {{RF0}}\nv_and_b32 {{t1}}, {{SH}}, {{RF1}}\n{OFF}\n"
                        "v_or_b32 {t0}, {t0}, {t1}\n"), "jump"),
    # JMP32: signed compares of the low words == compares of the sign-extended words (Q3)
    "H_JEQ32_IMM": (jump(f"{on('SRC1')}\nv_cmp_eq_u32 vcc, {{IMML}}, {{RF0}}\n{OFF}", False), "jump"),
    "H_JEQ32_REG": (jump(f"{on('SRC1')}\nv_cmp_eq_u32 vcc, {{SL}}, {{RF0}}\n{OFF}", True), "jump"),
    "H_JGT32_IMM": (jump(f"{on('SRC1')}\nv_cmp_lt_i32 vcc, {{IMML}}, {{RF0}}\n{OFF}", False), "jump"),
    "H_JGT32_REG": (jump(f"{on('SRC1')}\nv_cmp_lt_i32 vcc, {{SL}}, {{RF0}}\n{OFF}", True), "jump"),
    "H_JLT32_IMM": (jump(f"{on('SRC1')}\nv_cmp_gt_i32 vcc, {{IMML}}, {{RF0}}\n{OFF}", False), "jump"),
    "H_JLT32_REG": (jump(f"{on('SRC1')}\nv_cmp_gt_i32 vcc, {{SL}}, {{RF0}}\n{OFF}", True), "jump"),
    "H_JSET32_IMM": (jump("v_cmp_ne_u32 vcc, 0, {t0}", False,
                          f"{on('SRC1')}\nv_and_b32 {{t0}}, {{IMML}}, {{RF0}}\n{OFF}\n"), "jump"),
    "H_JSET32_REG": (jump("v_cmp_ne_u32 vcc, 0, {t0}", True,
                          f"{on('SRC1')}\nv_and_b32 {{t0}}, {{SL}}, {{RF0}}\n{OFF}\n"), "jump"),
    "H_LDXK": ("ldxk", "ool"),
    "H_LDXK1": ("ldxk1", "ool"),
    "H_LDXK2": ("ldxk2", "ool"),
    "H_LDXK_FAR": ("ldxkfar", "ool"),
    "H_LDX": ("ldx", "ool"),
    "H_LDX1": ("ldx1", "ool"),
}
DONE = "H_DONE"


def window_addr(dst, b):
    """LDS address of window dword b (a multiple of 4) of this lane: the 16-byte chunk bits
    (b & 0x30) are XOR-swizzled per lane (interp.hip win_off); SWZ has only bits 4-5 set, so
    the address is (b ^ SWZ) + WIN."""
    return f"v_xad_u32 {dst}, {{SWZ}}, {b}, {{WIN}}"


def window_tail(a0, shift):
    """{WD0..2} = the three dwords at (a0 & ~3) (LDS reads or global loads in flight), byte
    shift in `shift`; mask to the access width (k), zero the bytes at or past len (the zeroed
    image, main.rs:16; never the case in the FIXED layout, where every packet is >= 64 bytes
    long), merge into the old dst value (upper bytes kept, Q1) and commit."""
    return f""".if %[fixed] == 0
v_sub_u32_e64 {{LENM}}, {{LEN}}, {a0}
v_cmp_lt_u32 vcc, {a0}, {{LEN}}
v_cndmask_b32 {{LENM}}, 0, {{LENM}}, vcc
v_min_u32 {{LENM}}, 8, {{LENM}}
v_lshlrev_b32 {{LENM}}, 3, {{LENM}}
v_sub_u32 {{LENM}}, 64, {{LENM}}
.endif
{WAIT}
v_alignbyte_b32 {{RL}}, {{WD1}}, {{WD0}}, {shift}
v_alignbyte_b32 {{RH}}, {{WD2}}, {{WD1}}, {shift}
.if %[fixed] == 0
v_and_b32 {{RL}}, {{KML}}, {{RL}}
v_and_b32 {{RH}}, {{KMH}}, {{RH}}
v_lshlrev_b64 {{R}}, {{LENM}}, {{R}}
v_lshrrev_b64 {{R}}, {{LENM}}, {{R}}
v_cndmask_b32 {{RL}}, 0, {{RL}}, vcc
v_cndmask_b32 {{RH}}, 0, {{RH}}, vcc
.endif
{on('SRC2,DST')}
v_bfi_b32 {{RF0}}, {{KML}}, {{RL}}, {{RF0}}
v_bfi_b32 {{RF1}}, {{KMH}}, {{RH}}, {{RF1}}
{OFF}"""


WAIT = "s_waitcnt lgkmcnt(0)"


def far_read(a0v, tag, save="{T0}"):
    """Current exec = lanes reading packet bytes outside the window (a0v < len): {WD0..2} =
    the dwords at (a0 & ~3) + 0/4/8, each loaded only if it holds a packet byte (pkt_read in
    interp.hip: no access leaves the page of a valid byte), else 0."""
    return f"""v_and_b32 {{t10}}, -4, {a0v}
v_mov_b32 {{t11}}, 0
v_lshl_add_u64 {{T89}}, {{BASE}}, 0, {{T1011}}
global_load_dword {{WD0}}, {{T89}}, off
v_mov_b32 {{WD1}}, 0
v_mov_b32 {{WD2}}, 0
s_mov_b64 {save}, exec
v_add_u32 {{t12}}, 4, {{t10}}
v_cmp_lt_u32 vcc, {{t12}}, {{LEN}}
s_and_b64 exec, {save}, vcc
s_cbranch_scc0 .Lfa_{tag}%=
global_load_dword {{WD1}}, {{T89}}, off offset:4
.Lfa_{tag}%=:
s_mov_b64 exec, {save}
v_add_u32 {{t12}}, 8, {{t10}}
v_cmp_lt_u32 vcc, {{t12}}, {{LEN}}
s_and_b64 exec, {save}, vcc
s_cbranch_scc0 .Lfb_{tag}%=
global_load_dword {{WD2}}, {{T89}}, off offset:8
.Lfb_{tag}%=:
s_mov_b64 exec, {save}
s_waitcnt vmcnt(0)"""


def kcheck():
    return "s_cmp_gt_u32 {KEND}, {KMEM}\ns_cbranch_scc1 .Lkfault%="


def ldxk1(sfx):
    """LDXK, the access inside one window dword (a0 % 4 + width <= 4): shift it down, zero the
    bytes at or past len (not in the FIXED layout, where packets are >= 64 bytes), merge into the
    low word of dst (upper bytes kept, Q1; the high word is untouched)."""
    return f""".Lldxk1{sfx}%=:
{kcheck()}
{window_addr("{WD0}", "{W0}")}
ds_read_b32 {{WD0}}, {{WD0}}
.if %[fixed] == 0
v_subrev_u32 {{LENM}}, {{A0}}, {{LEN}}
v_min_u32 {{LENM}}, 4, {{LENM}}
v_lshlrev_b32 {{LENM}}, 3, {{LENM}}
v_sub_u32 {{LENM}}, 32, {{LENM}}
.endif
{WAIT}
v_lshrrev_b32 {{RL}}, {{KSHIFT}}, {{WD0}}
.if %[fixed] == 0
v_lshlrev_b32 {{RL}}, {{LENM}}, {{RL}}
v_lshrrev_b32 {{RL}}, {{LENM}}, {{RL}}
v_cmp_lt_u32 vcc, {{A0}}, {{LEN}}
v_cndmask_b32 {{RL}}, 0, {{RL}}, vcc
.endif
{on('SRC2,DST')}
v_bfi_b32 {{RF0}}, {{KML}}, {{RL}}, {{RF0}}
{OFF}
{TAILS[sfx]}"""


def ldxk2(sfx):
    """LDXK, a width <= 4 access spanning two window dwords."""
    return f""".Lldxk2{sfx}%=:
{kcheck()}
{window_addr("{WD0}", "{W0}")}
{window_addr("{WD1}", "{W1}")}
ds_read_b32 {{WD0}}, {{WD0}}
ds_read_b32 {{WD1}}, {{WD1}}
.if %[fixed] == 0
v_subrev_u32 {{LENM}}, {{A0}}, {{LEN}}
v_min_u32 {{LENM}}, 4, {{LENM}}
v_lshlrev_b32 {{LENM}}, 3, {{LENM}}
v_sub_u32 {{LENM}}, 32, {{LENM}}
.endif
{WAIT}
v_alignbyte_b32 {{RL}}, {{WD1}}, {{WD0}}, {{A0}}
.if %[fixed] == 0
v_lshlrev_b32 {{RL}}, {{LENM}}, {{RL}}
v_lshrrev_b32 {{RL}}, {{LENM}}, {{RL}}
v_cmp_lt_u32 vcc, {{A0}}, {{LEN}}
v_cndmask_b32 {{RL}}, 0, {{RL}}, vcc
.endif
{on('SRC2,DST')}
v_bfi_b32 {{RF0}}, {{KML}}, {{RL}}, {{RF0}}
{OFF}
{TAILS[sfx]}"""


def ldxk(sfx):
    """LDXK, general (8-byte) form: constant address a0 = A0 inside the window, end = KEND."""
    return f""".Lldxk{sfx}%=:
{kcheck()}
{window_addr("{WD0}", "{W0}")}
{window_addr("{WD1}", "{W1}")}
{window_addr("{WD2}", "{W2}")}
ds_read_b32 {{WD0}}, {{WD0}}
ds_read_b32 {{WD1}}, {{WD1}}
ds_read_b32 {{WD2}}, {{WD2}}
s_and_b32 {{T3}}, {{A0}}, 3
{window_tail("{A0}", "{T3}")}
{STEP}
{TAILS[sfx]}"""


# Step budget (loop mode). Block mode: some lane could run out of budget inside this block --
# restart the tile in exact mode (the one-micro-op-per-block table: a dispatch is one step), where
# the budget is checked before every step as the reference's max_steps (oracle: ST_STEPS when
# steps == max_steps before an instruction). Bit 62 of the pc set marks exact mode (entry 62 of
# every table is a second DONE sentinel). The restart re-reads the window from the packet where
# refills are possible (WB = -64: no byte is in the window) and keeps it otherwise (never refilled).
BUDGET = f""".Lbudget%=:
s_bitcmp1_b64 {{LIVE}}, 62
s_cbranch_scc1 .Lbexact%=
s_load_dwordx2 {{PROG}}, %[ka], %[o_tprog_exact]
s_mov_b64 exec, -1
s_mov_b64 {{LIVE}}, 0
s_bitset1_b64 {{LIVE}}, 62
s_cmp_eq_u32 %[aligned], 0
s_cbranch_scc1 .Lbkeep%=
v_mov_b32 {{WB}}, -64
.Lbkeep%=:
s_waitcnt lgkmcnt(0)
s_branch .Lreinit%=
.Lbexact%=:
s_mov_b64 {{T4}}, exec
s_mov_b64 exec, vcc
v_mov_b32 {{ST}}, 5
v_mov_b32 {{LPC}}, -1
v_subrev_u32 {{NST}}, 1, {{NST}}
s_andn2_b64 exec, {{T4}}, vcc
s_cbranch_scc0 .Ldisp%=
s_add_u32 {{JTL}}, {{SLOTBL}}, {{HOFF}}
s_addc_u32 {{JTH}}, {{SLOTBH}}, 0
s_setpc_b64 {{JT}}"""


# a fault of a constant-address load hits every active lane alike (mmu.rs:13-30)
KFAULT = f""".Lkfault%=:
s_cmp_ge_u32 {{A0}}, {{KMEM}}
s_cselect_b32 {{T3}}, {ST_MEM}, {ST_MEM_UB}
v_mov_b32 {{ST}}, {{T3}}
v_mov_b32 {{LPC}}, -1
v_subrev_u32 {{NST}}, {{REMK}}, {{NST}}
.Ldisp%=:
{DISPATCH}"""


def ldxkfar(sfx):
    """LDXK outside the window: a0 < 2^32 (the host faults larger constants statically)."""
    return f""".Lldxkfar{sfx}%=:
s_cmp_gt_u32 {{KEND}}, {{KMEM}}
s_cbranch_scc1 .Lkfault%=
v_mov_b32 {{t7}}, {{A0}}
v_mov_b32 {{WD0}}, 0
v_mov_b32 {{WD1}}, 0
v_mov_b32 {{WD2}}, 0
s_mov_b64 {{T7}}, exec
v_cmp_lt_u32 vcc, {{A0}}, {{LEN}}
s_and_b64 exec, {{T7}}, vcc
s_cbranch_scc0 .Lkf_none{sfx}%=
{far_read("{t7}", "kf" + sfx)}
.Lkf_none{sfx}%=:
s_mov_b64 exec, {{T7}}
s_and_b32 {{T3}}, {{A0}}, 3
{window_tail_ldx("{A0}", "{T3}")}
{STEP}
{TAILS[sfx]}"""


def ldx(sfx):
    """LDX: address = S + sext(off) (IMM), mmu.rs bounds per lane: the high word != 0 (every
    signed-overflowing sum has one too: emu.rs:344's panic, ST_MEM like the reference's slice
    panic) or addr >= mem -> ST_MEM; addr + width > mem -> ST_MEM_UB (mmu.rs:13-30); then the
    window (addr + width <= 64), or the packet bytes past it, or zeros past the packet."""
    return f""".Lldx{sfx}%=:
{READ_S}
v_lshl_add_u64 {{T01}}, {{S}}, 0, {{IMM}}
v_cmp_ne_u32_e64 {{T0}}, 0, {{t1}}
v_cmp_le_u32_e64 {{T1}}, {{KMEM}}, {{t0}}
s_or_b64 {{T0}}, {{T0}}, {{T1}}
v_add_u32 {{t4}}, {{WID}}, {{t0}}
v_cmp_lt_u32_e64 vcc, {{KMEM}}, {{t4}}
s_or_b64 vcc, vcc, {{T0}}
v_cndmask_b32_e64 {{t5}}, {ST_MEM_UB}, {ST_MEM}, {{T0}}
{fault_split("ldx" + sfx, "{t5}", "{REMX}")}
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
v_cmp_lt_u32_e64 {{T0}}, {{t0}}, {{LEN}}
s_and_b64 {{T7}}, {{T1}}, {{T0}}
s_cbranch_scc0 .Lldx_near{sfx}%=
{WAIT}
s_mov_b64 {{T5}}, exec
s_mov_b64 exec, {{T7}}
{far_read("{t0}", "ldx" + sfx)}
s_mov_b64 exec, {{T5}}
.Lldx_near{sfx}%=:
v_and_b32 {{SHF}}, 3, {{t0}}
{window_tail_ldx("{t0}", "{SHF}")}
{STEP}
{TAILS[sfx]}"""


def ldx_loop(sfx):
    """LDX in loop mode: the lane's 64-byte LDS window holds packet bytes [WB, WB + 64). An access
    outside it (that needs packet bytes, a < len) refills it from WB = a & ~15 with four 16-byte
    loads (chunks wholly past the packet are skipped: their bytes read as zero anyway) -- when
    every packet base of the tile is 16-byte aligned (%[aligned]), so that no 16-byte load
    leaves the page of a packet byte; otherwise such lanes read the packet dwords directly
    (far_read). Bounds and faults as ldx()."""
    return f""".Lldxl{sfx}%=:
{READ_S}
v_lshl_add_u64 {{T01}}, {{S}}, 0, {{IMM}}
v_cmp_ne_u32_e64 {{T0}}, 0, {{t1}}
v_cmp_le_u32_e64 {{T1}}, {{KMEM}}, {{t0}}
s_or_b64 {{T0}}, {{T0}}, {{T1}}
v_add_u32 {{t4}}, {{WID}}, {{t0}}
v_cmp_lt_u32_e64 vcc, {{KMEM}}, {{t4}}
s_or_b64 vcc, vcc, {{T0}}
v_cndmask_b32_e64 {{t5}}, {ST_MEM_UB}, {ST_MEM}, {{T0}}
{fault_split("ldxl" + sfx, "{t5}", "{REMX}")}
v_sub_u32 {{t6}}, {{t0}}, {{WB}}
s_sub_u32 {{T3}}, 64, {{WID}}
v_cmp_lt_u32_e64 {{T1}}, {{T3}}, {{t6}}
v_cmp_lt_u32_e64 {{T0}}, {{t0}}, {{LEN}}
s_and_b64 {{T7}}, {{T1}}, {{T0}}
s_cbranch_scc0 .Lldxl_win{sfx}%=
s_cmp_eq_u32 %[aligned], 0
s_cbranch_scc1 .Lldxl_win{sfx}%=
s_mov_b64 {{T5}}, exec
s_mov_b64 exec, {{T7}}
v_and_b32 {{WB}}, -16, {{t0}}
v_mov_b32 {{t7}}, 0
v_mov_b32 {{t6}}, {{WB}}
v_lshl_add_u64 {{T67}}, {{BASE}}, 0, {{T67}}
""" + "\n".join(f"""v_add_u32 {{t1}}, {16 * c}, {{WB}}
v_cmp_lt_u32 vcc, {{t1}}, {{LEN}}
s_and_b64 exec, {{T7}}, vcc
global_load_dwordx4 {reg}, {{T67}}, off offset:{16 * c}""" for c, reg in
               enumerate(("v[44:47]", "v[48:51]", "v[52:55]", "v[38:41]"))) + f"""
s_mov_b64 exec, {{T7}}
s_waitcnt vmcnt(0)
""" + "\n".join(f"""v_xad_u32 {{t1}}, {{SWZ}}, {16 * c}, {{WIN}}
ds_write_b128 {{t1}}, {reg}""" for c, reg in
                 enumerate(("v[44:47]", "v[48:51]", "v[52:55]", "v[38:41]"))) + f"""
s_waitcnt lgkmcnt(0)
s_mov_b64 exec, {{T5}}
.Lldxl_win{sfx}%=:
v_sub_u32 {{t6}}, {{t0}}, {{WB}}
v_and_b32 {{t6}}, -4, {{t6}}
v_min_u32 {{t6}}, 60, {{t6}}
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
v_sub_u32 {{t6}}, {{t0}}, {{WB}}
s_sub_u32 {{T3}}, 64, {{WID}}
v_cmp_lt_u32_e64 {{T1}}, {{T3}}, {{t6}}
v_cmp_lt_u32_e64 {{T0}}, {{t0}}, {{LEN}}
s_and_b64 {{T7}}, {{T1}}, {{T0}}
s_cbranch_scc0 .Lldxl_near{sfx}%=
{WAIT}
s_mov_b64 {{T5}}, exec
s_mov_b64 exec, {{T7}}
{far_read("{t0}", "ldxl" + sfx)}
s_mov_b64 exec, {{T5}}
.Lldxl_near{sfx}%=:
v_and_b32 {{SHF}}, 3, {{t0}}
{window_tail_ldx("{t0}", "{SHF}")}
{TAILS[sfx]}"""


def refill(tag):
    """Loop mode: exec = lanes whose access needs packet bytes outside their window (T7), tile
    aligned: WB = a & ~15, four 16-byte loads of [WB, WB + 64) (chunks wholly past the packet
    skipped), written to the lane's LDS window. Clobbers t1..t19 except t0 (the address)."""
    return f"""s_mov_b64 {{T5}}, exec
s_mov_b64 exec, {{T7}}
v_and_b32 {{WB}}, -16, {{t0}}
v_mov_b32 {{t7}}, 0
v_mov_b32 {{t6}}, {{WB}}
v_lshl_add_u64 {{T67}}, {{BASE}}, 0, {{T67}}
""" + "\n".join(f"""v_add_u32 {{t1}}, {16 * c}, {{WB}}
v_cmp_lt_u32 vcc, {{t1}}, {{LEN}}
s_and_b64 exec, {{T7}}, vcc
global_load_dwordx4 {reg}, {{T67}}, off offset:{16 * c}""" for c, reg in
                 enumerate(("v[44:47]", "v[48:51]", "v[52:55]", "v[38:41]"))) + f"""
s_mov_b64 exec, {{T7}}
s_waitcnt vmcnt(0)
""" + "\n".join(f"""v_xad_u32 {{t1}}, {{SWZ}}, {16 * c}, {{WIN}}
ds_write_b128 {{t1}}, {reg}""" for c, reg in
                 enumerate(("v[44:47]", "v[48:51]", "v[52:55]", "v[38:41]"))) + f"""
s_waitcnt lgkmcnt(0)
s_mov_b64 exec, {{T5}}"""


def ldx1(sfx, loop):
    """LDX of one byte (ldxb), register-based address: one window dword. a = S + sext(off);
    the high word != 0 or a >= mem -> ST_MEM (for one byte, a + 1 > mem is a >= mem; emu.rs:344,
    mmu.rs:23-30). Window bytes from LDS (loop mode: the window at WB, refilled as in
    ldx_loop), packet bytes past it from HBM (the dword holding byte a), bytes at or past len
    read as zero (main.rs:16); merged into the low byte of dst (Q1)."""
    lab = f"ldx1{'l' if loop else ''}{sfx}"
    win = "v_sub_u32 {t6}, {t0}, {WB}" if loop else "v_mov_b32 {t6}, {t0}"
    out = f""".L{lab}%=:
{READ_S}
v_lshl_add_u64 {{T01}}, {{S}}, 0, {{IMM}}
v_cmp_ne_u32_e64 {{T0}}, 0, {{t1}}
v_cmp_le_u32_e64 {{T1}}, {{KMEM}}, {{t0}}
s_or_b64 vcc, {{T0}}, {{T1}}
{fault_split(lab, ST_MEM, "{REMX}")}
{win}
v_cmp_lt_u32_e64 {{T0}}, {{t0}}, {{LEN}}
v_cmp_le_u32_e64 {{T1}}, 64, {{t6}}
s_and_b64 {{T7}}, {{T1}}, {{T0}}
"""
    if loop:
        out += f"""s_cbranch_scc0 .L{lab}_win%=
s_cmp_eq_u32 %[aligned], 0
s_cbranch_scc1 .L{lab}_win%=
{refill(lab)}
v_sub_u32 {{t6}}, {{t0}}, {{WB}}
v_cmp_le_u32_e64 {{T1}}, 64, {{t6}}
v_cmp_lt_u32_e64 {{T0}}, {{t0}}, {{LEN}}
s_and_b64 {{T7}}, {{T1}}, {{T0}}
.L{lab}_win%=:
"""
    out += f"""v_and_b32 {{t6}}, -4, {{t6}}
v_min_u32 {{t6}}, 60, {{t6}}
{window_addr("{WD0}", "{t6}")}
ds_read_b32 {{WD0}}, {{WD0}}
s_and_b64 {{T7}}, {{T7}}, exec
s_cbranch_scc0 .L{lab}_near%=
{WAIT}
s_mov_b64 {{T5}}, exec
s_mov_b64 exec, {{T7}}
v_and_b32 {{t10}}, -4, {{t0}}
v_mov_b32 {{t11}}, 0
v_lshl_add_u64 {{T89}}, {{BASE}}, 0, {{T1011}}
global_load_dword {{WD0}}, {{T89}}, off
s_waitcnt vmcnt(0)
s_mov_b64 exec, {{T5}}
.L{lab}_near%=:
v_and_b32 {{SHF}}, 3, {{t0}}
v_lshlrev_b32 {{SHF}}, 3, {{SHF}}
{WAIT}
v_bfe_u32 {{RL}}, {{WD0}}, {{SHF}}, 8
v_cmp_lt_u32 vcc, {{t0}}, {{LEN}}
v_cndmask_b32 {{RL}}, 0, {{RL}}, vcc
{on('SRC2,DST')}
v_bfi_b32 {{RF0}}, {{KML}}, {{RL}}, {{RF0}}
{OFF}
{TAILS[sfx]}"""
    return out


def window_tail_ldx(a0, shift):
    """As window_tail for a register-based address, whose bytes may also come from far_read.
    Bytes past len read as zero (main.rs:16): in the FIXED layout every packet is >= 64 bytes
    and a multiple of 16 long, so window bytes are packet bytes and far_read's whole-dword
    selection zeroes the rest of a read that starts inside the packet; a read that starts at or
    past len (whose registers still hold the window bytes at 0) is zeroed whole. Otherwise mask
    them byte by byte."""
    return f""".if %[fixed] == 0
v_sub_u32_e64 {{LENM}}, {{LEN}}, {a0}
v_cmp_lt_u32 vcc, {a0}, {{LEN}}
v_cndmask_b32 {{LENM}}, 0, {{LENM}}, vcc
v_min_u32 {{LENM}}, 8, {{LENM}}
v_lshlrev_b32 {{LENM}}, 3, {{LENM}}
v_sub_u32 {{LENM}}, 64, {{LENM}}
.endif
{WAIT}
v_alignbyte_b32 {{RL}}, {{WD1}}, {{WD0}}, {shift}
v_alignbyte_b32 {{RH}}, {{WD2}}, {{WD1}}, {shift}
.if %[fixed] == 0
v_and_b32 {{RL}}, {{KML}}, {{RL}}
v_and_b32 {{RH}}, {{KMH}}, {{RH}}
v_lshlrev_b64 {{R}}, {{LENM}}, {{R}}
v_lshrrev_b64 {{R}}, {{LENM}}, {{R}}
v_cndmask_b32 {{RL}}, 0, {{RL}}, vcc
v_cndmask_b32 {{RH}}, 0, {{RH}}, vcc
.else
v_cmp_lt_u32 vcc, {a0}, {{LEN}}
v_cndmask_b32 {{RL}}, 0, {{RL}}, vcc
v_cndmask_b32 {{RH}}, 0, {{RH}}, vcc
.endif
{on('SRC2,DST')}
v_bfi_b32 {{RF0}}, {{KML}}, {{RL}}, {{RF0}}
v_bfi_b32 {{RF1}}, {{KMH}}, {{RH}}, {{RF1}}
{OFF}"""


# bit-serial restoring division: T45 dividend, T67 divisor -> T01 quotient, T23 remainder;
# division by zero: DIV -> 0, MOD -> dividend (T1011) (emu.rs:90-100,126-135, Q5)
def divmod(sfx):
    return f""".Ldivmod{sfx}%=:
v_mov_b32 {{t0}}, 0
v_mov_b32 {{t1}}, 0
v_mov_b32 {{t2}}, 0
v_mov_b32 {{t3}}, 0
s_mov_b32 {{CNT}}, 64
.Ldivloop{sfx}%=:
v_lshlrev_b64 {{T23}}, 1, {{T23}}
v_lshrrev_b32 {{t8}}, 31, {{t5}}
v_or_b32 {{t2}}, {{t2}}, {{t8}}
v_lshlrev_b64 {{T45}}, 1, {{T45}}
v_lshlrev_b64 {{T01}}, 1, {{T01}}
v_cmp_ge_u64 vcc, {{T23}}, {{T67}}
v_sub_co_u32_e64 {{t8}}, {{T5}}, {{t2}}, {{t6}}
v_subb_co_u32_e64 {{t9}}, {{T5}}, {{t3}}, {{t7}}, {{T5}}
v_cndmask_b32 {{t2}}, {{t2}}, {{t8}}, vcc
v_cndmask_b32 {{t3}}, {{t3}}, {{t9}}, vcc
v_cndmask_b32_e64 {{t8}}, 0, 1, vcc
v_or_b32 {{t0}}, {{t0}}, {{t8}}
s_sub_u32 {{CNT}}, {{CNT}}, 1
s_cmp_lg_u32 {{CNT}}, 0
s_cbranch_scc1 .Ldivloop{sfx}%=
v_cmp_eq_u64 vcc, 0, {{T67}}
s_cmp_eq_u32 {{MODE}}, 0
s_cbranch_scc0 .Lmodres{sfx}%=
v_cndmask_b32_e64 {{RL}}, {{t0}}, 0, vcc
v_cndmask_b32_e64 {{RH}}, {{t1}}, 0, vcc
s_branch .Ldivend{sfx}%=
.Lmodres{sfx}%=:
v_cndmask_b32 {{RL}}, {{t2}}, {{t10}}, vcc
v_cndmask_b32 {{RH}}, {{t3}}, {{t11}}, vcc
.Ldivend{sfx}%=:
{WRITE_R}
{STEP}
{TAILS[sfx]}"""


TAILS = {"c": CHAIN, "e": END_N, "j": ""}

def fixed_dma(winb):
    """FIXED layout: DMA the header windows of tile T0 / 64 (T0 = tile << 6) into the LDS window
    buffer at `winb` (as dma_window_stride in interp.hip): round r moves packets 16r..16r+15, lane
    l filling chunk slot (l & 3) of packet 16r + l/4 from logical chunk (l & 3) ^ ((l >> 4) & 3);
    lanes past the batch read the micro-op table instead. Four global_load_lds_dwordx4 in flight
    afterwards; t0 (the lane) is kept."""
    return """v_lshrrev_b32 {t4}, 2, {t0}
v_mov_b32 {t5}, 0
v_lshl_add_u64 {T45}, {T45}, 0, {T0}
v_and_b32 {t6}, 3, {t0}
v_bfe_u32 {t7}, {t0}, 4, 2
v_xor_b32 {t6}, {t6}, {t7}
v_lshlrev_b32 {t6}, 4, {t6}
v_mov_b32 {t7}, 0
v_mov_b32 {t10}, {KSTL}
v_mad_u64_u32 {T89}, {T4}, {t4}, {t10}, {KFR}
v_mul_lo_u32 {t11}, {t5}, {KSTL}
v_mul_lo_u32 {t12}, {t4}, {KSTH}
v_add3_u32 {t9}, {t9}, {t11}, {t12}
v_lshl_add_u64 {T89}, {T89}, 0, {T67}
s_lshl_b64 {T1}, {KST}, 4
v_mov_b32 {t10}, {PROGL}
v_mov_b32 {t11}, {PROGH}
""" + "\n".join(f"""v_cmp_gt_u64 vcc, {{KN}}, {{T45}}
v_cndmask_b32 {{t12}}, {{t10}}, {{t8}}, vcc
v_cndmask_b32 {{t13}}, {{t11}}, {{t9}}, vcc
s_add_u32 m0, {winb}, {1024 * r}
s_nop 0
global_load_lds_dwordx4 {{T1213}}, off
v_lshl_add_u64 {{T45}}, {{T45}}, 0, 16
v_lshl_add_u64 {{T89}}, {{T89}}, 0, {{T1}}""" for r in range(4))


def fixed_dma_db(winb, tag):
    """As fixed_dma, for the double-buffered compiled kernel: a whole tile (the scalar check
    (T0 + 64 <= n), every tile but a batch's last) takes per-lane offsets from %[dmaoff] (lane l:
    (l/4) * stride + its swizzled chunk * 16, computed once per wave) and a scalar tile base --
    one VALU per round instead of five; a partial tile takes fixed_dma's per-lane checks.
    64-byte slots: one address and the four 1 KiB rows by the instruction offset, which the
    LDS-DMA adds to both the global and the LDS address. `; @DMAX@` / `; @DMAXE@` (jit.cpp
    window_chunks): exec = the lanes of the window chunks the compiled program reads, then all."""
    return f"""; @DMAX@
s_add_u32 {{T5L}}, {{T0L}}, 64
s_addc_u32 {{T5H}}, {{T0H}}, 0
s_sub_u32 {{T5L}}, {{KNL}}, {{T5L}}
s_subb_u32 {{T5H}}, {{KNH}}, {{T5H}}
s_cbranch_scc1 .Lpart{tag}%=
s_cmp_eq_u64 {{KST}}, 64
s_cbranch_scc0 .Lgen{tag}%=
s_lshl_b64 {{T7}}, {{T0}}, 6
s_add_u32 {{T7L}}, {{T7L}}, {{KFRL}}
s_addc_u32 {{T7H}}, {{T7H}}, {{KFRH}}
v_lshl_add_u64 {{T1213}}, %[dmaoff], 0, {{T7}}
s_mov_b32 m0, {winb}
s_nop 0
""" + "\n".join(f"global_load_lds_dwordx4 {{T1213}}, off offset:{1024 * r} ; @DMAPOLICY@"
                for r in range(4)) + f"""
s_branch .Ldmaok{tag}%=
.Lgen{tag}%=:
s_mul_i32 {{T7L}}, {{T0L}}, {{KSTL}}
s_mul_hi_u32 {{T7H}}, {{T0L}}, {{KSTL}}
s_mul_i32 {{T5L}}, {{T0L}}, {{KSTH}}
s_add_u32 {{T7H}}, {{T7H}}, {{T5L}}
s_mul_i32 {{T5L}}, {{T0H}}, {{KSTL}}
s_add_u32 {{T7H}}, {{T7H}}, {{T5L}}
s_add_u32 {{T7L}}, {{T7L}}, {{KFRL}}
s_addc_u32 {{T7H}}, {{T7H}}, {{KFRH}}
s_lshl_b64 {{T1}}, {{KST}}, 4
""" + "\n".join(f"""v_lshl_add_u64 {{T1213}}, %[dmaoff], 0, {{T7}}
s_add_u32 m0, {winb}, {1024 * r}
s_nop 0
global_load_lds_dwordx4 {{T1213}}, off ; @DMAPOLICY@
s_add_u32 {{T7L}}, {{T7L}}, {{T1L}}
s_addc_u32 {{T7H}}, {{T7H}}, {{T1H}}""" for r in range(4)) + f"""
s_branch .Ldmaok{tag}%=
.Lpart{tag}%=:
""" + fixed_dma(winb) + f"""
.Ldmaok{tag}%=:
; @DMAXE@"""


# ---- prologue / epilogue ----
# %[ka]: the kernel-argument segment (LaunchArgs at offset 0; LA_* offsets are "i" operands);
# %[tile]: the tile index (64-bit SGPR pair); %[winb]: this wave's window region (LDS byte
# address); %[metab]: this wave's metadata region (offsets u32[64], lengths u32[64]; with %[plen],
# the compiled forward var kernels, lengths u16[64]: interp.hip dma_meta<true>).
# the main.rs:28-31 register layout (r1 = 0, r2 = len, r10 = the batch's r10, the rest 0)
DEFAULT_INIT = "\n".join(f"v_mov_b64 v[{i}:{i + 1}], 0" for i in range(0, 20, 2) if i != 4) + """
v_mov_b32 v4, {LEN}
v_mov_b32 v5, 0
v_mov_b32 v20, {KR10L}
v_mov_b32 v21, {KR10H}
"""
# compiled programs: only the registers the program may read before writing them, and r0 (the
# compiler fills in ;@@JITINIT@@) -- all of them when the batch asks for the final registers
JIT_INIT = """s_load_dwordx2 {T5}, %[ka], %[o_regs]
s_waitcnt lgkmcnt(0)
s_cmp_lg_u64 {T5}, 0
s_cbranch_scc1 .Lallinit%=
;@@JITINIT@@
s_branch .Linitd%=
.Lallinit%=:
""" + DEFAULT_INIT
FIXED_DMA = """.if %[fixed]
""" + fixed_dma("%[winb]") + """
s_waitcnt vmcnt(0)
.endif
"""
PROLOGUE = """s_mov_b32 {M0S}, m0
s_mov_b64 {LIVE}, 0
s_load_dwordx2 {PROG}, %[ka], %[o_tprog]
s_load_dwordx2 {KFR}, %[ka], %[o_frames]
s_load_dwordx2 {KST}, %[ka], %[o_stride]
s_load_dwordx2 {KN}, %[ka], %[o_n]
s_load_dword {KMEM}, %[ka], %[o_mem]
.if %[fixed] == 0
s_load_dwordx2 {KOFF}, %[ka], %[o_offsets]
s_load_dwordx2 {KLEN}, %[ka], %[o_lens]
s_load_dword {T5L}, %[ka], %[o_xdp]
.endif
v_mbcnt_lo_u32_b32 {t0}, -1, 0
v_mbcnt_hi_u32_b32 {t0}, -1, {t0}
s_lshl_b64 {T0}, %[tile], 6
v_mov_b32 {t1}, 0
v_lshl_add_u64 {T23}, {T01}, 0, {T0}
.if %[fixed] == 0
v_lshlrev_b32 {t5}, 2, {t0}
v_add_u32 {t5}, %[metab], {t5}
ds_read_b32 {t6}, {t5}
.if %[plen]
v_lshlrev_b32 {t7}, 1, {t0}
v_add_u32 {t7}, %[metab], {t7}
ds_read_u16 {t7}, {t7} offset:256
.else
ds_read_b32 {t7}, {t5} offset:256
.endif
.endif
s_waitcnt lgkmcnt(0)
""" + FIXED_DMA + """v_cmp_gt_u64 vcc, {KN}, {T23}
s_and_b64 {VM}, vcc, exec
s_cmp_gt_u32 {KSTH}, 0
s_cselect_b32 {T3}, -1, {KSTL}
v_mov_b32 {LEN}, {T3}
v_mov_b32 {t4}, {KSTL}
v_mad_u64_u32 {BASE}, {T4}, {t2}, {t4}, {KFR}
v_mul_lo_u32 {t4}, {t3}, {KSTL}
v_mul_lo_u32 {t9}, {t2}, {KSTH}
v_add3_u32 {BASEH}, {BASEH}, {t4}, {t9}
.if %[fixed] == 0
s_cmp_lg_u64 {KOFF}, 0
s_cbranch_scc0 .Lnooff%=
v_mov_b32 {t8}, {t6}
v_mov_b32 {t9}, 0
v_lshl_add_u64 {BASE}, {KFR}, 0, {T89}
.Lnooff%=:
s_cmp_lg_u64 {KLEN}, 0
s_cbranch_scc0 .Lnolen%=
v_and_b32 {LEN}, 0xffff, {t7}
.Lnolen%=:
s_cmp_lg_u32 {T5L}, 0
s_cbranch_scc0 .Lnoxdp%=
v_min_u32 {LEN}, 0xffff, {LEN}
v_add_u32 {LEN}, 8, {LEN}
v_lshl_add_u64 {BASE}, {BASE}, 0, -8
.Lnoxdp%=:
.endif
v_cndmask_b32 {LEN}, 0, {LEN}, vcc
v_lshlrev_b32 {WIN}, 6, {t0}
v_add_u32 {WIN}, %[winb], {WIN}
v_lshrrev_b32 {SWZ}, 2, {t0}
v_and_b32 {SWZ}, 3, {SWZ}
v_lshlrev_b32 {SWZ}, 4, {SWZ}
.if %[loops]
s_load_dwordx2 {T5}, %[ka], %[o_maxs]
v_mov_b32 {WB}, 0
s_waitcnt lgkmcnt(0)
s_cmp_lg_u32 s67, 0
s_cselect_b32 {MAXS}, -1, s66
.endif
.Lreinit%=:
v_mov_b32 {NST}, 0
v_mov_b32 {ST}, 0
v_mov_b32 {LPC}, -1
v_cmp_lt_u32 {T0}, {KMEM}, {LEN}
s_and_b64 {T0}, {T0}, {VM}
s_andn2_b64 {T1}, {VM}, {T0}
s_mov_b64 exec, {T0}
v_mov_b32 {ST}, 7
s_mov_b64 exec, {T1}
v_mov_b32 {LPC}, 0
s_mov_b64 exec, {EXEC0}
s_cmp_lg_u64 {T1}, 0
s_cselect_b64 {T0}, 1, 0
s_or_b64 {LIVE}, {LIVE}, {T0}
s_bitset1_b64 {LIVE}, 63
s_load_dwordx2 {KINIT}, %[ka], %[o_init]
s_load_dwordx2 {KR10}, %[ka], %[o_r10]
s_waitcnt lgkmcnt(0)
s_cmp_lg_u64 {KINIT}, 0
s_cbranch_scc1 .Linitc%=
""" + DEFAULT_INIT + """s_branch .Linitd%=
.Linitc%=:
s_mov_b64 {T5}, {KINIT}
s_load_dwordx16 {UOP}, {T5}, 0x0
s_waitcnt lgkmcnt(0)
""" + "\n".join(f"v_mov_b32 v{i}, s{UB + i}" for i in range(16)) + """
s_load_dwordx4 s[36:39], {T5}, 0x40
s_load_dwordx2 s[40:41], {T5}, 0x50
s_waitcnt lgkmcnt(0)
""" + "\n".join(f"v_mov_b32 v{16 + i}, s{UB + i}" for i in range(6)) + """
.Linitd%=:
"""
# the interpreter's dispatch entry: handler slots follow the statement's prologue
SLOTS_HEAD = """s_getpc_b64 {SLOTB}
.Lpc%=:
s_add_u32 {SLOTBL}, {SLOTBL}, .Lslots%=-.Lpc%=
s_addc_u32 {SLOTBH}, {SLOTBH}, 0
""" + DISPATCH + """
.p2align 8
.Lslots%=:"""

# bucket: 0..4 r0, 5 r0 >= 5, 6 fault, 7 not a packet, 8 deoptimized (status 0x80, jit.h kStDeopt:
# a compiled store-mode lane that left for the general interpreter -- no outputs, no steps, its
# packet listed by the C++ after the statement); stores of the valid lanes
EPILOGUE = """.Ldone%=:
s_mov_b64 exec, {EXEC0}
v_cmp_gt_u64 vcc, 5, {RF}
v_cndmask_b32 %[bkt], 5, {RF0}, vcc
v_cmp_ne_u32 vcc, 0, {ST}
v_cndmask_b32_e64 %[bkt], %[bkt], 6, vcc
v_cndmask_b32_e64 %[bkt], 7, %[bkt], {VM}
v_cndmask_b32_e64 %[nst], 0, {NST}, {VM}
v_cmp_eq_u32 vcc, 0x80, {ST}
s_and_b64 vcc, vcc, {VM}
v_cndmask_b32_e64 %[bkt], %[bkt], 8, vcc
v_cndmask_b32_e64 %[nst], %[nst], 0, vcc
s_andn2_b64 {VM}, {VM}, vcc
s_mov_b64 exec, {VM}
s_cmp_lg_u64 exec, 0
s_cbranch_scc0 .Lend%=
v_mbcnt_lo_u32_b32 {t0}, -1, 0
v_mbcnt_hi_u32_b32 {t0}, -1, {t0}
s_lshl_b64 {T0}, %[tile], 6
v_mov_b32 {t1}, 0
v_lshl_add_u64 {T23}, {T01}, 0, {T0}
.if %[loops]
s_load_dwordx2 {T1}, %[ka], %[o_perm]
s_waitcnt lgkmcnt(0)
s_cmp_lg_u64 {T1}, 0
s_cbranch_scc0 .Lnoperm%=
v_lshlrev_b64 {T45}, 2, {T23}
v_lshl_add_u64 {T45}, {T45}, 0, {T1}
global_load_dword {t2}, {T45}, off
v_mov_b32 {t3}, 0
s_waitcnt vmcnt(0)
.Lnoperm%=:
.endif
s_load_dwordx2 {EV}, %[ka], %[o_verdict]
s_load_dwordx2 {ER0}, %[ka], %[o_r0]
s_load_dwordx2 {EST}, %[ka], %[o_status]
s_load_dwordx2 {ERG}, %[ka], %[o_regs]
s_waitcnt lgkmcnt(0)
s_cmp_lg_u64 {EV}, 0
s_cbranch_scc0 .Lnov%=
v_cmp_gt_u32 vcc, 5, %[bkt]
v_mov_b32 {t5}, 0xfe
v_cndmask_b32 {t4}, {t5}, {RF0}, vcc
v_cmp_ne_u32 vcc, 6, %[bkt]
v_mov_b32 {t5}, 0xff
v_cndmask_b32 {t4}, {t5}, {t4}, vcc
v_lshl_add_u64 {T67}, {T23}, 0, {EV}
global_store_byte {T67}, {t4}, off
.Lnov%=:
s_cmp_lg_u64 {ER0}, 0
s_cbranch_scc0 .Lnor%=
v_lshlrev_b64 {T67}, 3, {T23}
v_lshl_add_u64 {T67}, {T67}, 0, {ER0}
global_store_dwordx2 {T67}, {RF}, off
.Lnor%=:
s_cmp_lg_u64 {EST}, 0
s_cbranch_scc0 .Lnos%=
v_lshl_add_u64 {T67}, {T23}, 0, {EST}
global_store_byte {T67}, {ST}, off
.Lnos%=:
s_cmp_lg_u64 {ERG}, 0
s_cbranch_scc0 .Lend%=
v_mov_b32 {t6}, 88
v_mad_u64_u32 {T89}, {T4}, {t2}, {t6}, {ERG}
v_mul_lo_u32 {t6}, {t3}, {t6}
v_add_u32 {t9}, {t9}, {t6}
""" + "\n".join(f"global_store_dwordx2 {{T89}}, v[{2 * r}:{2 * r + 1}], off offset:{8 * r}"
                for r in range(11)) + """
.Lend%=:
s_mov_b64 exec, {EXEC0}
s_mov_b32 m0, {M0S}"""


# ---- JIT templates (jit.cpp): the same handler bodies, compiled per program ----
# A compiled program is straight-line code over its micro-ops in pc order (forward jumps only):
# exec holds the lanes running the current basic block; lanes that jump park at the target with
# LPC = target, and each jump target's entry adds them back (LPC == pc), so the lowest pc runs
# first exactly as in the interpreter's min-pc dispatch. The handler bodies are those above with
#   * every s_set_gpr_idx region rewritten to direct register operands: @D<k>@ / @D<a>:<b>@ (dst
#     register pair 2*dst + k) and @S..@ (src), filled in by the compiler per micro-op;
#   * the micro-op's fields (s37..s51, TUop dwords 1..15) as tokens @K<d>@ / @K<a>:<b>@: inline
#     constants where the value is one, else an s_mov into the same SGPR before the micro-op;
#   * labels unique per micro-op (@U@), the dispatcher replaced by the next block entry (@NEXT@),
#     and tails by @JTAIL@ (conditional jump), @JA@, @EXIT@.
GPRIDX_OF = {M["DST2"]: "D", M["SRC2"]: "S"}


def _direct_operands(line, idx, roles):
    """One VALU line of an s_set_gpr_idx region: the VGPR operands in the enabled roles get the
    index (VGPR index mode adds it to those operands only, never to SGPR or constant ones)."""
    mn, rest = line.split(None, 1)
    ops = [o.strip() for o in rest.split(",")]
    if mn.startswith("v_cmp"):
        slots = ["SDST", "SRC0", "SRC1"]
    elif "_co_" in mn:
        slots = ["DST", "SDST", "SRC0", "SRC1", "SRC2"]
    else:
        slots = ["DST", "SRC0", "SRC1", "SRC2"]
    assert len(ops) <= len(slots), line
    out = []
    for slot, o in zip(slots, ops):
        if slot in roles:
            m1 = re.fullmatch(r"v(\d+)", o)
            m2 = re.fullmatch(r"v\[(\d+):(\d+)\]", o)
            if m1:
                o = f"@{idx}{m1.group(1)}@"
            elif m2:
                o = f"@{idx}{m2.group(1)}:{m2.group(2)}@"
        out.append(o)
    return f"{mn} " + ", ".join(out)


def jit_text(raw):
    """A handler body (register names substituted) -> JIT template text."""
    out, mode = [], None
    for line in raw.split("\n"):
        m = re.match(r"s_set_gpr_idx_on (\S+), gpr_idx\(([A-Z0-9,]+)\)$", line.strip())
        if m:
            mode = (GPRIDX_OF[m.group(1)], set(m.group(2).split(",")))
            continue
        if line.strip() == "s_set_gpr_idx_off":
            mode = None
            continue
        if mode and line.startswith("v_"):
            line = _direct_operands(line, *mode)
        out.append(line)
    assert mode is None
    t = "\n".join(out)
    t = t.replace(".Ldisp%=", "@NEXT@").replace(".Lkfault%=", ".Lkf@U@")
    t = re.sub(r"\.L(\w+)%=", r".L\1@U@", t)
    assert "%=" not in t, t

    def field(m):
        a = int(m.group(1)) - UB
        if m.group(2) is None:
            return f"@K{a}@" if 1 <= a <= 15 else m.group(0)
        b = int(m.group(2)) - UB
        return f"@K{a}:{b}@" if 1 <= a and b <= 15 else m.group(0)
    t = re.sub(r"\bs\[(\d+):(\d+)\]", lambda m: field(m) if int(m.group(1)) >= UB else m.group(0), t)
    t = re.sub(r"\bs(\d+)\b", lambda m: (f"@K{int(m.group(1)) - UB}@"
                                         if UB + 1 <= int(m.group(1)) <= UB + 15 else m.group(0)), t)
    assert "s_set_gpr_idx" not in t and "s_setpc" not in t and "s_load_dwordx16" not in t, t
    return t


# a constant-address load outside the image: every active lane faults alike (KFAULT above)
KFAULT_JIT = f""".Lkf@U@:
s_cmp_ge_u32 {{A0}}, {{KMEM}}
s_cselect_b32 {{T3}}, {ST_MEM}, {ST_MEM_UB}
v_mov_b32 {{ST}}, {{T3}}
v_subrev_u32 {{NST}}, {{REMK}}, {{NST}}
@EXIT@
s_branch @NEXT@"""

JIT_TERM = {
    "H_EXIT": "@EXIT@",
    "H_JA": "@JA@",
    "H_FAULT": "v_mov_b32 {ST}, {IMML}\nv_subrev_u32 {NST}, 1, {NST}\n@EXIT@",
    "H_SLOW": f"v_mov_b32 {{ST}}, {ST_INSN}\nv_subrev_u32 {{NST}}, 1, {{NST}}\n@EXIT@",
}
JIT_OOL = {"ldxk": ldxk, "ldxk1": ldxk1, "ldxk2": ldxk2, "ldxkfar": ldxkfar, "ldx": ldx}


def jit_template(base):
    """(main, out-of-line) JIT template text of handler `base`."""
    if base == DONE:
        return "", ""
    body, kind = H[base]
    if kind == "term":
        raw = JIT_TERM[base]
    elif kind == "jump":
        raw = body + "\n@JTAIL@"
    elif kind == "alu":
        raw = body
    elif kind == "div":
        raw = body + "\n" + divmod("j")
    elif body == "ldx1":  # loop programs: the refillable-window forms
        raw = ".if %[loops]\n" + ldx1("j", True) + "\n.else\n" + ldx1("j", False) + "\n.endif"
    elif body == "ldx":
        raw = ".if %[loops]\n" + ldx_loop("j") + "\n.else\n" + ldx("j") + "\n.endif"
    else:
        raw = JIT_OOL[body]("j")
    main = jit_text(F(raw))
    ool = jit_text(F(KFAULT_JIT)) if ".Lkf@U@" in main else ""
    return main, ool


def cstr(text):
    return "\n".join('"' + ln.replace("\\", "\\\\").replace('"', '\\"') + '\\n"'
                     for ln in text.splitlines()) or '""'


# The template kernel's statement (ebpf_tile_jit_var, every layout but the fixed-slot one): the
# prologue, a marker the compiler fills in at load time, the epilogue. The marker line carries the
# statement's label number and operand registers.
# (s70: loop programs' exact-mode flag, set by the compiled code's step-budget restart)
# s70 bit 1: the registers are not the main.rs layout (init_regs) or are outputs (regs) -- the
# compiled loop programs' proven copy (jit.cpp prove_loads) assumes the layout and dead registers
JIT_STATEMENT = ("s_mov_b32 s70, 0\n" + PROLOGUE.replace(DEFAULT_INIT, JIT_INIT) + """
; JIT N=%= fixed=%[fixed] loops=%[loops] aligned=%[aligned]
;@@JIT@@
""" + EPILOGUE).replace(".Lallinit%=:\n", ".Lallinit%=:\ns_or_b32 s70, s70, 2\n").replace(
    ".Linitc%=:\n", ".Linitc%=:\ns_or_b32 s70, s70, 2\n")


# ---- the compiled fixed-slot kernel's tile loop (ebpf_tile_jit_fixed) ----
# One statement runs up to %[cdn] (511) of the wave's tiles back to back, so nothing of the
# C++ around it is paid per tile (PMC: the per-tile statement above cost 241 instructions per
# tile of 64 packets for a 3-instruction program, 116 of them SALU). Per tile:
#   * the next ordinal of the workgroup's LDS counter, fetched one tile ahead (%[ordv]), gives
#     the wave's next tile nt = wg + (ordinal + 16) * grid; its four window DMAs go to the other
#     buffer (%[nwinb]) before this tile runs;
#   * this tile's lanes: packet address = tile base + lane * stride, LDS window, registers;
#   * the compiled program;
#   * the verdict byte, and the lane's counter bucket as one add to a packed per-lane word
#     (%[acc]: seven 9-bit fields, bucket b at bit 9b; <= 511 tiles per statement), retired steps
#     added per lane (%[ret]) -- the C++ after the statement unpacks and sums them per wave.
# Tiles wholly inside the batch in 64-byte slots take the inline DMA (%[nfast]: the tiles below
# it); the batch's last partial tile and other slot sizes take fixed_dma_db out of line.
# Loop state lives in the C++ operands (SGPRs / VGPRs outside the statement's v[0:95] and
# s[33:71], which the program's code owns).
def loop_dma(tidx, winb, tag):
    """DMA tile `tidx` (an SGPR holding the tile index) into the window buffer `winb`. Returns
    (inline text, out-of-line text)."""
    main = f"""s_cmp_lt_u32 {tidx}, %[nfast]
s_cbranch_scc0 .Lx{tag}%=
s_mul_i32 {{T7L}}, {tidx}, %[tbytes]
s_mul_hi_u32 {{T7H}}, {tidx}, %[tbytes]
s_add_u32 {{T7L}}, {{T7L}}, %[fr_lo]
s_addc_u32 {{T7H}}, {{T7H}}, %[fr_hi]
v_lshl_add_u64 {{T1213}}, %[dmaoff], 0, {{T7}}
; @DMAX@
s_mov_b32 m0, {winb}
s_nop 0
""" + "\n".join(f"global_load_lds_dwordx4 {{T1213}}, off offset:{1024 * r} ; @DMAPOLICY@"
                for r in range(4)) + f"""
; @DMAXE@
.Ld{tag}%=:
"""
    ool = f""".Lx{tag}%=:
s_mov_b64 {{KFR}}, %[k_frames]
s_mov_b64 {{KST}}, %[k_stride]
s_mov_b64 {{KN}}, %[k_n]
s_mov_b64 {{PROG}}, %[k_tprog]
s_mov_b32 {{T0L}}, {tidx}
s_mov_b32 {{T0H}}, 0
s_lshl_b64 {{T0}}, {{T0}}, 6
v_mbcnt_lo_u32_b32 {{t0}}, -1, 0
v_mbcnt_hi_u32_b32 {{t0}}, -1, {{t0}}
""" + fixed_dma_db(winb, "y" + tag) + f"""
s_branch .Ld{tag}%=
"""
    return main, ool


# The fixed-slot statement's store mode (marker st=1, jit.cpp body_store): lanes that left for the
# general interpreter (status 0x80, jit.h kStDeopt) produce nothing here; their packet indices go
# to the deopt list (one returning atomic per wave) -- or, with no pass to follow (%[dfl] bit 1,
# StackPlan::no_deopt), they fault EBPF_ST_JIT. Other programs: one compare and branch per tile.
STORE_DEOPT_FIXED = """s_mov_b64 exec, {VM}
v_cmp_eq_u32 vcc, 0x80, {ST}
s_cbranch_vccz .Lnodo%=
s_bitcmp1_b32 %[dfl], 1
s_cbranch_scc1 .Ldofail%=
s_andn2_b64 {VM}, {VM}, vcc
s_mov_b64 {T0}, vcc
s_mov_b64 exec, vcc
v_mbcnt_lo_u32_b32 {t5}, {T0L}, 0
v_mbcnt_hi_u32_b32 {t5}, {T0H}, {t5}
s_bcnt1_i32_b64 {T3}, {T0}
s_ff1_i32_b64 {T1L}, {T0}
s_lshl_b64 {T1}, 1, {T1L}
s_mov_b64 exec, {T1}
v_mov_b32 {t6}, {T3}
v_mov_b64 {T89}, %[k_deopt]
global_atomic_add {t4}, {T89}, {t6}, off sc0
s_waitcnt vmcnt(0)
v_readfirstlane_b32 {T3}, {t4}
s_mov_b64 exec, {T0}
v_add_u32 {t10}, {T3}, {t5}
v_mov_b32 {t11}, 0
v_lshlrev_b64 {T1011}, 2, {T1011}
v_lshl_add_u64 {T89}, {T1011}, 0, %[k_dix]
s_lshl_b32 {T1L}, %[tile], 6
v_mbcnt_lo_u32_b32 {t4}, -1, 0
v_mbcnt_hi_u32_b32 {t4}, -1, {t4}
v_add_u32 {t4}, {T1L}, {t4}
global_store_dword {T89}, {t4}, off
s_branch .Lnodo%=
.Ldofail%=:
s_mov_b64 exec, vcc
v_mov_b32 {ST}, 8
.Lnodo%=:
"""


def jit_statement_loop(single=False):
    """single: the occupancy variant (ebpf_tile_jit_fixed_occ) -- one window buffer per wave, so
    the next tile is claimed and its windows DMA'd only once this tile's code is done with the
    buffer; the other waves of the SIMD (6 instead of 4) hide that DMA."""
    dma_f, ool_f = loop_dma("{T3}", "%[winb]", "f")
    dma_n, ool_n = loop_dma("%[ntile]", "%[nwinb]", "n")
    if single:
        dma_n, ool_n = loop_dma("{T3}", "%[winb]", "g")
    # the r0 / status / register outputs (%[oflags]): EPILOGUE's stores with T23 = packet index
    out_tail = EPILOGUE[EPILOGUE.index("s_cmp_lg_u64 {ER0}, 0"):EPILOGUE.index(".Lend%=:")]
    out_tail = out_tail.replace(".Lend%=", ".Loutd%=") + "s_branch .Loutd%="
    main = """s_mov_b32 {M0S}, m0
s_cmp_eq_u32 %[first], 0
s_cbranch_scc1 .Lent%=
; the wave's first tile: its windows
s_mov_b32 {T3}, %[tile]
""" + dma_f + """.Lent%=:
s_movk_i32 %[cdn], 511
.Lloop%=:
""" + ("""; this tile's windows (one buffer: DMA'd at the end of the tile before)
s_waitcnt vmcnt(0)
""" if single else """; the next tile: nt = wg + (ordinal + waves) * grid, DMA'd into the other buffer
s_mov_b64 exec, 1
ds_add_rtn_u32 %[ordv], %[nxa], %[one]
s_waitcnt lgkmcnt(0)
s_mov_b64 exec, -1
v_readfirstlane_b32 {T3}, %[ordv]
s_add_u32 {T3}, {T3}, %[wpb]
s_mul_i32 {T3}, {T3}, %[grid]
s_add_u32 %[ntile], {T3}, %[wg]
s_cmp_lt_u32 %[ntile], %[ntiles]
s_cbranch_scc0 .Lnonext%=
""" + dma_n + """s_waitcnt vmcnt(4)
s_branch .Ldmad%=
.Lnonext%=:
s_waitcnt vmcnt(0)
.Ldmad%=:
""") + """; this tile's lanes (fixed slots: every lane of a whole tile is a packet of length %[lenc])
s_mov_b32 {KMEM}, %[k_mem]
s_mov_b64 {KR10}, %[k_r10]
s_mov_b64 {VM}, -1
s_mul_i32 {T0L}, %[tile], %[tbytes]
s_mul_hi_u32 {T0H}, %[tile], %[tbytes]
s_add_u32 {T0L}, {T0L}, %[fr_lo]
s_addc_u32 {T0H}, {T0H}, %[fr_hi]
v_lshl_add_u64 {BASE}, %[laneoff], 0, {T0}
v_mov_b32 {LEN}, %[lenc]
v_add_u32 {WIN}, %[winb], %[lane64]
v_mov_b32 {SWZ}, %[swz]
v_mov_b32 {NST}, 0
v_mov_b32 {ST}, 0
v_mov_b32 {LPC}, 0
s_cmp_lt_u32 %[tile], %[nfull]
s_cbranch_scc0 .Lvm%=
.Lvmd%=:
s_cmp_gt_u32 %[lenc], %[k_mem]
s_cbranch_scc1 .Lbad%=
.Lbadd%=:
s_cmp_lg_u32 %[initx], 0
s_cbranch_scc1 .Linitx%=
;@@JITINIT@@
.Linitd%=:

; JIT N=%= fixed=%[fixed] loops=%[loops] aligned=%[aligned] xdp=%[xdpf] pm=1""" + (
        " occ=1 waves=%[wpb]" if single else " st=1 ovf=%[k_ovf] tile=%[tile] dm=s[78:79]") + """
;@@JIT@@
.Ldone%=:
""" + ("" if single else STORE_DEOPT_FIXED) + """; verdict byte, the lane's counter bucket (verdict 0..4, 0xfe -> 5, 0xff -> 6) into %[acc]
s_mov_b64 exec, {VM}
v_cmp_gt_u64 vcc, 5, {RF}
v_mov_b32 {t5}, 0xfe
v_cndmask_b32 {t4}, {t5}, {RF0}, vcc
v_cmp_eq_u32 vcc, 0, {ST}
v_mov_b32 {t5}, 0xff
v_cndmask_b32 {t4}, {t5}, {t4}, vcc
v_subrev_u32 {t5}, 0xf9, {t4}
v_min_u32 {t5}, {t4}, {t5}
v_mul_u32_u24 {t5}, 9, {t5}
v_lshlrev_b64 {T67}, {t5}, 1
v_lshl_add_u64 %[acc], %[acc], 0, {T67}
v_add_u32 %[ret], %[ret], {NST}
s_cmp_lg_u64 %[k_verdict], 0
s_cbranch_scc0 .Lnov%=
s_lshl_b32 {T0L}, %[tile], 6
s_lshr_b32 {T0H}, %[tile], 26
s_add_u32 {T0L}, {T0L}, %[vd_lo]
s_addc_u32 {T0H}, {T0H}, %[vd_hi]
v_lshl_add_u64 {T67}, %[lanep], 0, {T0}
global_store_byte {T67}, {t4}, off
.Lnov%=:
s_cmp_lg_u32 %[oflags], 0
s_cbranch_scc1 .Lout%=
.Loutd%=:
s_mov_b64 exec, -1
s_sub_u32 %[cdn], %[cdn], 1
""" + ("""; the next tile into the one buffer (every LDS read of this tile has returned: the wait below)
s_mov_b64 exec, 1
ds_add_rtn_u32 %[ordv], %[nxa], %[one]
s_waitcnt lgkmcnt(0)
s_mov_b64 exec, -1
v_readfirstlane_b32 {T3}, %[ordv]
s_add_u32 {T3}, {T3}, %[wpb]
s_mul_i32 {T3}, {T3}, %[grid]
s_add_u32 %[ntile], {T3}, %[wg]
s_cmp_lt_u32 %[ntile], %[ntiles]
s_cbranch_scc0 .Lfin%=
s_mov_b32 %[tile], %[ntile]
s_mov_b32 {T3}, %[ntile]
""" + dma_n if single else """s_cmp_lt_u32 %[ntile], %[ntiles]
s_cbranch_scc0 .Lfin%=
s_mov_b32 %[tile], %[ntile]
s_xor_b32 %[winb], %[winb], %[wx]
s_xor_b32 %[nwinb], %[nwinb], %[wx]
""") + """s_cmp_eq_u32 %[cdn], 0
s_cbranch_scc0 .Lloop%=
s_branch .Lexit%=
.Lfin%=:
s_mov_b32 %[tile], %[ntiles]
.Lexit%=:
s_waitcnt lgkmcnt(0)
s_mov_b32 m0, {M0S}
s_branch .Lend%=
"""
    # out of line: partial tile lanes, ST_BADPKT, init_regs / every register, the rare outputs
    ool = ool_f + ool_n + """.Lvm%=:
v_mbcnt_lo_u32_b32 {t0}, -1, 0
v_mbcnt_hi_u32_b32 {t0}, -1, {t0}
s_mov_b32 {T1L}, %[tile]
s_mov_b32 {T1H}, 0
s_lshl_b64 {T1}, {T1}, 6
v_mov_b32 {t1}, 0
v_lshl_add_u64 {T23}, {T01}, 0, {T1}
v_cmp_gt_u64 vcc, %[k_n], {T23}
s_mov_b64 {VM}, vcc
s_not_b64 exec, vcc
v_mov_b32 {LPC}, -1
v_mov_b32 {LEN}, 0
s_mov_b64 exec, -1
s_branch .Lvmd%=
.Lbad%=:
s_mov_b64 exec, {VM}
v_mov_b32 {ST}, 7
v_mov_b32 {LPC}, -1
s_mov_b64 exec, -1
s_branch .Lbadd%=
.Linitx%=:
s_bitcmp1_b32 %[k_flags], 0
s_cbranch_scc1 .Linitc%=
""" + DEFAULT_INIT + """s_branch .Linitd%=
.Linitc%=:
s_load_dwordx2 {T5}, %[ka], %[o_init]
s_waitcnt lgkmcnt(0)
s_load_dwordx16 {UOP}, {T5}, 0x0
s_waitcnt lgkmcnt(0)
""" + "\n".join(f"v_mov_b32 v{i}, s{UB + i}" for i in range(16)) + """
s_load_dwordx4 s[36:39], {T5}, 0x40
s_load_dwordx2 s[40:41], {T5}, 0x50
s_waitcnt lgkmcnt(0)
""" + "\n".join(f"v_mov_b32 v{16 + i}, s{UB + i}" for i in range(6)) + """
s_branch .Linitd%=
.Lout%=:
s_mov_b32 {T1L}, %[tile]
s_mov_b32 {T1H}, 0
s_lshl_b64 {T1}, {T1}, 6
v_lshl_add_u64 {T23}, %[lanep], 0, {T1}
s_load_dwordx2 {ER0}, %[ka], %[o_r0]
s_load_dwordx2 {EST}, %[ka], %[o_status]
s_load_dwordx2 {ERG}, %[ka], %[o_regs]
s_waitcnt lgkmcnt(0)
""" + out_tail + """
.Lend%=:
"""
    return main + ool


# ---- the compiled var kernel's tile loop (ebpf_tile_jit_varl) ----
# offsets + lens batches (a capture's or a NIC ring's layout) whose length array is 4-byte aligned
# (or absent). One statement runs up to %[cdn] (511) of the wave's tiles (tile, tile + W, ...: W =
# the grid's waves) as the fixed-slot kernel's loop does, with two window buffers and two metadata
# buffers per wave (interp.hip kVarlWaveLds: offsets u32[64], then the lengths as u16[64]). On
# entry and at the top of every tile the tile's windows (DMA'd or staged by the C++) and the next
# tile's metadata are in flight or landed; per tile:
#   * wait; this lane's offset / length from the metadata (BASE, LEN, xdp_md: BASE - 8, 8 + len);
#   * the next tile nt = tile + W: a whole tile whose packets are all 16-byte aligned (lanes of
#     length 0 excepted) has its four window DMAs issued into the other window buffer (packet
#     16r + l/4's chunk (l & 3) ^ ((l >> 4) & 3), chunks wholly past the packet from a dummy
#     address); any other tile -- misaligned packets, the batch's partial last tile -- ends the
#     statement after this one (%[stage] = 1): the C++ stages its windows lane by lane and comes
#     back;
#   * the metadata of nt + W (a whole tile) into this tile's metadata buffer, read above;
#   * the compiled program, the verdict byte and the packed counter bucket as the fixed-slot loop.
# The program's code is the var flavour with the preloaded window (jit.cpp body, marker varl=1):
# window loads from v[64:79], bytes at or past LEN zero.
def jit_statement_varl():
    out_tail = EPILOGUE[EPILOGUE.index("s_cmp_lg_u64 {ER0}, 0"):EPILOGUE.index(".Lend%=:")]
    out_tail = out_tail.replace(".Lend%=", ".Loutd%=") + "s_branch .Loutd%="
    # round r: packet 16r + l/4's offset (in the low word of the address pair) + frames + the
    # lane's chunk (%[fc]); the lanes whose chunk starts before the packet's end (mask in
    # MASKS[r]) issue the DMA -- the others leave their slot stale: bytes at or past LEN are
    # masked wherever the program reads them
    masks = ["{T0}", "{T1}", "{T4}", "{T5}"]
    rounds = "\n".join(f"""v_mov_b32 {{t{13 + 2 * r}}}, 0
v_lshl_add_u64 {{T{12 + 2 * r}{13 + 2 * r}}}, {{T{12 + 2 * r}{13 + 2 * r}}}, 0, %[fc]
v_cmp_lt_u32_e64 {masks[r]}, %[c16], {{t{8 + r}}}""" for r in range(4))
    srounds = "\n".join(f"""v_lshl_add_u64 {{T{12 + 2 * r}{13 + 2 * r}}}, %[db], 0, {{T7}}
s_add_u32 {{T7L}}, {{T7L}}, %[s16]
s_addc_u32 {{T7H}}, {{T7H}}, 0""" for r in range(4))
    smasks = "\n".join(f"v_cmp_lt_u32_e64 {masks[r]}, %[c16], {{t{8 + r}}}" for r in range(4))
    # a tile whose packets are not all 16-byte aligned (a capture's records: 24 + 16 + sum of the
    # earlier records) is DMA'd straight from the packets: round r's lane moves packet bytes
    # [16c, 16c + 16) from packet + 16c, whatever its alignment (the LDS side of the DMA is the
    # lane's slot either way: tools/probe_dma_align.hip). Nothing may be read past the 16-byte block
    # that holds the packet's last byte (the page the next block lies in may not be mapped), so a
    # lane whose chunk would reach past it -- the last chunk of a packet shorter than the window,
    # when 16c + 16 + m > ceil16(m + len), m = packet & 15 -- moves the aligned block below
    # instead, (packet + 16c) & ~15, whose bytes hold the chunk's packet bytes m bytes higher; at
    # the tile's top those lanes shift that one slot down by m in LDS (tailfix).
    trounds = "\n".join(f"""v_add_u32 {{t1}}, %[fr_lo], {{t{12 + 2 * r}}}
v_and_b32 {{t1}}, 15, {{t1}}
v_add3_u32 {{t2}}, {{t1}}, {{t{8 + r}}}, 15
v_and_b32 {{t2}}, -16, {{t2}}
v_add3_u32 {{t3}}, %[c16], {{t1}}, 16
v_cmp_gt_u32 vcc, {{t3}}, {{t2}}""" + "\n" + rounds.split("\n")[3 * r] + "\n" +
        rounds.split("\n")[3 * r + 1] + "\n" + rounds.split("\n")[3 * r + 2] + f"""
v_and_b32 {{t2}}, -16, {{t{12 + 2 * r}}}
v_cndmask_b32 {{t{12 + 2 * r}}}, {{t{12 + 2 * r}}}, {{t2}}, vcc""" for r in range(4))
    # the tail lanes of a tile DMA'd from unaligned packets (above): chunk c = (len - 1) >> 4 of a
    # packet of 1..64 bytes whose 16c + 16 + m > ceil16(m + len); dword j of the slot becomes
    # bytes [4j + m, 4j + m + 4) of it (bytes at or past 16 - m are past the packet: masked)
    d = [f"v{36 + k}" for k in range(5)]
    sel = "\n".join(
        "\n".join(f"v_cndmask_b32_e64 {d[k]}, {d[k]}, {d[k + i]}, {m}"
                   for i, m in ((1, "{T1}"), (2, "{T4}"), (3, "{T5}")) if k + i < 5)
        for k in range(4))
    tailfix = f"""; this tile was DMA'd from unaligned packets: its tail lanes' last slot down by m bytes
s_bitcmp1_b32 %[mis], 0
s_cbranch_scc0 .Lrad%=
v_and_b32 {{t16}}, 15, {{BASEL}}
v_add3_u32 {{t17}}, {{t16}}, {{LEN}}, 15
v_and_b32 {{t17}}, -16, {{t17}}
v_add_u32 {{t18}}, -1, {{LEN}}
v_and_b32 {{t18}}, -16, {{t18}}
v_add3_u32 {{t19}}, {{t18}}, {{t16}}, 16
v_cmp_gt_u32_e64 {{T4}}, {{t19}}, {{t17}}
v_cmp_ne_u32_e64 {{T1}}, 0, {{LEN}}
s_and_b64 {{T4}}, {{T4}}, {{T1}}
v_cmp_ge_u32_e64 {{T1}}, 64, {{LEN}}
s_and_b64 {{T4}}, {{T4}}, {{T1}}
s_and_b64 {{T4}}, {{T4}}, {{VM}}
s_cbranch_scc0 .Lrad%=
s_mov_b64 exec, {{T4}}
v_add_u32 {{t17}}, %[winb], %[lane64]
v_xad_u32 {{t18}}, %[swz], {{t18}}, {{t17}}
ds_read_b128 v[36:39], {{t18}}
v_mov_b32 v40, 0
v_lshrrev_b32 {{t19}}, 2, {{t16}}
v_cmp_eq_u32_e64 {{T1}}, 1, {{t19}}
v_cmp_eq_u32_e64 {{T4}}, 2, {{t19}}
v_cmp_eq_u32_e64 {{T5}}, 3, {{t19}}
s_waitcnt lgkmcnt(0)
{sel}
""" + "\n".join(f"v_alignbyte_b32 {d[j]}, {d[j + 1]}, {d[j]}, {{t16}}" for j in range(4)) + f"""
ds_write_b128 {{t18}}, v[36:39]
s_mov_b64 exec, -1
s_mov_b64 vcc, {{VM}}
.Lrad%=:"""
    dmas = "\n".join(f"""s_mov_b64 exec, {masks[r]}
s_add_u32 m0, %[nwinb], {1024 * r}
s_nop 0
global_load_lds_dwordx4 {{T{12 + 2 * r}{13 + 2 * r}}}, off ; @DMAPOLICY@""" for r in range(4)) + \
        "\ns_mov_b64 exec, -1"
    main = """s_mov_b32 {M0S}, m0
s_movk_i32 %[cdn], 511
s_mov_b32 %[stage], 0
.Lloop%=:
; this tile's windows and the next tile's metadata: landed
s_waitcnt vmcnt(0)
v_add_u32 {t0}, %[metab], %[lane4]
ds_read_b32 {t6}, {t0}
s_bitcmp1_b32 %[fl], 6
s_cbranch_scc0 .Lnl%=
v_add_u32 {t1}, %[metab], %[lane2]
ds_read_u16 {t7}, {t1}
s_branch .Lnld%=
.Lnl%=:
v_mov_b32 {t7}, %[lenc]
.Lnld%=:
s_mov_b32 {T1L}, %[tile]
s_mov_b32 {T1H}, 0
s_lshl_b64 {T1}, {T1}, 6
v_lshl_add_u64 {T23}, %[lanep], 0, {T1}
v_cmp_gt_u64 vcc, %[k_n], {T23}
s_mov_b64 {VM}, vcc
s_waitcnt lgkmcnt(0)
v_mov_b32 {LEN}, {t7}
s_bitcmp1_b32 %[fl], 8
s_cbranch_scc1 .Lsb%=
v_mov_b32 {t7}, 0
v_lshl_add_u64 {BASE}, %[k_frames], 0, {T67}
s_branch .Lsbd%=
.Lsb%=:
; (stride layout: packet tile * 64 + lane at frames + lane * stride + tile * 64 * stride)
s_mul_i32 {T5L}, %[tile], %[tbytes]
s_mul_hi_u32 {T5H}, %[tile], %[tbytes]
v_lshl_add_u64 {BASE}, %[lb], 0, {T5}
.Lsbd%=:
""" + tailfix + """
s_bitcmp1_b32 %[fl], 7
s_cbranch_scc0 .Lnx%=
v_min_u32 {LEN}, 0xffff, {LEN}
v_add_u32 {LEN}, 8, {LEN}
v_lshl_add_u64 {BASE}, {BASE}, 0, -8
.Lnx%=:
v_cndmask_b32 {LEN}, 0, {LEN}, vcc
; the next tile
s_add_u32 {T3}, %[tile], %[W]
s_cmp_lt_u32 {T3}, %[ntiles]
s_cbranch_scc0 .Lnonext%=
s_cmp_lt_u32 {T3}, %[nfull]
s_cbranch_scc0 .Lstg%=
s_bitcmp1_b32 %[fl], 8
s_cbranch_scc1 .Lsn%=
v_add_u32 {t0}, %[nmetab], %[lane4]
ds_read_b32 {t6}, {t0}
v_add_u32 {t0}, %[nmetab], %[moff]
ds_read_b32 {t12}, {t0}
ds_read_b32 {t14}, {t0} offset:64
ds_read_b32 {t16}, {t0} offset:128
ds_read_b32 {t18}, {t0} offset:192
s_bitcmp1_b32 %[fl], 6
s_cbranch_scc0 .Lnl2%=
v_add_u32 {t1}, %[nmetab], %[lane2]
ds_read_u16 {t7}, {t1}
v_add_u32 {t1}, %[nmetab], %[loff]
ds_read_u16 {t8}, {t1}
ds_read_u16 {t9}, {t1} offset:32
ds_read_u16 {t10}, {t1} offset:64
ds_read_u16 {t11}, {t1} offset:96
s_branch .Lnl2d%=
.Lnl2%=:
v_mov_b32 {t7}, %[lenc]
v_mov_b32 {t8}, %[lenc]
v_mov_b32 {t9}, %[lenc]
v_mov_b32 {t10}, %[lenc]
v_mov_b32 {t11}, %[lenc]
.Lnl2d%=:
s_waitcnt lgkmcnt(0)
; every packet of the next tile 16-byte aligned (lanes of length 0 excepted): DMA'd as they are;
; else straight from the packets, the tail lanes from aligned blocks (fixed at its top: %[mis]
; bit 1, bit 0 once it is this tile)
v_add_u32 {t0}, %[fr_lo], {t6}
v_and_b32 {t0}, 15, {t0}
v_cmp_ne_u32 vcc, 0, {t0}
v_cmp_ne_u32_e64 {T0}, 0, {t7}
s_and_b64 vcc, vcc, {T0}
s_cbranch_vccnz .Lmis%=
""" + rounds + """
""" + dmas + """
s_branch .Lmeta%=
.Lmis%=:
; (no packet shorter than the window: no tail lanes, the chunks straight from the packets)
v_cmp_gt_u32 vcc, 64, {t7}
s_cbranch_vccz .Lmnt%=
s_or_b32 %[mis], %[mis], 2
""" + trounds + """
""" + dmas + """
s_branch .Lmeta%=
.Lmnt%=:
""" + rounds + """
""" + dmas + """
s_branch .Lmeta%=
.Lsn%=:
; stride layout (16-byte aligned slots): round r's packet 16r + l/4 at frames + its chunk +
; (l/4) * stride (%[db]) + nt * 64 * stride + r * 16 * stride
s_bitcmp1_b32 %[fl], 6
s_cbranch_scc0 .Lsl%=
v_add_u32 {t1}, %[nmetab], %[loff]
ds_read_u16 {t8}, {t1}
ds_read_u16 {t9}, {t1} offset:32
ds_read_u16 {t10}, {t1} offset:64
ds_read_u16 {t11}, {t1} offset:96
s_branch .Lsld%=
.Lsl%=:
v_mov_b32 {t8}, %[lenc]
v_mov_b32 {t9}, %[lenc]
v_mov_b32 {t10}, %[lenc]
v_mov_b32 {t11}, %[lenc]
.Lsld%=:
s_mul_i32 {T7L}, {T3}, %[tbytes]
s_mul_hi_u32 {T7H}, {T3}, %[tbytes]
""" + srounds + """
s_waitcnt lgkmcnt(0)
""" + smasks + """
""" + dmas + """
s_branch .Lmeta%=
.Lstg%=:
s_mov_b32 %[stage], 1
.Lmeta%=:
; the metadata of nt + W (a whole tile) into this tile's metadata buffer
s_add_u32 {T3}, {T3}, %[W]
s_cmp_lt_u32 {T3}, %[nfull]
s_cbranch_scc0 .Lnonext%=
s_bitcmp1_b32 %[fl], 8
s_cbranch_scc1 .Lml%=
s_mov_b32 {T1L}, {T3}
s_mov_b32 {T1H}, 0
s_lshl_b64 {T1}, {T1}, 8
s_add_u32 {T1L}, {T1L}, %[of_lo]
s_addc_u32 {T1H}, {T1H}, %[of_hi]
v_mov_b32 {t1}, 0
v_mov_b32 {t0}, %[lane4]
v_lshl_add_u64 {T01}, {T01}, 0, {T1}
s_mov_b32 m0, %[metab]
s_nop 0
global_load_lds_dword {T01}, off
.Lml%=:
s_bitcmp1_b32 %[fl], 6
s_cbranch_scc0 .Lnonext%=
s_mov_b32 {T1L}, {T3}
s_mov_b32 {T1H}, 0
s_lshl_b64 {T1}, {T1}, 7
s_add_u32 {T1L}, {T1L}, %[ln_lo]
s_addc_u32 {T1H}, {T1H}, %[ln_hi]
v_mov_b32 {t1}, 0
v_mov_b32 {t0}, %[lane4]
v_lshl_add_u64 {T01}, {T01}, 0, {T1}
s_add_u32 m0, %[metab], 256
s_mov_b32 exec_hi, 0
s_nop 0
global_load_lds_dword {T01}, off
s_mov_b64 exec, -1
.Lnonext%=:
; this tile's lanes
s_mov_b32 {KMEM}, %[k_mem]
s_mov_b64 {KR10}, %[k_r10]
v_add_u32 {WIN}, %[winb], %[lane64]
v_mov_b32 {SWZ}, %[swz]
v_mov_b32 {NST}, 0
v_mov_b32 {ST}, 0
v_mov_b32 {LPC}, -1
s_mov_b64 exec, {VM}
v_mov_b32 {LPC}, 0
v_cmp_lt_u32 vcc, {KMEM}, {LEN}
s_and_b64 exec, exec, vcc
v_mov_b32 {ST}, 7
v_mov_b32 {LPC}, -1
s_mov_b64 exec, -1
s_bitcmp1_b32 %[fl], 4
s_cbranch_scc1 .Linitx%=
;@@JITINIT@@
.Linitd%=:

; JIT N=%= fixed=0 loops=0 aligned=%[aligned] xdp=%[xdpf] ovf=%[k_ovf] tile=%[tile] dm=%[dmask] varl=1
;@@JIT@@
.Ldone%=:
; store mode: lanes that left for the general interpreter (status 0x80, jit.h kStDeopt) produce
; nothing here; their packet indices go to the deopt list (one returning atomic per wave)
s_mov_b64 exec, {VM}
v_cmp_eq_u32 vcc, 0x80, {ST}
s_cbranch_vccz .Lnodo%=
s_bitcmp1_b32 %[fl], 10
s_cbranch_scc1 .Ldofail%=
s_andn2_b64 {VM}, {VM}, vcc
s_mov_b64 {T0}, vcc
s_mov_b64 exec, vcc
v_mbcnt_lo_u32_b32 {t5}, {T0L}, 0
v_mbcnt_hi_u32_b32 {t5}, {T0H}, {t5}
s_bcnt1_i32_b64 {T3}, {T0}
s_ff1_i32_b64 {T1L}, {T0}
s_lshl_b64 {T1}, 1, {T1L}
s_mov_b64 exec, {T1}
v_mov_b32 {t6}, {T3}
v_mov_b64 {T89}, %[k_deopt]
global_atomic_add {t4}, {T89}, {t6}, off sc0
s_waitcnt vmcnt(0)
v_readfirstlane_b32 {T3}, {t4}
s_mov_b64 exec, {T0}
v_add_u32 {t10}, {T3}, {t5}
v_mov_b32 {t11}, 0
v_lshlrev_b64 {T1011}, 2, {T1011}
v_lshl_add_u64 {T89}, {T1011}, 0, %[k_dix]
s_lshl_b32 {T1L}, %[tile], 6
v_add_u32 {t4}, {T1L}, %[lane]
global_store_dword {T89}, {t4}, off
s_branch .Lnodo%=
.Ldofail%=:
; (no deopt pass follows this launch, StackPlan::no_deopt: a lane that left anyway is a failed
; load-time proof -- status EBPF_ST_JIT, counted as a fault, never silently dropped)
s_mov_b64 exec, vcc
v_mov_b32 {ST}, 8
.Lnodo%=:
s_mov_b64 exec, {VM}
v_cmp_gt_u64 vcc, 5, {RF}
v_mov_b32 {t5}, 0xfe
v_cndmask_b32 {t4}, {t5}, {RF0}, vcc
v_cmp_eq_u32 vcc, 0, {ST}
v_mov_b32 {t5}, 0xff
v_cndmask_b32 {t4}, {t5}, {t4}, vcc
v_subrev_u32 {t5}, 0xf9, {t4}
v_min_u32 {t5}, {t4}, {t5}
v_mul_u32_u24 {t5}, 9, {t5}
v_lshlrev_b64 {T67}, {t5}, 1
v_lshl_add_u64 %[acc], %[acc], 0, {T67}
v_add_u32 %[ret], %[ret], {NST}
s_bitcmp1_b32 %[fl], 9
s_cbranch_scc0 .Lnov%=
s_lshl_b32 {T0L}, %[tile], 6
s_lshr_b32 {T0H}, %[tile], 26
s_add_u32 {T0L}, {T0L}, %[vd_lo]
s_addc_u32 {T0H}, {T0H}, %[vd_hi]
v_lshl_add_u64 {T67}, %[lanep], 0, {T0}
global_store_byte {T67}, {t4}, off
.Lnov%=:
s_bitcmp1_b32 %[fl], 5
s_cbranch_scc1 .Lout%=
.Loutd%=:
s_mov_b64 exec, -1
s_lshr_b32 %[mis], %[mis], 1
s_sub_u32 %[cdn], %[cdn], 1
s_add_u32 %[tile], %[tile], %[W]
s_xor_b32 %[winb], %[winb], %[wx]
s_xor_b32 %[nwinb], %[nwinb], %[wx]
s_xor_b32 %[metab], %[metab], %[mx]
s_xor_b32 %[nmetab], %[nmetab], %[mx]
s_cmp_ge_u32 %[tile], %[ntiles]
s_cbranch_scc1 .Lexit%=
s_cmp_lg_u32 %[stage], 0
s_cbranch_scc1 .Lexit%=
s_cmp_eq_u32 %[cdn], 0
s_cbranch_scc0 .Lloop%=
.Lexit%=:
s_waitcnt lgkmcnt(0)
s_mov_b32 m0, {M0S}
s_branch .Lend%=
"""
    ool = """.Linitx%=:
s_bitcmp1_b32 %[fl], 0
s_cbranch_scc1 .Linitc%=
""" + DEFAULT_INIT + """s_branch .Linitd%=
.Linitc%=:
s_load_dwordx2 {T5}, %[ka], %[o_init]
s_waitcnt lgkmcnt(0)
s_load_dwordx16 {UOP}, {T5}, 0x0
s_waitcnt lgkmcnt(0)
""" + "\n".join(f"v_mov_b32 v{i}, s{UB + i}" for i in range(16)) + """
s_load_dwordx4 s[36:39], {T5}, 0x40
s_load_dwordx2 s[40:41], {T5}, 0x50
s_waitcnt lgkmcnt(0)
""" + "\n".join(f"v_mov_b32 v{16 + i}, s{UB + i}" for i in range(6)) + """
s_branch .Linitd%=
.Lout%=:
s_mov_b32 {T1L}, %[tile]
s_mov_b32 {T1H}, 0
s_lshl_b64 {T1}, {T1}, 6
v_lshl_add_u64 {T23}, %[lanep], 0, {T1}
s_load_dwordx2 {ER0}, %[ka], %[o_r0]
s_load_dwordx2 {EST}, %[ka], %[o_status]
s_load_dwordx2 {ERG}, %[ka], %[o_regs]
s_waitcnt lgkmcnt(0)
""" + out_tail + """
.Lend%=:
"""
    return main + ool


def handler_table():
    """Handler names in slot order and their id: every "alu"/"div"/"ool" kind has a chained (_C)
    and a block-end (_E) form; the others one form (_E); then DONE."""
    out = []
    for n, (body, kind) in H.items():
        if kind in ("alu", "div", "ool"):
            out.append((n + "_C", n, "c"))
        out.append((n + "_E", n, "e"))
    out.append((DONE, DONE, "e"))
    return out


def main():
    table = handler_table()
    parts = [PROLOGUE + SLOTS_HEAD]
    for idx, (name, base, sfx) in enumerate(table):
        if base == DONE:
            code = "s_branch .Ldone%="
        else:
            body, kind = H[base]
            if kind == "term":
                code = body
            elif kind == "jump":
                code = body + "\n" + STEP + "\n" + JTAIL
            elif kind == "alu":
                code = (body + "\n" if body else "") + STEP + "\n" + TAILS[sfx]
            elif kind == "div":
                code = body + f"\ns_branch .Ldivmod{sfx}%="
            elif body == "ldx":  # ool, two modes
                code = f".if %[loops]\ns_branch .Lldxl{sfx}%=\n.else\ns_branch .Lldx{sfx}%=\n.endif"
            elif body == "ldx1":
                code = f".if %[loops]\ns_branch .Lldx1l{sfx}%=\n.else\ns_branch .Lldx1{sfx}%=\n.endif"
            else:  # ool
                code = f"s_branch .L{body}{sfx}%="
        code = re.sub(r"\.L(nf_\w+?)%=", lambda m: f".L{m.group(1)}_{idx}%=", code)
        parts.append(f"; {name}\n.org .Lslots%=+{idx * SLOT}\n" + code)
    parts.append(f".org .Lslots%=+{len(table) * SLOT}")
    for sfx in ("c", "e"):
        parts += [ldxk(sfx), ldxk1(sfx), ldxk2(sfx), ldxkfar(sfx), ldx(sfx), ldx_loop(sfx),
                  ldx1(sfx, False), ".if %[loops]", ldx1(sfx, True), ".endif", divmod(sfx)]
    parts += [KFAULT, ".if %[loops]", BUDGET, ".endif", EPILOGUE]
    text = F("\n".join(parts))
    assert "{" not in text, "unsubstituted register name: " + text[text.index("{"):][:40]
    out = ["// GENERATED by gen_tile.py -- do not edit. One inline-asm statement (tile_kernel).",
           "// clang-format off"]
    for line in text.splitlines():
        out.append('"' + line.replace("\\", "\\\\").replace('"', '\\"') + '\\n"')
    out.append("// clang-format on")
    with open(os.path.join(HERE, "tile.inc"), "w") as f:
        f.write("\n".join(out) + "\n")
    # ids: T_<base>_C / T_<base>_E (byte offsets = id * TILE_SLOT)
    ids = ["// GENERATED by gen_tile.py -- do not edit. Handler slots of tile.inc (uop.h TUop::hoff",
           "// = id * TILE_SLOT). Chained (_C) forms continue with the next micro-op; block-end (_E)",
           "// forms update the pc set and dispatch.",
           "#pragma once", f"#define TILE_SLOT {SLOT}", f"#define TILE_NVGPR {NVGPR}"]
    for idx, (name, base, sfx) in enumerate(table):
        ids.append(f"#define T{name[1:]} {idx}")
    ids.append(f"#define T_COUNT {len(table)}")
    # old (dag_asm.h) id -> tile ids, for the host's table builder
    c_map, e_map = [], []
    for n in sorted(IDS_OLD, key=lambda k: IDS_OLD[k]):
        if n == "H_COUNT":
            continue
        e = f"T{n[1:]}_E"
        c = f"T{n[1:]}_C" if any(t[0] == n + "_C" for t in table) else e
        c_map.append(c)
        e_map.append(e)
    ids.append("// indexed by dag_asm.h H_* ids")
    ids.append("static const short kTileIdChained[] = {" + ", ".join(c_map) + "};")
    ids.append("static const short kTileIdEnd[] = {" + ", ".join(e_map) + "};")
    with open(os.path.join(HERE, "tile_ids.h"), "w") as f:
        f.write("\n".join(ids) + "\n")
    # JIT: the template kernels' statements and the per-handler templates, indexed by tile id
    text = F(JIT_STATEMENT)
    assert "{" not in text
    with open(os.path.join(HERE, "tile_jit.inc"), "w") as f:
        f.write("// GENERATED by gen_tile.py -- do not edit. The JIT template kernel's statement.\n"
                "// clang-format off\n" + cstr(text) + "\n// clang-format on\n")
    # the var kernel's statement for stack-window programs (memory tier 0.5 on offsets / lens and
    # xdp_md layouts: ebpf_tile_jit_var_stack, whose statement also owns v[64:95])
    text = F(JIT_STATEMENT).replace("aligned=%[aligned]\n", "aligned=%[aligned] stack=1\n")
    assert "stack=1" in text
    with open(os.path.join(HERE, "tile_jit_stack.inc"), "w") as f:
        f.write("// GENERATED by gen_tile.py -- do not edit. The JIT template kernel's statement for "
                "stack-window programs.\n// clang-format off\n" + cstr(text) + "\n// clang-format on\n")
    # the loop kernel's statement with a deeper refill prefetch (ebpf_tile_jit_loop_deep, whose
    # statement also owns the prefetch stages v[72:103] and their tags v104, v105)
    text = F(JIT_STATEMENT).replace("aligned=%[aligned]\n", "aligned=%[aligned] deep=1\n")
    assert "deep=1" in text
    with open(os.path.join(HERE, "tile_jit_deep.inc"), "w") as f:
        f.write("// GENERATED by gen_tile.py -- do not edit. The JIT template kernel's statement for "
                "loop programs with a deep refill prefetch.\n// clang-format off\n" + cstr(text) +
                "\n// clang-format on\n")
    # the compiled fixed-slot kernel's tile loop (jit_statement_loop)
    text = F(jit_statement_loop())
    assert "{" not in text, "unsubstituted register name: " + text[text.index("{"):][:40]
    with open(os.path.join(HERE, "tile_jit_loop.inc"), "w") as f:
        f.write("// GENERATED by gen_tile.py -- do not edit. The compiled fixed-slot kernel's tile "
                "loop (one statement, many tiles).\n// clang-format off\n" + cstr(text) +
                "\n// clang-format on\n")
    # ... its occupancy variant (ebpf_tile_jit_fixed_occ: one window buffer per wave)
    text = F(jit_statement_loop(single=True))
    assert "{" not in text, "unsubstituted register name: " + text[text.index("{"):][:40]
    with open(os.path.join(HERE, "tile_jit_loop1.inc"), "w") as f:
        f.write("// GENERATED by gen_tile.py -- do not edit. The compiled fixed-slot kernel's tile "
                "loop, one window buffer per wave (ebpf_tile_jit_fixed_occ).\n// clang-format off\n" +
                cstr(text) + "\n// clang-format on\n")
    # the compiled var kernel's tile loop (jit_statement_varl), and its statement for
    # stack-window programs (ebpf_tile_jit_varl_stack: the stack window in v[80:95] too)
    text = F(jit_statement_varl())
    assert "{" not in text, "unsubstituted register name: " + text[text.index("{"):][:40]
    with open(os.path.join(HERE, "tile_jit_varl.inc"), "w") as f:
        f.write("// GENERATED by gen_tile.py -- do not edit. The compiled var kernel's tile loop "
                "(offsets + lens batches, one statement, many tiles).\n// clang-format off\n" +
                cstr(text) + "\n// clang-format on\n")
    text = text.replace(" varl=1\n", " varl=1 stack=1\n")
    assert "stack=1" in text
    with open(os.path.join(HERE, "tile_jit_varl_stack.inc"), "w") as f:
        f.write("// GENERATED by gen_tile.py -- do not edit. The var tile loop's statement for "
                "stack-window programs.\n// clang-format off\n" + cstr(text) +
                "\n// clang-format on\n")
    out = ["// GENERATED by gen_tile.py -- do not edit. Per-handler JIT templates (jit.cpp), indexed",
           "// by tile id (tile_ids.h): {main text, out-of-line text}.", "#pragma once",
           "// clang-format off", "static const char* const kJitTemplates[T_COUNT][2] = {"]
    for idx, (name, base, sfx) in enumerate(table):
        main_t, ool_t = jit_template(base)
        out.append(f"// {name}\n{{{cstr(main_t)},\n{cstr(ool_t)}}},")
    out += ["};"]
    # per-register initialisation of the main.rs layout (the compiler's ;@@JITINIT@@)
    inits = []
    for r in range(11):
        if r == 2:
            t = "v_mov_b32 v4, {LEN}\nv_mov_b32 v5, 0"
        elif r == 10:
            t = "v_mov_b32 v20, {KR10L}\nv_mov_b32 v21, {KR10H}"
        else:
            t = f"v_mov_b64 v[{2 * r}:{2 * r + 1}], 0"
        inits.append(cstr(F(t)))
    assert F("\n".join(DEFAULT_INIT.split("\n"))) == F(DEFAULT_INIT)
    out += ["static const char* const kJitInitReg[11] = {" + ",\n".join(inits) + "};"]
    # loop programs' window refill (refill() above): exec = the lanes whose access needs packet
    # bytes outside their window (T7), v36 = the address; WB = a & ~15 and 64 bytes from there
    out += ["static const char* const kJitRefill =\n" + cstr(F(refill("x"))) + ";",
            "// clang-format on"]
    with open(os.path.join(HERE, "jit_tmpl.h"), "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "--clobbers":
        print(", ".join(f'"s{s}"' for s in SGPRS) + ", " +
              ", ".join(f'"v{v}"' for v in range(NVGPR)))
    else:
        main()
