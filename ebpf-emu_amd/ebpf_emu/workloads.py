"""Synthetic XDP workloads of BASELINE.json configs 2-5.

Frames: seeded (numpy PCG64, seed 0x5EED0000 + config id) Ethernet frames. EtherType IPv4
(90 %), IPv6 (5 %), ARP (5 %); IPv4 IHL 5 (95 %) or 6 with 4 option bytes (5 %); protocol TCP
(45 %), UDP (45 %), ICMP (10 %); ~25 % of UDP flows to port 53; random addresses, ports and
payload. Fixed 64-byte frames use the stride layout; mixed 64 / 1500-byte frames use
offsets + lengths with every frame starting on a 64-byte boundary (a NIC-ring-like layout).

Programs (hand-assembled: the container's LLVM has no BPF target). Jump offsets follow the
reference's decoded-entry indexing (asm.py).
"""
from __future__ import annotations

import numpy as np

from .asm import assemble

SEED_BASE = 0x5EED0000

# config 2: XDP_DROP-all, 3 instructions, touches the frame
DROP_ALL = """
    ldxb r3, [r1+0]
    mov r0, 1
    exit
"""

# config 3/4: IPv4 5-tuple parse -> PASS (2) / DROP (1), 32 instructions.
# Loads are little-endian (the reference's memcpy into an i64, emu.rs:341-349), so big-endian
# header fields are compared byte-swapped or converted with be16 (END, emu.rs:165-209).
FIVE_TUPLE = """
    mov r0, 2                 # default XDP_PASS
    jlt r2, 34, out           # shorter than Ethernet + IPv4 header
    ldxh r3, [r1+12]          # EtherType
    jne r3, 0x0008, out       # 0x0800 read little-endian
    ldxb r4, [r1+14]          # version / IHL
    and r4, 0x0f
    lsh r4, 2                 # IHL * 4
    jlt r4, 20, drop          # malformed header
    ldxb r5, [r1+23]          # protocol
    ldxw r6, [r1+26]          # saddr (first octet in the low byte)
    ldxw r7, [r1+30]          # daddr
    mov r8, r1
    add r8, r4                # r8 + 14 = L4 header
    jeq r5, 1, icmp
    jeq r5, 17, udp
    jne r5, 6, out
    ldxh r9, [r8+16]          # TCP dport
    be16 r9
    jge r9, 1024, out         # only well-known ports are filtered
    and r6, 0xff
    jeq r6, 10, drop          # 10.0.0.0/8 -> well-known TCP port: drop
    ja out
udp:
    ldxh r9, [r8+16]          # UDP dport
    be16 r9
    jeq r9, 53, drop          # DNS: drop
    ja out
icmp:
    and r7, 0xf0
    jeq r7, 0xe0, drop        # ICMP to 224.0.0.0/4: drop
    ja out
drop:
    mov r0, 1                 # XDP_DROP
out:
    exit
"""

# config 5: per-byte checksum loop, ~6 instructions per byte, then fold + parity.
CHECKSUM = """
    mov r0, 0
    mov r3, 0
    jge r3, r2, done
loop:
    mov r4, r1
    add r4, r3
    ldxb r5, [r4+0]
    add r0, r5
    add r3, 1
    jlt r3, r2, loop
done:
    mov r6, r0
    rsh r6, 8
    xor r0, r6
    and r0, 1
    add r0, 1                 # DROP (1) or PASS (2) by parity
    exit
"""

# config 5 as a standard XDP program under the xdp_md calling convention (xdp.rs:16-20): the sum
# over ctx->data .. ctx->data_end. Same verdicts as CHECKSUM on the same packets. A loop program:
# its xdp_md batches are staged (interp.hip xdp_stage) for the compiled loop kernels.
CHECKSUM_XDP = """
    ldxw r2, [r1+0]           # ctx->data
    ldxw r3, [r1+4]           # ctx->data_end
    mov r0, 0
    jge r2, r3, done
loop:
    ldxb r5, [r2+0]
    add r0, r5
    add r2, 1
    jlt r2, r3, loop
done:
    mov r6, r0
    rsh r6, 8
    xor r0, r6
    and r0, 1
    add r0, 1                 # DROP (1) or PASS (2) by parity
    exit
"""

# CHECKSUM_XDP with ctx->data_end reloaded in every iteration (a loop that reads the ctx: run in
# place, its refilled windows carry the synthesised ctx -- jit.cpp ctx_load). Same verdicts.
CHECKSUM_XDP_RELOAD = """
    ldxw r2, [r1+0]           # ctx->data
    mov r0, 0
loop:
    ldxw r3, [r1+4]           # ctx->data_end, every iteration
    jge r2, r3, done
    ldxb r5, [r2+0]
    add r0, r5
    add r2, 1
    ja loop
done:
    mov r6, r0
    rsh r6, 8
    xor r0, r6
    and r0, 1
    add r0, 1                 # DROP (1) or PASS (2) by parity
    exit
"""

# config 5 with its running sum kept in a stack slot (r10 - 8) instead of a register, the way
# compiled C keeps a spilled accumulator: memory tier 0.5 with a loop (the loop kernel's stack
# variant). Same verdicts as CHECKSUM.
CHECKSUM_STACK = """
    stdw [r10-8], 0
    mov r3, 0
    jge r3, r2, done
loop:
    mov r4, r1
    add r4, r3
    ldxb r5, [r4+0]
    ldxdw r0, [r10-8]
    add r0, r5
    stxdw [r10-8], r0
    add r3, 1
    jlt r3, r2, loop
done:
    ldxdw r0, [r10-8]
    mov r6, r0
    rsh r6, 8
    xor r0, r6
    and r0, 1
    add r0, 1                 # DROP (1) or PASS (2) by parity
    exit
"""

# the 5-tuple with its flow key spilled to the stack and read back (memory tier 0.5, the XDP
# pattern of building a map key at r10 - N): saddr, daddr, protocol and destination port stored
# at r10 - 16 .. r10 - 5, the decisions taken on the reloaded key. Same verdicts as FIVE_TUPLE.
FIVE_TUPLE_STACK = """
    mov r0, 2                 # default XDP_PASS
    jlt r2, 34, out
    ldxh r3, [r1+12]          # EtherType
    jne r3, 0x0008, out
    ldxb r4, [r1+14]
    and r4, 0x0f
    lsh r4, 2                 # IHL * 4
    jlt r4, 20, drop
    ldxw r6, [r1+26]          # saddr
    stxw [r10-16], r6         # key.saddr
    ldxw r7, [r1+30]          # daddr
    stxw [r10-12], r7         # key.daddr
    ldxb r5, [r1+23]          # protocol
    stxb [r10-8], r5          # key.proto
    stb [r10-7], 0            # key.pad
    mov r8, r1
    add r8, r4
    ldxh r9, [r8+16]          # L4 destination port
    stxh [r10-6], r9          # key.dport
    ldxb r5, [r10-8]          # reload the key
    jeq r5, 1, icmp
    ldxh r9, [r10-6]
    be16 r9
    jeq r5, 17, udp
    jne r5, 6, out
    jge r9, 1024, out
    ldxb r6, [r10-16]         # first octet of key.saddr (upper bytes kept: emu.rs:341-349)
    and r6, 0xff
    jeq r6, 10, drop
    ja out
udp:
    jeq r9, 53, drop
    ja out
icmp:
    ldxw r7, [r10-12]
    and r7, 0xf0
    jeq r7, 0xe0, drop
    ja out
drop:
    mov r0, 1                 # XDP_DROP
out:
    exit
"""

# an XDP_TX reflector that swaps the Ethernet source and destination MACs in the packet (stores
# into the packet: emu.rs:354-372), accumulates the length into a stack slot with an atomic add
# (emu.rs:373-437) and reflects frames of >= 60 bytes (XDP_TX), dropping runts. Memory tier 0.5
# with packet-window stores on fixed slots (the compiled kernel), tier 1 elsewhere.
MAC_SWAP_TX = """
    ldxw r3, [r1+0]           # destination MAC
    ldxh r4, [r1+4]
    ldxw r5, [r1+6]           # source MAC
    ldxh r6, [r1+10]
    stxw [r1+0], r5           # swap them in the packet
    stxh [r1+4], r6
    stxw [r1+6], r3
    stxh [r1+10], r4
    stdw [r10-8], 0
    mov r7, r2
    lock add [r10-8], r7      # length into a stack counter
    ldxdw r0, [r10-8]
    jlt r0, 60, drop
    mov r0, 3                 # XDP_TX
    exit
drop:
    mov r0, 1
    exit
"""

# a NAT / router rewrite (memory store mode): IPv4 TTL decremented in place with the header
# checksum adjusted (RFC 1624: + 0x0100 with the end-around carry), and TCP/UDP destination ports
# 53 and 80 redirected to 8053 / 8080 -- the L4 header sits behind the variable-length IPv4
# header (IHL), so the port store goes through a register (host.cpp analyze_stack: store mode,
# the header window in LDS). Verdicts: XDP_TX for redirected frames, PASS otherwise, DROP at TTL <= 1
# or IHL < 5. Same frames as the 5-tuple.
NAT_REWRITE = """
    mov r0, 2                 # XDP_PASS
    jlt r2, 34, out
    ldxh r3, [r1+12]          # EtherType (a little-endian load of big-endian bytes)
    jne r3, 0x0008, out       # IPv4 only
    ldxb r4, [r1+22]          # TTL
    jle r4, 1, drop
    sub r4, 1
    stxb [r1+22], r4          # TTL - 1, in place
    ldxh r5, [r1+24]          # header checksum
    be16 r5
    add r5, 0x100             # RFC 1624 for the TTL byte (the high byte of its word)
    mov r6, r5
    rsh r6, 16
    and r5, 0xffff
    add r5, r6
    be16 r5
    stxh [r1+24], r5
    ldxb r6, [r1+14]          # version / IHL
    and r6, 15
    jlt r6, 5, drop           # malformed
    lsh r6, 2
    mov r7, r1
    add r7, r6
    add r7, 14                # the L4 header, behind the IPv4 options
    ldxb r8, [r1+23]          # protocol
    jeq r8, 6, l4
    jne r8, 17, out
l4:
    ldxh r9, [r7+2]           # destination port
    be16 r9
    jeq r9, 53, redirect
    jne r9, 80, out
redirect:
    add r9, 8000              # 53 -> 8053, 80 -> 8080
    be16 r9
    stxh [r7+2], r9           # a register-address store into the packet
    ldxh r3, [r7+2]           # read back through the pointer
    jne r3, r9, drop          # (never taken)
    mov r0, 3                 # XDP_TX
    exit
drop:
    mov r0, 1
out:
    exit
"""

# an XDP responder over 1500-byte frames (memory store mode with the overflow image, jit.cpp
# ovf_fill): ICMP echo requests answered in place -- Ethernet and IPv4 addresses swapped, type 8
# -> 0 with the ICMP checksum adjusted (RFC 1624), XDP_TX -- and every other IPv4 frame's 4-byte
# telemetry trailer (the frame's last 4 bytes: r1 + r2 - 4, byte 1500 of a 1504-byte slot)
# incremented in place, read back, XDP_PASS. The ICMP header sits behind the IPv4 options, the
# trailer at the packet's length: both register-address stores, the trailer far past the
# 64-byte header window.
RESPONDER = """
    mov r0, 2                 # XDP_PASS
    jlt r2, 42, out
    ldxh r3, [r1+12]          # EtherType
    jne r3, 0x0008, out
    ldxb r6, [r1+14]          # version / IHL
    and r6, 15
    jlt r6, 5, drop
    ldxb r4, [r1+23]          # protocol
    jne r4, 1, trailer
    lsh r6, 2
    mov r7, r1
    add r7, r6
    add r7, 14                # the ICMP header, behind the IPv4 options
    ldxb r5, [r7+0]           # type
    jne r5, 8, trailer        # echo request only
    ldxw r3, [r1+0]           # swap the MACs
    ldxh r4, [r1+4]
    ldxw r5, [r1+6]
    ldxh r8, [r1+10]
    stxw [r1+0], r5
    stxh [r1+4], r8
    stxw [r1+6], r3
    stxh [r1+10], r4
    ldxw r3, [r1+26]          # swap the IPv4 addresses
    ldxw r4, [r1+30]
    stxw [r1+26], r4
    stxw [r1+30], r3
    stb [r7+0], 0             # echo reply
    ldxh r5, [r7+2]           # checksum + 0x0800 (RFC 1624, end-around carry)
    be16 r5
    add r5, 0x0800
    mov r6, r5
    rsh r6, 16
    and r5, 0xffff
    add r5, r6
    be16 r5
    stxh [r7+2], r5
    mov r0, 3                 # XDP_TX
    exit
trailer:
    mov r9, r1
    add r9, r2                # the packet's end
    ldxw r3, [r9-4]           # the telemetry trailer
    add32 r3, 1
    stxw [r9-4], r3           # a register-address store at the frame's tail
    ldxw r4, [r9-4]           # read back through the pointer
    jne r4, r3, drop          # (never taken)
    exit
drop:
    mov r0, 1
out:
    exit
"""

# a firewall of ~100 instructions (past the tile interpreter's 62 micro-ops: compiled by the
# forward-program compiler instead of interpreted by dag_kernel): 802.1Q, IPv4 sanity (version,
# IHL, TTL, fragments), source and destination address rules, TCP flag and port rules, UDP
# service rules, ICMP types, IPv6 next header / hop limit, ARP opcodes. Loads are little-endian
# (emu.rs:341-349): big-endian fields are compared byte-swapped or converted with be16.
ACL = """
    mov r0, 2                 # XDP_PASS
    jlt r2, 34, out
    ldxh r3, [r1+12]          # EtherType
    mov r8, 14                # L3 offset
    jne r3, 0x0081, novlan    # 802.1Q (0x8100)
    ldxh r3, [r1+16]
    mov r8, 18
novlan:
    jeq r3, 0xdd86, ipv6      # 0x86DD
    jeq r3, 0x0608, arp       # 0x0806
    jne r3, 0x0008, out       # 0x0800
    mov r4, r1
    add r4, r8                # IPv4 header
    ldxb r5, [r4+0]           # version / IHL
    mov r6, r5
    rsh r6, 4
    jne r6, 4, drop
    and r5, 0x0f
    jlt r5, 5, drop
    lsh r5, 2                 # IHL * 4
    ldxb r6, [r4+8]           # TTL
    jlt r6, 2, drop
    ldxh r6, [r4+6]           # flags / fragment offset
    be16 r6
    and r6, 0x1fff
    jne r6, 0, drop           # fragments
    ldxb r7, [r4+9]           # protocol
    ldxw r9, [r4+12]          # saddr (first octet in the low byte)
    mov r6, r9
    and r6, 0xff
    jeq r6, 127, drop         # loopback source
    jeq r6, 0, drop           # 0.0.0.0/8 source
    mov r6, r9
    and r6, 0xffff
    jeq r6, 0xfea9, drop      # 169.254.0.0/16 source
    ldxw r3, [r4+16]          # daddr
    mov r6, r3
    and r6, 0xf0
    jeq r6, 0xe0, mcast       # 224.0.0.0/4
    jeq r6, 0xf0, drop        # 240.0.0.0/4
    add r4, r5                # L4 header
    jeq r7, 6, tcp
    jeq r7, 17, udp
    jeq r7, 1, icmp
    jeq r7, 47, drop          # GRE
    ja out
mcast:
    jne r7, 17, drop          # multicast: UDP only
    ja out
tcp:
    ldxh r6, [r4+2]           # destination port
    be16 r6
    ldxb r3, [r4+13]          # flags
    mov r5, r3
    and r5, 0x03
    jeq r5, 3, drop           # SYN + FIN
    jeq r3, 0, drop           # null scan
    jeq r6, 23, drop          # telnet
    jeq r6, 3389, drop        # RDP
    jeq r6, 445, drop         # SMB
    jge r6, 1024, out
    mov r5, r9
    and r5, 0xff
    jeq r5, 10, drop          # 10.0.0.0/8 to a well-known port
    ja out
udp:
    ldxh r6, [r4+2]
    be16 r6
    jeq r6, 53, dns
    jeq r6, 1900, drop        # SSDP
    jeq r6, 19, drop          # chargen
    jeq r6, 123, ntp
    ja out
dns:
    mov r5, r9
    and r5, 0xffff
    jeq r5, 0xa8c0, out       # resolvers in 192.168.0.0/16
    ja drop
ntp:
    ldxh r5, [r4+4]           # UDP length
    be16 r5
    jgt r5, 100, drop         # amplification-sized
    ja out
icmp:
    ldxb r5, [r4+0]           # type
    jeq r5, 8, out            # echo request
    jeq r5, 0, out            # echo reply
    jeq r5, 3, out            # unreachable
    jeq r5, 11, out           # time exceeded
    ja drop
ipv6:
    mov r4, r1
    add r4, r8
    ldxb r5, [r4+6]           # next header
    ldxb r6, [r4+7]           # hop limit
    jlt r6, 2, drop
    jeq r5, 58, out           # ICMPv6
    jeq r5, 0, drop           # hop-by-hop options
    ja out
arp:
    ldxh r5, [r1+20]          # opcode
    be16 r5
    jgt r5, 2, drop
    ja out
drop:
    mov r0, 1                 # XDP_DROP
out:
    exit
"""

# the 5-tuple classifier as a standard XDP program (the xdp_md calling convention, xdp.rs:16-20:
# r1 = the ctx, packet bytes between ctx->data and ctx->data_end), with the verifier-style bounds
# checks before the header and port reads. Same verdicts as FIVE_TUPLE on the synthetic frames
# (their L4 ports lie inside every frame).
FIVE_TUPLE_XDP = """
    ldxw r2, [r1+0]           # ctx->data
    ldxw r1, [r1+4]           # ctx->data_end
    mov r0, 2                 # default XDP_PASS
    mov r3, r2
    add r3, 34
    jgt r3, r1, out           # no Ethernet + IPv4 header
    ldxh r3, [r2+12]          # EtherType
    jne r3, 0x0008, out
    ldxb r4, [r2+14]          # version / IHL
    and r4, 0x0f
    lsh r4, 2                 # IHL * 4
    jlt r4, 20, drop
    ldxb r5, [r2+23]          # protocol
    ldxw r6, [r2+26]          # saddr
    ldxw r7, [r2+30]          # daddr
    mov r8, r2
    add r8, r4                # r8 + 14 = L4 header
    jeq r5, 1, icmp
    mov r9, r8
    add r9, 18
    jgt r9, r1, out           # no L4 ports
    jeq r5, 17, udp
    jne r5, 6, out
    ldxh r9, [r8+16]          # TCP dport
    be16 r9
    jge r9, 1024, out
    and r6, 0xff
    jeq r6, 10, drop
    ja out
udp:
    ldxh r9, [r8+16]          # UDP dport
    be16 r9
    jeq r9, 53, drop
    ja out
icmp:
    and r7, 0xf0
    jeq r7, 0xe0, drop
    ja out
drop:
    mov r0, 1                 # XDP_DROP
out:
    exit
"""

# the 5-tuple with its L4 decision as a local function (CALL, emu.rs:265-279), the pattern of a
# bpf-to-bpf call. The reference pushes the callee's entry + 1 as the return address (Q12), so
# l4's EXIT returns into l4 itself: its body after the first instruction runs a second time and
# that EXIT, with the frame stack empty, ends the program. The body is idempotent, so the verdicts
# are FIVE_TUPLE's. On the compiled kernels the calls are flattened at load time (flatten_calls).
FIVE_TUPLE_CALL = """
    mov r0, 2                 # default XDP_PASS
    jlt r2, 34, out
    ldxh r3, [r1+12]          # EtherType
    jne r3, 0x0008, out
    ldxb r4, [r1+14]
    and r4, 0x0f
    lsh r4, 2                 # IHL * 4
    jlt r4, 20, drop
    ldxb r5, [r1+23]          # protocol
    ldxw r6, [r1+26]          # saddr
    ldxw r7, [r1+30]          # daddr
    call l4
drop:
    mov r0, 1                 # XDP_DROP
out:
    exit
l4:
    mov r0, 2                 # skipped by the return pass (entry + 1)
    mov r8, r1
    add r8, r4                # r8 + 14 = L4 header
    jeq r5, 1, icmp
    jeq r5, 17, udp
    jne r5, 6, l4_out
    ldxh r9, [r8+16]          # TCP dport
    be16 r9
    jge r9, 1024, l4_out
    and r6, 0xff
    jeq r6, 10, l4_drop
    ja l4_out
udp:
    ldxh r9, [r8+16]          # UDP dport
    be16 r9
    jeq r9, 53, l4_drop
    ja l4_out
icmp:
    and r7, 0xf0
    jeq r7, 0xe0, l4_drop
    ja l4_out
l4_drop:
    mov r0, 1
l4_out:
    exit
"""



def acl_rules_source(rules: int = 128, seed: int = 11) -> str:
    """A rule-table firewall of `rules` seeded rules (~9 instructions each: 1,200 instructions at
    128 -- past the compiler's near-branch reach, jit.cpp far mode), the shape of an iptables-style
    chain written as straight-line XDP: the Ethernet/IPv4 5-tuple loaded once (IHL 5; frames
    without one pass), then rule k: (saddr & mask) == prefix, (daddr & mask) == prefix, protocol,
    destination port in [lo, hi] -> its verdict, else rule k + 1; no rule: XDP_PASS. Prefixes are
    /8 on saddr's first octet (10 or a seeded octet: the synthetic frames randomise the rest), or
    wider; most packets match no rule and run every rule's first test."""
    import random as _random

    rng = _random.Random(seed)
    out = ["    mov r0, 2", "    jlt r2, 38, out", "    ldxh r3, [r1+12]", "    jne r3, 0x0008, out",
           "    ldxb r4, [r1+23]           # protocol", "    ldxw r5, [r1+26]           # saddr",
           "    ldxw r6, [r1+30]           # daddr", "    ldxh r7, [r1+36]           # dport",
           "    be16 r7"]
    for k in range(rules):
        nxt = f"r{k + 1}" if k + 1 < rules else "out"
        out.append(f"r{k}:")
        octet = 10 if rng.random() < 0.15 else rng.randrange(256)
        kind = rng.random()
        if kind < 0.6:  # saddr /8
            out += ["    mov r8, r5", "    and r8, 0xff", f"    jne r8, {octet}, {nxt}"]
        else:           # saddr /16 (the second octet is random in the frames: rare)
            out += ["    mov r8, r5", "    and r8, 0xffff",
                    f"    jne r8, {octet | (rng.randrange(256) << 8)}, {nxt}"]
        if rng.random() < 0.3:  # daddr /8
            out += ["    mov r8, r6", "    and r8, 0xff", f"    jne r8, {rng.randrange(256)}, {nxt}"]
        proto = rng.choice([6, 17, None])
        if proto is not None:
            out.append(f"    jne r4, {proto}, {nxt}")
            lo = rng.choice([0, 0, 53, 80, 443, 1024, rng.randrange(65536)])
            hi = min(65535, lo + rng.choice([0, 0, 10, 1023, 30000]))
            out += [f"    jlt r7, {lo}, {nxt}", f"    jgt r7, {hi}, {nxt}"]
        out += [f"    mov r0, {1 if rng.random() < 0.7 else 2}", "    ja out"]
    out += ["out:", "    exit"]
    return "\n".join(out) + "\n"


ACL_RULES = acl_rules_source()

PROGRAMS = {"drop": DROP_ALL, "5tuple": FIVE_TUPLE, "checksum": CHECKSUM,
            "5tuple_stack": FIVE_TUPLE_STACK, "mac_swap_tx": MAC_SWAP_TX, "acl": ACL,
            "5tuple_xdp": FIVE_TUPLE_XDP, "checksum_stack": CHECKSUM_STACK,
            "5tuple_call": FIVE_TUPLE_CALL, "nat": NAT_REWRITE, "checksum_xdp": CHECKSUM_XDP,
            "checksum_xdp_reload": CHECKSUM_XDP_RELOAD,
            "responder": RESPONDER}


# long programs (far mode), kept apart from PROGRAMS (the compact benchmark programs)
LONG_PROGRAMS = {"acl_rules": ACL_RULES}


def program(name: str) -> bytes:
    return assemble(PROGRAMS[name] if name in PROGRAMS else LONG_PROGRAMS[name])


def _headers(rng: np.random.Generator, n: int, frame_len: np.ndarray, buf: np.ndarray,
             starts: np.ndarray) -> None:
    """Write Ethernet/IPv4/L4 headers into buf at starts (frames already hold random bytes)."""
    u = rng.random(n)
    ethertype = np.where(u < 0.90, 0x0800, np.where(u < 0.95, 0x86DD, 0x0806)).astype(np.uint16)
    ihl = np.where(rng.random(n) < 0.95, 5, 6).astype(np.uint8)
    p = rng.random(n)
    proto = np.where(p < 0.45, 6, np.where(p < 0.90, 17, 1)).astype(np.uint8)
    dport = rng.integers(0, 65536, n, dtype=np.uint32).astype(np.uint16)
    dns = (proto == 17) & (rng.random(n) < 0.25)
    dport[dns] = 53
    low = (proto == 6) & (rng.random(n) < 0.30)
    dport[low] = rng.integers(0, 1024, int(low.sum()), dtype=np.uint32).astype(np.uint16)
    saddr0 = rng.integers(0, 256, n, dtype=np.uint32).astype(np.uint8)
    ten = rng.random(n) < 0.20
    saddr0[ten] = 10

    def put(off, vals):
        idx = starts + off
        ok = off < frame_len
        buf[idx[ok]] = vals[ok]

    put(12, (ethertype >> 8).astype(np.uint8))
    put(13, (ethertype & 0xFF).astype(np.uint8))
    put(14, (0x40 | ihl).astype(np.uint8))
    put(23, proto)
    put(26, saddr0)
    l4 = 14 + ihl.astype(np.int64) * 4
    for k, v in ((2, dport >> 8), (3, dport & 0xFF)):
        idx = starts + l4 + k
        ok = (l4 + k) < frame_len
        buf[idx[ok]] = v.astype(np.uint8)[ok]


def frames_fixed(n: int, frame: int = 64, config_id: int = 3) -> np.ndarray:
    """n fixed-size frames, stride layout: uint8[n * frame]."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + config_id))
    buf = rng.integers(0, 256, n * frame, dtype=np.uint8)
    starts = np.arange(n, dtype=np.int64) * frame
    _headers(rng, n, np.full(n, frame, dtype=np.int64), buf, starts)
    return buf


def frames_mixed(n: int, small: int = 64, large: int = 1500, align: int = 64,
                 config_id: int = 5):
    """Mixed 64/1500-byte frames (50/50 by seeded coin): (buf uint8, offsets uint32, lens uint16)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + config_id))
    lens = np.where(rng.random(n) < 0.5, small, large).astype(np.int64)
    slots = (lens + align - 1) // align * align
    offsets = np.zeros(n, dtype=np.int64)
    offsets[1:] = np.cumsum(slots)[:-1]
    total = int(offsets[-1] + slots[-1]) if n else 0
    if total >= 1 << 32:
        raise ValueError("mixed batch exceeds the u32 offset range")
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    _headers(rng, n, lens, buf, offsets)
    return buf, offsets.astype(np.uint32), lens.astype(np.uint16)
