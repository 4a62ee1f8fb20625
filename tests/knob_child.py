"""Child process of tests/test_knobs.py: the library reads its environment switches once, when
it is loaded, so each switch runs in a fresh process. argv: <case> <ebpf-emu_amd dir> <oracle dir>.
Runs the case's batch on cuda:0 with the switch the parent set, checks every output against the
C oracle (oracle/, restating emu.rs / mmu.rs / main.rs), prints one JSON line and exits 0."""
import ctypes
import json
import random
import struct
import sys

import numpy as np


def main():
    case, pkg, ordir = sys.argv[1:4]
    sys.path[:0] = [pkg, ordir]
    import torch

    import oracle
    from ebpf_emu import Program, _lib
    from ebpf_emu import workloads as W
    from ebpf_emu.asm import assemble

    dev = torch.device("cuda", 0)
    out = {"case": case}
    if case in ("trace", "fold"):
        # the headline workload on fixed 64-byte slots (ebpf_tile_jit_fixed)
        n = 100_003
        buf = W.frames_fixed(n, 64, 3)
        img = W.program("5tuple")
        prog = Program(img)
        cnt = torch.zeros(8, dtype=torch.int64, device=dev)
        res = prog.run(torch.from_numpy(buf).to(dev), n=n, stride=64, r0=True, status=True,
                       counters=cnt)
        torch.cuda.synchronize()
        r0, st, ocnt = oracle.Program(img).run_batch(buf, n, stride=64, threads=8)
        assert np.array_equal(res.status.cpu().numpy(), st)
        assert np.array_equal(res.r0.cpu().numpy().view(np.uint64), r0)
        assert list(cnt.cpu().numpy().view(np.uint64)) == list(ocnt)
        out["kernel"] = prog.batch_kernel(prog.make_batch(torch.zeros(64, dtype=torch.uint8,
                                                                      device=dev), n=1, stride=64))
        if case == "trace":  # the stamp buffer (ebpf_debug_trace): allocated and written
            p = ctypes.c_void_p()
            nb = ctypes.c_size_t()
            rc = _lib.lib().ebpf_debug_trace(0, ctypes.byref(p), ctypes.byref(nb))
            assert rc == 0 and p.value and nb.value > 0, (rc, p.value, nb.value)
            words = torch.empty(nb.value // 8, dtype=torch.int64, device=dev)
            hip = ctypes.CDLL("libamdhip64.so")
            assert hip.hipMemcpy(ctypes.c_void_p(words.data_ptr()), p, nb, 3) == 0  # D2D
            torch.cuda.synchronize()
            out["stamps_nonzero"] = int((words != 0).sum().item())
            assert out["stamps_nonzero"] > 0
    elif case == "xdp_stage":
        # every xdp_md batch through xdp_stage's copy: the staged path for a parser and a loop
        rng = random.Random(3)
        pkts = []
        for _ in range(500):
            pk = bytearray(rng.getrandbits(8) for _ in range(rng.choice([0, 14, 34, 60, 64, 300, 1000])))
            if len(pk) >= 24 and rng.random() < 0.7:
                pk[12:14] = b"\x08\x00"
                pk[23] = rng.choice([6, 17])
            pkts.append(bytes(pk))
        offs, pos, chunks = [], 0, []
        for pk in pkts:
            pad = (-pos) % 16
            chunks.append(bytes(pad))
            pos += pad
            offs.append(pos)
            chunks.append(pk)
            pos += len(pk)
        frames = torch.tensor(np.frombuffer(b"".join(chunks) + bytes(16), dtype=np.uint8).copy(),
                              device=dev)
        kw = dict(n=len(pkts), offsets=torch.tensor(np.array(offs, dtype=np.uint32).view(np.int32),
                                                    device=dev),
                  lens=torch.tensor(np.array([len(q) for q in pkts], dtype=np.uint16).view(np.int16),
                                    device=dev))
        staged = []
        for name in ("5tuple_xdp", "checksum_xdp"):
            img = W.program(name)
            prog = Program(img)
            staged.append(prog.batch_staged(prog.make_batch(frames, xdp_md=True, **kw)))
            res = prog.run(frames, r0=True, status=True, xdp_md=True, **kw)
            torch.cuda.synchronize()
            op = oracle.Program(img)
            status = res.status.cpu().numpy()
            r0 = res.r0.cpu().numpy().view(np.uint64)
            for i, pk in enumerate(pkts):
                s, o0, _ = op.run_packet(struct.pack("<II", 8, 8 + len(pk)) + pk, 1024, 512, 1 << 22)
                assert status[i] == s, (name, i)
                if s == 0:
                    assert int(r0[i]) == o0, (name, i)
        out["staged"] = staged
        assert all(staged)
    elif case in ("bin", "bin_default"):
        # a promoted slot-accumulator loop (no byte-sum idiom: the plain loop kernel), length-binned
        # (forced for a small batch) with lanes whose packet reaches the slots deoptimized: the
        # deopt list through the binned order (interp.hip a.perm[slot]) -- ADVICE round 4
        img = assemble(SLOT_XOR)
        prog = Program(img)
        rng = random.Random(9)
        # (bin_default: >= 16384 packets, binned without the switch, host.cpp kBinMinPackets)
        nb = 3001 if case == "bin" else 17001
        lens = [rng.choice([0, 1, 60, 64, 200, 503, 504, 505, 700, 1000]) for _ in range(nb)]
        pkts = [bytes(rng.getrandbits(8) for _ in range(ln)) for ln in lens]
        offs, pos, chunks = [], 0, []
        for pk in pkts:
            pad = (-pos) % 16
            chunks.append(bytes(pad))
            pos += pad
            offs.append(pos)
            chunks.append(pk)
            pos += len(pk)
        buf = np.frombuffer(b"".join(chunks) + bytes(16), dtype=np.uint8).copy()
        frames = torch.tensor(buf, device=dev)
        ln = np.array(lens, dtype=np.uint16)
        kw = dict(n=len(pkts), offsets=torch.tensor(np.array(offs, dtype=np.uint32).view(np.int32),
                                                    device=dev),
                  lens=torch.tensor(ln.view(np.int16), device=dev))
        assert prog.promoted
        out["kernel"] = prog.batch_kernel(prog.make_batch(frames, **kw))
        assert out["kernel"] == _lib.EBPF_KERNEL_JIT_LOOP, out["kernel"]
        cnt = torch.zeros(8, dtype=torch.int64, device=dev)
        res = prog.run(frames, r0=True, status=True, counters=cnt, **kw)
        torch.cuda.synchronize()
        r0, st, ocnt = oracle.Program(img).run_batch(buf, len(pkts), offsets=np.array(offs),
                                                     lens=ln, threads=8)
        got_st = res.status.cpu().numpy()
        assert np.array_equal(got_st, st)
        ok = st == 0
        assert np.array_equal(res.r0.cpu().numpy().view(np.uint64)[ok], r0[ok])
        assert list(cnt.cpu().numpy().view(np.uint64)) == list(ocnt)
        out["deopt_lanes"] = int(sum(1 for x in lens if x > 512 - 8))
    else:
        raise SystemExit(f"unknown case {case}")
    print(json.dumps(out))


# xor-and-shift accumulator kept in the stack slot r10-8 (promote_slots: slot -> register; not a
# byte sum, so no cooperative sum and no deep kernel)
SLOT_XOR = """
    mov r3, 0
    stdw [r10-8], 5
loop:
    jge r3, r2, done
    ldxb r5, [r3+0]
    ldxdw r0, [r10-8]
    lsh r0, 1
    xor r0, r5
    stxdw [r10-8], r0
    add r3, 1
    ja loop
done:
    ldxdw r0, [r10-8]
    exit
"""

if __name__ == "__main__":
    main()
