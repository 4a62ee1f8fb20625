#!/usr/bin/env python3
"""Diagnostic (round 6): one store-mode program over random fixed-slot packets -- the compiled
route, the general interpreter and the oracle side by side; prints the packets where any two
disagree (r0 / status), with the lane's bytes. usage: tools/debug_store.py <program hex> [stride]"""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ebpf-emu_amd"), os.path.join(ROOT, "oracle")]


def main():
    import torch

    import oracle
    from ebpf_emu import Program, _lib

    img = bytes.fromhex(sys.argv[1])
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    mem, r10 = (1024, 512) if stride <= 128 else (2048, 2048)
    rng = random.Random(1)
    lens = [0, 1, 5, 13, 14, 34, 60, 63, 64, 65, 100, 128]
    pkts = [bytes(rng.getrandbits(8) for _ in range(rng.choice(lens)))[:stride].ljust(stride, b"\0")
            for _ in range(2000)]
    buf = np.frombuffer(b"".join(pkts), dtype=np.uint8).copy()
    fr = torch.from_numpy(buf).cuda()
    p = Program(img)
    b = p.make_batch(fr, n=len(pkts), stride=stride, mem_size=mem, r10=r10)
    print("kernel", _lib.KERNEL_NAMES[p.batch_kernel(b)])
    got = p.run(fr, n=len(pkts), stride=stride, mem_size=mem, r10=r10, r0=True, status=True, regs=True)
    gen = p.run(fr, n=len(pkts), stride=stride, mem_size=mem, r10=r10, r0=True, status=True, regs=True,
                generic=True)
    torch.cuda.synchronize()
    op = oracle.Program(img)
    bad = 0
    gr, gs = got.regs.cpu().numpy().view(np.uint64), got.status.cpu().numpy()
    nr, ns = gen.regs.cpu().numpy().view(np.uint64), gen.status.cpu().numpy()
    for i, pk in enumerate(pkts):
        st, regs, _, _ = op.run_full(pk, mem, r10, 1 << 22)
        if gs[i] != st or ns[i] != st or (st == 0 and (list(gr[i]) != regs or list(nr[i]) != regs)):
            bad += 1
            if bad <= 6:
                print(f"pkt {i}: status compiled {gs[i]} generic {ns[i]} oracle {st}")
                for r in range(11):
                    if st == 0 and (gr[i][r] != regs[r] or nr[i][r] != regs[r]):
                        print(f"  r{r}: compiled {int(gr[i][r]):#x} generic {int(nr[i][r]):#x} "
                              f"oracle {regs[r]:#x}")
                print("  bytes", pk[:128].hex())
    print("mismatching packets:", bad, "of", len(pkts))


if __name__ == "__main__":
    main()
