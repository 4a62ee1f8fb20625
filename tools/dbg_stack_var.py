"""Debug: a var-layout stack-program run (tests/test_stack_tier.py) -- print register mismatches
between the compiled kernel and the general interpreter / oracle, with the packet lengths.
usage: dbg_stack_var.py <seed-bytes> <layout> <n_iters> <nmin> <nmax> <pw_every>"""
import os
import random
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ebpf-emu_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fuzzgen import gen_stack_program  # noqa: E402
from test_stack_tier import VAR_LAYOUTS, _run_var, _var_packets, _images_of  # noqa: E402
from ebpf_emu import Program, _lib  # noqa: E402
import oracle  # noqa: E402

seed, layout, iters, nmin, nmax = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
dev = torch.device("cuda", 0)
rng = random.Random(zlib.crc32(seed.encode() + layout.encode()))
for it in range(iters):
    kw = dict(n=rng.randrange(nmin, nmax)) if nmax > 0 else {}
    img = gen_stack_program(rng, pw_atomics=it % 2 == 1, **kw)
    if nmax <= 0:
        try:
            oracle.Program(img)
        except oracle.OracleDecodeError:
            continue
    p = Program(img)
    k = p.stack_window
    p.close()
    if not k:
        continue
    pkts = _var_packets(rng, 100) if nmax > 0 else _var_packets(rng, rng.choice([64, 100, 130]))
    got, xdp = _run_var(img, pkts, dev, VAR_LAYOUTS[layout])
    ref, _ = _run_var(img, pkts, dev, VAR_LAYOUTS[layout], generic=True)
    bad = np.nonzero((got["regs"] != ref["regs"]).any(axis=1) & (got["status"] != 7))[0]
    if len(bad):
        i = bad[0]
        print(layout, "it", it, "k", k, "kernel", _lib.KERNEL_NAMES[got["kernel"]], "bad", list(bad[:12]),
              "lens", [len(pkts[j]) for j in bad[:12]])
        print(" prog", img.hex())
        op = oracle.Program(img)
        st, oregs, _, _ = op.run_full(_images_of(pkts, xdp)[i], 1024, 512, 20000)
        for r in range(11):
            if got["regs"][i][r] != ref["regs"][i][r] or oregs[r] != ref["regs"][i][r]:
                print(f"  r{r}: compiled {int(got['regs'][i][r]):#x} general {int(ref['regs'][i][r]):#x} oracle {oregs[r]:#x}")
        p = Program(img)
        p.compile()
        with open(f"gpurun_out/dbg_{layout}_{it}.s", "w") as f:
            f.write(p.jit_asm(1))
        p.close()
print("done")
