"""Debug: the var-stack fuzz (tests/test_stack_tier.py) -- print the first register mismatch
between the compiled var-stack kernel and the general interpreter, with the packet."""
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

dev = torch.device("cuda", 0)
for layout in sys.argv[1:] or ["offsets16"]:
    rng = random.Random(zlib.crc32(layout.encode()))
    shown = 0
    for it in range(30):
        img = gen_stack_program(rng, pw_atomics=it % 2 == 1)
        try:
            oracle.Program(img)
        except oracle.OracleDecodeError:
            continue
        p = Program(img)
        k = p.stack_window
        p.close()
        if not k:
            continue
        pkts = _var_packets(rng, rng.choice([64, 100, 130]))
        got, xdp = _run_var(img, pkts, dev, VAR_LAYOUTS[layout])
        ref, _ = _run_var(img, pkts, dev, VAR_LAYOUTS[layout], generic=True)
        bad = np.nonzero((got["regs"] != ref["regs"]).any(axis=1) & (got["status"] != 7))[0]
        if len(bad) and shown < 3:
            shown += 1
            i = bad[0]
            print(layout, "it", it, "k", k, "kernel", _lib.KERNEL_NAMES[got["kernel"]], "bad lanes", list(bad[:10]),
                  "lens", [len(pkts[j]) for j in bad[:10]])
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
