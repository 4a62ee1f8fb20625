"""The library's environment switches: the complete list (every getenv site in
ebpf-emu_amd/csrc), and a test that runs each with the switch set.

After round 5's pruning only diagnostics and test hooks remain (the A/B switches of variants that
were measured slower, and the overrides of defaults, are gone with their code paths):
  EBPFEMU_TRACE=1               per-wave stamps of the compiled kernels (tools/trace_*.py)
  EBPFEMU_TEST_FAIL_STACK_JIT=1 a stack-window program's compile fails (test_stack_tier.py)
  EBPFEMU_BIN=0|1               length binning off / forced for loop programs' offsets batches
  EBPFEMU_XDP_STAGE=1           every xdp_md batch through xdp_stage's copy
  EBPFEMU_FOLD=kernel           counters folded by fold_counters (the path of launches whose
                                per-shard sums could pass 2^48)
  EBPFEMU_FIXED_WGS=n           caps ebpf_tile_jit_fixed's grid (test_gpu_jit.py tile loop re-entry)
  EBPFEMU_VARL_WGS=n            caps ebpf_tile_jit_varl's grid (test_varl.py statement re-entry)
  EBPFEMU_FIXED_OCC=0|1         the fixed-slot kernel's occupancy variant off / for every program
                                (A/B; default: programs of >= 96 micro-ops, test_occ.py)
The first five are read once when the library loads, so their tests run a child process
(tests/knob_child.py); the last two are read per launch.
"""
import json
import os
import re
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "ebpf-emu_amd", "csrc")

KNOBS = {"EBPFEMU_TRACE", "EBPFEMU_TEST_FAIL_STACK_JIT", "EBPFEMU_BIN", "EBPFEMU_XDP_STAGE",
         "EBPFEMU_FOLD", "EBPFEMU_FIXED_WGS", "EBPFEMU_VARL_WGS", "EBPFEMU_FIXED_OCC"}


def test_knob_inventory():
    """Every switch the library reads is one of KNOBS (each tested below or where named above),
    and there are at most 15."""
    found = set()
    for fn in os.listdir(CSRC):
        if fn.endswith((".cpp", ".hip", ".h")):
            with open(os.path.join(CSRC, fn)) as f:
                found |= set(re.findall(r'getenv\("(EBPFEMU_[A-Z0-9_]+)"\)', f.read()))
    assert found == KNOBS, (sorted(found - KNOBS), sorted(KNOBS - found))
    assert len(found) <= 15


def _child(case, env):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, os.path.join(HERE, "knob_child.py"), case,
                        os.path.join(ROOT, "ebpf-emu_amd"), os.path.join(ROOT, "oracle")],
                       capture_output=True, text=True, timeout=170, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_knob_trace():
    """EBPFEMU_TRACE=1: the compiled fixed-slot kernel writes its stamps (ebpf_debug_trace) and
    its outputs are still the oracle's."""
    from ebpf_emu import _lib

    d = _child("trace", {"EBPFEMU_TRACE": "1"})
    assert d["kernel"] in (_lib.EBPF_KERNEL_JIT_FIXED, _lib.EBPF_KERNEL_JIT_FIXED_OCC)
    assert d["stamps_nonzero"] > 0


@pytest.mark.gpu
def test_knob_fold_kernel():
    """EBPFEMU_FOLD=kernel: shard sums folded by fold_counters after the launch; counters ==
    the oracle's."""
    _child("fold", {"EBPFEMU_FOLD": "kernel"})


@pytest.mark.gpu
def test_knob_xdp_stage():
    """EBPFEMU_XDP_STAGE=1: a forward and a loop xdp_md program both staged, outputs == the
    oracle's on the ctx-prefixed images."""
    d = _child("xdp_stage", {"EBPFEMU_XDP_STAGE": "1"})
    assert d["staged"] == [True, True]


@pytest.mark.gpu
def test_knob_bin_with_deopt():
    """EBPFEMU_BIN=1: a promoted (stack-slot) loop program on a small offsets + lens batch,
    length-binned, with lanes whose packet reaches the slots deoptimized to the general
    interpreter through the binned order; status, r0 and counters == the oracle's."""
    d = _child("bin", {"EBPFEMU_BIN": "1"})
    assert d["deopt_lanes"] > 100


@pytest.mark.gpu
def test_binned_deopt_default():
    """The same without the switch: 17 001 packets (>= 16384, binned by default) -- ADVICE round 4:
    a promoted program binned and deoptimizing at once; == the oracle."""
    d = _child("bin_default", {})
    assert d["deopt_lanes"] > 1000


@pytest.mark.parametrize("val,want", [("0", [False, False]), ("1", [True, True])])
def test_knob_fixed_occ(val, want):
    """EBPFEMU_FIXED_OCC=0|1 (read once, at the first compile): acl_rules and the 5-tuple without /
    with code in ebpf_tile_jit_fixed_occ (by default both, test_occ.py)."""
    code = ("import sys; sys.path[:0] = [sys.argv[1], sys.argv[2]]\n"
            "from test_occ import _occ_body\n"
            "from ebpf_emu import Program, workloads as W\n"
            "out = []\n"
            "for name in ('acl_rules', '5tuple'):\n"
            "    p = Program(W.program(name)); p.compile()\n"
            "    out.append(_occ_body(p.jit_asm(1)) is not None)\n"
            "print(out)\n")
    r = subprocess.run([sys.executable, "-c", code, os.path.join(ROOT, "ebpf-emu_amd"), HERE],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, EBPFEMU_FIXED_OCC=val))
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().splitlines()[-1] == str(want)
