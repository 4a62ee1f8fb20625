"""Pin the oracle: the reference-embedded KATs and every directed quirk case (tests/cases.py)
against the C oracle AND the independent Python restatement; differential fuzzing of the two
restatements (decode errors, status, steps, all registers and the full memory image)."""
import random

import pytest

import pyref
from cases import CASES, REJECTS
from fuzzgen import gen_packet, gen_program


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_case_c_oracle(oracle_mod, case):
    st, r0, steps = oracle_mod.Program(case.prog).run_packet(case.pkt, case.mem_size, case.r10,
                                                             case.max_steps)
    assert st == case.status, case.cite
    if case.status == 0:
        assert r0 == case.r0, case.cite


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_case_pyref(case):
    st, r0, steps = pyref.run_packet(case.prog, case.pkt, case.mem_size, case.r10, case.max_steps)
    assert st == case.status, case.cite
    if case.status == 0:
        assert r0 == case.r0, case.cite


@pytest.mark.parametrize("rej", REJECTS, ids=[r[0] for r in REJECTS])
def test_rejects(oracle_mod, rej):
    name, img, code, word, cite = rej
    with pytest.raises(oracle_mod.OracleDecodeError) as e1:
        oracle_mod.Program(img)
    with pytest.raises(pyref.DecodeError) as e2:
        pyref.decode(img)
    assert (e1.value.code, e1.value.word) == (code, word) == (e2.value.code, e2.value.word), cite


def test_decoded_fields_match_reference_unit_tests(oracle_mod):
    # ins.rs:373-432 test_wide through the oracle decoder
    img = bytes.fromhex("18000000f0debc9a0000000078563412")
    assert oracle_mod.Program(img).decoded() == [(0, 0x123456789ABCDEF0, 0, 0, 0, 0x18)]


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_c_vs_pyref(oracle_mod, seed):
    rng = random.Random(1000 + seed)
    for it in range(400):
        img = gen_program(rng, valid_only=(it % 4 != 0))
        try:
            op = oracle_mod.Program(img)
            oe = None
        except oracle_mod.OracleDecodeError as e:
            op, oe = None, (e.code, e.word)
        try:
            pyref.decode(img)
            pe = None
        except pyref.DecodeError as e:
            pe = (e.code, e.word)
        assert oe == pe, img.hex()
        if oe:
            continue
        for _ in range(2):
            pkt = gen_packet(rng)
            a = op.run_full(pkt, 1024, 512, 300)
            b = pyref.run_full(img, pkt, 1024, 512, 300)
            assert a[0] == b[0] and a[3] == b[3], (img.hex(), pkt.hex())
            if a[0] == 0:
                assert a[1] == b[1] and a[2] == b[2], (img.hex(), pkt.hex())


def test_batch_equals_single(oracle_mod):
    import numpy as np

    from ebpf_emu import workloads as W

    fr = W.frames_fixed(2000)
    p = oracle_mod.Program(W.program("5tuple"))
    r0, st, cnt = p.run_batch(fr, 2000, stride=64, threads=4)
    for i in range(0, 2000, 37):
        s, r, n = p.run_packet(bytes(fr[i * 64:(i + 1) * 64]))
        assert (s, r) == (st[i], r0[i])
    assert int(cnt[:7].sum()) == 2000
    assert int(cnt[1]) == int((r0 == 1).sum())
    assert np.all(st == 0)


def test_oracle_sanitizers():
    """ASan/UBSan build of the oracle (host code) over 20k random programs: no memory error/UB."""
    import os
    import subprocess

    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    r = subprocess.run(["make", "-C", here, "fuzz_asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + r.stderr[-200:])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0")
    r = subprocess.run([os.path.join(here, "fuzz_asan"), "20000"], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "status histogram" in r.stdout
