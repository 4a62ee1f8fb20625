"""bench.py's multi-rank launcher and its parity pins, on the CPU (no GPU).

`bench.py --gpus N` without WORLD_SIZE starts N rank processes itself (one process per
GPU); EBPFEMU_BENCH_STUB=1 replaces each rank's kernels by its own chunks' fixture counters, so the
spawn, the gloo reduction, the max-over-ranks time, the chunk assignment and the pin check run
here exactly as on a node. The pin fixture itself is checked against the config-4 fixture (both
come from the oracle: tests/golden/make_golden.py).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _bench(args, env_extra, timeout=180):
    env = dict(os.environ, EBPFEMU_BENCH_STUB="1", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


def _pins():
    with open(os.path.join(GOLDEN, "bench_pins.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("n,config", [(2, "5tuple"), (3, "acl"), (2, "checksum"),
                                           (2, "checksum_xdp"), (8, "5tuple"), (2, "acl_rules")])
def test_launcher_spawns_ranks_and_pins(n, config):
    steps = 5
    r = _bench(["--gpus", str(n), "--steps", str(steps), "--config", config], {})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == steps and d["stub"]
    assert d["parity_pinned"] and f"k*{n}+r" in d["parity_pinned"]
    # the summed counters are the fixture's counters of chunks k*n + r, computed independently
    cc = _pins()["programs"][config]["chunk_counters"]
    pool = 1 if config.startswith("checksum") else 8
    want = [0] * 8
    for i in range(steps):
        for rank in range(n):
            want = [a + b for a, b in zip(want, cc[(i % pool) * n + rank])]
    assert d["counters"]["drop"] == want[1] and d["counters"]["pass"] == want[2]
    assert d["counters"]["insns_retired"] == want[7]
    assert want[1] + want[2] + want[3] == steps * n * (1 << 20) or config == "acl"


def test_world_size_must_match_gpus():
    r = _bench(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_failed_rank_fails_the_launch():
    # rank 1 dies before the rendezvous: rank 0 would wait in init forever; the launcher
    # terminates it and returns rank 1's status
    r = _bench(["--gpus", "2", "--steps", "1"], {"EBPFEMU_BENCH_STUB_FAIL": "1"}, timeout=60)
    assert r.returncode == 3


def test_pin_fixture_matches_config4():
    """bench_pins.json's 5-tuple chunks are config4.json's chunks (one seed formula)."""
    with open(os.path.join(GOLDEN, "config4.json")) as f:
        c4 = json.load(f)
    pins = _pins()
    assert pins["chunk"] == c4["chunk"]
    full = [k for k, s in enumerate(c4["chunk_sizes"]) if s == c4["chunk"]]
    assert pins["programs"]["5tuple"]["chunk_counters"][:len(full)] == \
        [c4["chunk_counters"][k] for k in full]
    for name, p in pins["programs"].items():
        for row in p["chunk_counters"]:
            assert sum(row[:7]) == pins["chunk"], name


def test_pin_weak_logic():
    sys.path.insert(0, ROOT)
    import bench

    cc = _pins()["programs"]["5tuple"]["chunk_counters"]
    want, src = bench.pin_weak("5tuple", False, 64, 1 << 20, 1, 8, 3, None)
    assert want == [a + b + c for a, b, c in zip(cc[0], cc[1], cc[2])] and src
    # shapes without a fixture are reported, not pinned
    assert bench.pin_weak("5tuple", False, 1504, 1 << 20, 1, 8, 3, None)[0] is None
    assert bench.pin_weak("5tuple", False, 64, 1 << 16, 1, 8, 3, None)[0] is None
    assert bench.pin_weak("5tuple", False, 64, 1 << 20, 16, 16, 3, None)[0] is None
    # the chunk assignment: disjoint across ranks, 0 .. B*W-1 at any W
    for w in (1, 2, 4, 8):
        ids = sorted(bench.chunk_id(k, r, w) for k in range(8) for r in range(w))
        assert ids == list(range(8 * w))


def test_launcher_strong_scaling_8_ranks():
    """The driver's strong-scaling shape: `bench.py --gpus 8 --total-packets 100000000` (BASELINE
    config 4): 8 rank processes, each its contiguous shard of the 96 seeded chunks; the reduced
    counters equal steps x the config-4 fixture (the pin a real run asserts), and every packet is
    owned by exactly one rank."""
    steps = 2
    r = _bench(["--gpus", "8", "--steps", str(steps), "--total-packets", "100000000"], {},
               timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    with open(os.path.join(GOLDEN, "config4.json")) as f:
        c4 = json.load(f)
    assert d["n_gpus"] == 8 and d["scaling"] == "strong" and d["parity_pinned"]
    assert sum(d["packets_per_rank"]) == 100000000
    assert max(d["packets_per_rank"]) - min(d["packets_per_rank"]) <= 2 * (1 << 20)
    assert d["counters"]["drop"] == steps * c4["counters"][1]
    assert d["counters"]["pass"] == steps * c4["counters"][2]
    assert d["counters"]["insns_retired"] == steps * c4["counters"][7]
