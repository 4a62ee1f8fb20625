"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo): each rank owns a contiguous
shard of a chunked global batch, computes its counters (the oracle stands in for the kernel, as
this container has no GPU), and the single exchange step -- the counter all-reduce -- must give
exactly the single-process totals; the verdict shards concatenate to the single-process array."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CHUNK = 3000
TOTAL = 4 * CHUNK + 777  # ragged last chunk


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "ebpf-emu_amd"), os.path.join(root, "oracle")]
    import oracle
    from ebpf_emu import dist as D
    from ebpf_emu import workloads as W

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prog = oracle.Program(W.program("5tuple"))
    sizes = D.chunk_sizes(TOTAL, CHUNK)
    counters = torch.zeros(8, dtype=torch.int64)
    verdicts = []
    for k in D.shard_chunks(len(sizes), world, rank):
        buf = D.chunk_frames(k, sizes[k])
        r0, st, cnt = prog.run_batch(buf, sizes[k], stride=64, threads=2)
        counters += torch.from_numpy(cnt.view(np.int64))
        verdicts.append(np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8))
    D.reduce_counters(counters)
    np.save(os.path.join(out_dir, f"v{rank}.npy"),
            np.concatenate(verdicts) if verdicts else np.zeros(0, np.uint8))
    if rank == 0:
        np.save(os.path.join(out_dir, "counters.npy"), counters.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_counters_match_single_process(tmp_path, oracle_mod, world):
    from ebpf_emu import dist as D
    from ebpf_emu import workloads as W

    port = _free_port()
    mp.start_processes(_rank_main, args=(world, port, str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    got = np.load(tmp_path / "counters.npy").view(np.uint64)
    prog = oracle_mod.Program(W.program("5tuple"))
    total = np.zeros(8, np.uint64)
    ref_v = []
    for k, sz in enumerate(D.chunk_sizes(TOTAL, CHUNK)):
        buf = D.chunk_frames(k, sz)
        r0, st, cnt = prog.run_batch(buf, sz, stride=64, threads=2)
        total += cnt
        ref_v.append(np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8))
    assert list(got) == list(total)
    assert int(got[:7].sum()) == TOTAL
    shards = np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(world)])
    assert np.array_equal(shards, np.concatenate(ref_v))


def test_shard_ranges_partition():
    from ebpf_emu.dist import chunk_sizes, shard_chunks

    for k in (1, 7, 8, 100):
        for w in (1, 2, 3, 8):
            seen = [i for r in range(w) for i in shard_chunks(k, w, r)]
            assert seen == list(range(k))
            lens = [len(shard_chunks(k, w, r)) for r in range(w)]
            assert max(lens) - min(lens) <= 1
    assert chunk_sizes(10, 4) == [4, 4, 2]
    assert sum(chunk_sizes(100_000_000, 1 << 20)) == 100_000_000
