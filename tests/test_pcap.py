"""Host ingestion of classic pcap captures (ebpf_pcap_index, ebpf_emu.pcap): the record index on
the CPU, and a capture streamed through the GPU in chunks against the oracle on the same bytes."""
import random
import struct

import numpy as np
import pytest

from ebpf_emu import _lib, pcap


def _packets(seed, n, lens=(0, 1, 14, 60, 64, 65, 100, 1500)):
    rng = random.Random(seed)
    return [bytes(rng.getrandbits(8) for _ in range(rng.choice(lens))) for _ in range(n)]


@pytest.mark.parametrize("big_endian", [False, True])
@pytest.mark.parametrize("nanos", [False, True])
def test_index_round_trip(big_endian, nanos):
    pk = _packets(1, 300)
    buf = pcap.to_bytes(pk, nanos=nanos, big_endian=big_endian, linktype=1)
    offs, lens, lt = pcap.index(buf)
    assert lt == 1 and len(offs) == len(pk)
    for o, ln, p in zip(offs.tolist(), lens.tolist(), pk):
        assert buf[o:o + ln] == p
    # records are contiguous: header (16 bytes) + data
    assert offs[0] == 24 + 16
    assert all(int(offs[i + 1]) == int(offs[i]) + int(lens[i]) + 16 for i in range(len(pk) - 1))


def test_index_errors():
    good = pcap.to_bytes(_packets(2, 5))
    with pytest.raises(_lib.EbpfError) as e:
        pcap.index(b"\x00" * 24)  # bad magic
    assert e.value.code == _lib.EBPF_EPCAP
    with pytest.raises(_lib.EbpfError) as e:
        pcap.index(good[:-1])  # truncated last record
    assert e.value.code == _lib.EBPF_EPCAP
    with pytest.raises(_lib.EbpfError) as e:
        pcap.index(good[:24] + struct.pack("<IIII", 0, 0, 70000, 70000) + bytes(70000))
    assert e.value.code == _lib.EBPF_ETOOBIG
    assert len(pcap.index(good[:24])[0]) == 0  # header only: no records


def test_index_cap():
    import ctypes

    buf = np.frombuffer(pcap.to_bytes(_packets(3, 10)), dtype=np.uint8)
    offs = np.zeros(4, dtype=np.uint32)
    lens = np.zeros(4, dtype=np.uint16)
    n = ctypes.c_size_t(0)
    rc = _lib.lib().ebpf_pcap_index(buf.ctypes.data, buf.nbytes, offs.ctypes.data,
                                    lens.ctypes.data, 4, ctypes.byref(n), None)
    assert rc == _lib.EBPF_EINVAL and n.value == 10  # the first 4 indexed, all 10 counted
    full, _, _ = pcap.index(buf)
    assert list(offs) == list(full[:4])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["5tuple", "checksum"])
def test_capture_through_gpu(cuda, oracle_mod, name):
    """A capture of mixed frames, streamed in small chunks (so that copies, kernels and verdict
    copies overlap across buffers): every verdict and the counters equal the oracle's."""
    from ebpf_emu import Program
    from ebpf_emu import workloads as W

    pk = _packets(4, 5000, lens=(0, 14, 34, 60, 64, 65, 128, 600, 1500))
    buf = pcap.to_bytes(pk)
    cap = pcap.Capture(buf)
    img = W.program(name)
    prog = Program(img)
    verdict, counters = cap.run(prog, packets_per_chunk=777, mem_size=2048, r10=2048)
    offs, lens, _ = pcap.index(buf)
    r0, st, cnt = oracle_mod.Program(img).run_batch(np.frombuffer(buf, dtype=np.uint8), len(pk),
                                                    offsets=offs, lens=lens, mem_size=2048,
                                                    r10=2048, threads=8)
    want = np.where(st != 0, 0xFF, np.where(r0 < 5, r0, 0xFE)).astype(np.uint8)
    assert np.array_equal(verdict.numpy(), want)
    assert [int(c) for c in counters.cpu().numpy().view(np.uint64)] == [int(c) for c in cnt]
