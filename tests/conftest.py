"""Test configuration: import paths, the `gpu` marker, shared fixtures.

`-m "not gpu"` (this container): the oracle against the reference's known answers and golden
vectors, the two restatements against each other, host logic, the C ABI surface, gloo world-2
sharding. `-m gpu` (MI355X box): HIP parity through the C ABI against the oracle and fixtures.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ebpf-emu_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
          ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libebpfemu.so's HIP kernel)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def product_lib():
    from ebpf_emu import _lib

    return _lib.lib()


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test without a visible GPU")
    return torch.device("cuda", 0)
