"""Test configuration: import paths, the ``gpu`` marker, golden-fixture helpers."""

import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "torchao-fork_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device); run with -m gpu")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def bf16(a: np.ndarray) -> torch.Tensor:
    """uint16 bit patterns -> bf16 tensor."""
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16)


def unpack_u8_nibbles(q_u8: np.ndarray) -> torch.Tensor:
    """[N, K/2] bytes (q[2i] << 4 | q[2i+1]) -> int32 [N, K]."""
    q = np.empty((q_u8.shape[0], q_u8.shape[1] * 2), dtype=np.int32)
    q[:, 0::2] = q_u8 >> 4
    q[:, 1::2] = q_u8 & 0xF
    return torch.from_numpy(q)


def load_golden(name: str):
    return np.load(os.path.join(GOLDEN, name))


def golden_files(prefix: str):
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith(prefix) and f.endswith(".npz"))


def golden_ms(rec, key_prefix="x_M"):
    return sorted(int(k[len(key_prefix):]) for k in rec.files if k.startswith(key_prefix))
