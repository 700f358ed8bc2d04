"""The list passes' segmented list (tmfwm_internal.h shard_base): built for the
host from the header the kernels use, checked for exact capacity over block-row counts below,
at and above the segment count (the GPU side: test_gpu_parity.py::test_list_pass_segments_vs_oracle)."""
import ctypes
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "shard_host.cpp")
HDR = os.path.join(ROOT, "thatsmyface_amd", "csrc", "tmfwm_internal.h")
OUT = os.path.join(ROOT, "tests", "_build", "libshard_host.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(HIPCC) and not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        tmp = f"{OUT}.{os.getpid()}.tmp"
        subprocess.run([HIPCC, "-O2", "-std=c++17", "-fPIC", "-x", "hip", "--offload-arch=gfx950", "-shared", "-o", tmp, SRC],
                       check=True)
        os.replace(tmp, OUT)
    L = ctypes.CDLL(OUT)
    L.shard_check.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.shard_count.restype = ctypes.c_uint32
    return L


def test_segments_partition_the_list_exactly(lib):
    K = lib.shard_count()
    assert K == 2048
    # 4K at b = 4 (540 rows, 960 blocks per row) up to the chunk sizes the C-ABI plans
    for rows in (1, 2, 17, K - 1, K, K + 1, 2 * K - 1, 3 * K + 5, 540 * 64, 270 * 4096, 135 * 65535):
        for nbw in (1, 3, 240, 960):
            if rows * nbw < 2**32:
                assert lib.shard_check(rows, nbw) == 0, (rows, nbw)
