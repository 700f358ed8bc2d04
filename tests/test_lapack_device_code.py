"""The GPU's dgesdd route (thatsmyface_amd/csrc/tmfwm_lapack.h) compiled for the host CPU
and checked against the oracle's restatement (oracle/tmfwm_lapack.c) -- the same source
the fallback kernels run, exercised here without a GPU.  The GPU run of it is covered by
tests/test_gpu_parity.py (test_lapack_*_gpu)."""
import ctypes
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "lp_host.cpp")
HDR = os.path.join(ROOT, "thatsmyface_amd", "csrc", "tmfwm_lapack.h")
OUT = os.path.join(ROOT, "tests", "_build", "liblp_host.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def host():
    if not os.path.exists(HIPCC) and not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        tmp = f"{OUT}.{os.getpid()}.tmp"  # pytest-xdist workers may build at once: write aside, rename
        subprocess.run([HIPCC, "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-x", "hip",
                        "--offload-arch=gfx950", "-shared", "-o", tmp, SRC], check=True)
        os.replace(tmp, OUT)
    L = ctypes.CDLL(OUT)
    L.lp_host_dnrm2.restype = ctypes.c_double
    L.lp_host_dnrm2.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    L.lp_host_svd_blocks.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def test_x87_dnrm2_emulation(host):
    """Integer emulation of the x87 squares / sums / fsqrt / store vs long double."""
    rng = np.random.default_rng(0)
    for inc in (1, 3):
        for n in range(0, 41):
            for _ in range(100):
                x = rng.standard_normal(max(n * inc, 1)) * 10.0 ** rng.integers(-150, 150)
                a, b = host.lp_host_dnrm2(n, _p(x), inc), O.lp_dnrm2(x[: n * inc], inc)
                assert np.float64(a).view(np.uint64) == np.float64(b).view(np.uint64), (n, inc)


@pytest.mark.parametrize("reverse", [0, 1])
@pytest.mark.parametrize("b", [4, 6, 8, 10, 12, 14, 16])
def test_device_route_equals_oracle_route(host, b, reverse):
    """reverse=1 runs every per-element loop backwards: the wave-parallel form of the route
    (one element per lane) is only valid if no element's result depends on another's."""
    from test_oracle_lapack import KINDS, _cover_blocks

    for kind in KINDS:
        D = _cover_blocks(kind, b)
        nb = len(D)
        U, Vt, S = np.empty_like(D), np.empty_like(D), np.empty((nb, b), np.float32)
        assert host.lp_host_svd_blocks(_p(D), nb, b, _p(U), _p(S), _p(Vt), 1, reverse) == 0
        u, s, vt = O.lp_svd_blocks(D)
        for x, y in ((U, u), (S, s), (Vt, vt)):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (b, kind)
        S2 = np.empty((nb, b), np.float32)
        assert host.lp_host_svd_blocks(_p(D), nb, b, None, _p(S2), None, 0, reverse) == 0
        assert np.array_equal(S2.view(np.uint32), s.view(np.uint32)), (b, kind)


def test_tolerance_constant_is_glibc_pow():
    """dbdsqr's TOLMUL = eps**(-1/8) comes from gfortran's pow (glibc); the device header
    hard-codes its bits."""
    src = open(HDR).read()
    m = re.search(r"kTolmul = (0x[0-9a-fp.+-]+);", src)
    assert m and float.fromhex(m.group(1)) == (2.0**-53) ** -0.125


def test_workspace_bounds_asan(tmp_path):
    """The route's workspace indexing stays inside ws_doubles(n) -- the LDS size the fixup
    kernels give it -- for every n = 1..16 and eight input classes (noise, rank-deficient,
    zero, tiny / huge scale, ties, a single entry, graded rows), under both host policies:
    tests/native/lp_asan.cpp under AddressSanitizer, every array its own exact-size heap
    allocation (the b = 16 fault of the round-2 serial code)."""
    if not os.path.exists(HIPCC) and not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    exe = tmp_path / "lp_asan"
    src = os.path.join(ROOT, "tests", "native", "lp_asan.cpp")
    subprocess.run([HIPCC, "-x", "hip", "--cuda-host-only", "-O1", "-g", "-std=c++17", "-ffp-contract=off",
                    "-Xarch_host", "-fsanitize=address", "-fno-omit-frame-pointer", src, "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"cases": 2048' in r.stdout and '"not_converged": 0' in r.stdout, r.stdout
    # the compact workspace of the b > 8 embed pass: in bounds, same bits as the standard layout
    assert '"compact_cases": 256' in r.stdout and '"compact_mismatches": 0' in r.stdout, r.stdout
