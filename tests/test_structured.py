"""oracle/structured.py (the reference's cost model, bench.py's CPU baseline) computes the
reference's bytes: it calls the same numpy / scipy / OpenBLAS routines in the same loops,
so on this container's OpenBLAS core (SkylakeX) it must reproduce the golden fixtures."""
import numpy as np
import pytest

from oracle import structured as S
from test_oracle_lapack import needs_skylakex


def _rgb(a):
    return np.repeat(a[..., None], 3, -1) if a.ndim == 2 else np.ascontiguousarray(a[..., :3])


@needs_skylakex
@pytest.mark.parametrize("name", ["kat_a", "kat_b", "noise_128x96_pr", "flat_64x80", "black_96", "rgba_72x64",
                                  "diag_100x140_b4"])
def test_structured_matches_reference_fixtures(golden, name):
    cases, meta = golden
    m = meta["cases"][name]
    cov = _rgb(cases[f"{name}/cover"])
    emb = S.embed(cov, cases[f"{name}/tile"], m["block"], m["alpha"])
    assert np.array_equal(emb, cases[f"{name}/embed"]), name
    assert np.array_equal(S.extract(emb, cov, m["block"], m["alpha"]), cases[f"{name}/extract"]), name


def test_structured_pool_runs():
    """The process pool the bench uses (spawned children, single-threaded OpenBLAS)."""
    rng = np.random.default_rng(0)
    covers = [rng.integers(0, 256, (32, 48, 3), dtype=np.uint8) for _ in range(2)]
    tiles = [rng.integers(0, 256, (4, 6), dtype=np.uint8) for _ in range(2)]
    res, wall = S.run_pool(covers, tiles, 8, 0.1, 2)
    assert len(res) == 2 and wall > 0
    for (dt, out, ext), c, t in zip(res, covers, tiles):
        assert dt > 0
        assert np.array_equal(out, S.embed(c, t, 8, 0.1))
        assert np.array_equal(ext, S.extract(out, c, 8, 0.1))
