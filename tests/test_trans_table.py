"""The gfx950 v_rsq_f32 truth table the oracle models phase 1 of the Jacobi route with
(oracle/tmfwm_oracle.c rsq_hw).  The table (tests/golden/
gfx950_trans_delta.npz) was measured on an MI355X by tools/trans_table.py, which also
checked that every positive normal input follows from it by power-of-two scaling; the GPU
test re-measures it on the box and compares."""
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NPZ = os.path.join(ROOT, "tests", "golden", "gfx950_trans_delta.npz")
TOOL = os.path.join(ROOT, "tools", "micro", "trans_table")


def test_table_shape_and_range():
    with np.load(NPZ) as z:
        rsq, rcp = z["rsq"], z["rcp"]
    assert rsq.shape == (1 << 24,) and rcp.shape == (1 << 23,)
    assert set(np.unique(rsq).tolist()) <= {-1, 0, 1} and set(np.unique(rcp).tolist()) <= {-1, 0, 1}
    # mostly correctly rounded: 89 % of the canonical inputs
    assert (rsq == 0).mean() > 0.85


def test_model_faithful_and_scaled():
    """rsq_hw(x) is within one ulp of 1/sqrt(x) and scales exactly by 4^k."""
    L = O.lib()
    rng = np.random.default_rng(7)
    bits = rng.integers(0x00800000, 0x7F800000, 20000, dtype=np.uint32)
    xs = bits.view(np.float32)
    got = np.array([L.orc_rsq_hw(float(x)) for x in xs], np.float32)
    ref = (1.0 / np.sqrt(xs.astype(np.float64))).astype(np.float32)
    d = got.view(np.uint32).astype(np.int64) - ref.view(np.uint32).astype(np.int64)
    assert np.abs(d).max() <= 1
    for x in xs[:2000]:
        if 2.0 ** -120 < x < 2.0 ** 120:
            assert np.float32(L.orc_rsq_hw(float(x * np.float32(4.0)))) == np.float32(L.orc_rsq_hw(float(x))) / np.float32(2.0)


@pytest.mark.gpu
def test_table_matches_hardware(tmp_path):
    """Re-measure v_rsq_f32 / v_rcp_f32 on this GPU (all 2^31 positive normal inputs checked
    against the scaling model) and compare the canonical tables with the fixture."""
    if not os.path.exists(TOOL):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", TOOL + ".hip", "-o", TOOL], check=True)
    r = subprocess.run(["python3", os.path.join(ROOT, "tools", "trans_table.py"), str(tmp_path)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    st = json.loads(r.stdout.strip().splitlines()[-1])
    assert st["rsq_scaling_mismatches"] == 0 and st["rcp_scaling_mismatches"] == 0
    with np.load(tmp_path / "trans_delta.npz") as a, np.load(NPZ) as b:
        assert np.array_equal(a["rsq"], b["rsq"]) and np.array_equal(a["rcp"], b["rcp"])
