"""The counter tools behind bench.py's roofline.valu_issue / traffic, run on the committed
round-3 counter passes (profiles/r03/r03j/pmc_b{8,16}, rocprofv3 CSVs of the shipped build)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC = os.path.join(ROOT, "profiles", "r03", "r03j")


def _valu(tmp_path, block):
    out = tmp_path / "valu.json"
    ids = tmp_path / "ids.json"
    ids.write_text(json.dumps({"kernels": {}}))
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "valu.py"), os.path.join(PMC, f"pmc_b{block}"),
                    "--build", "test", "--ids", str(ids), "--out", str(out)], check=True, capture_output=True)
    return json.loads(out.read_text())["kernels"]


def test_valu_embed8_strip_and_list_pass(tmp_path):
    """embed<8>'s strip pass (embed_kernel<8, false>) gives the per-wave figures; its list pass
    (embed_kernel<8, true>) adds its issue cycles to the bound and its bytes to the traffic."""
    k = _valu(tmp_path, 8)
    e = k["embed_kernel<8>"]
    assert e["valu_instr_per_wave"] == 16615.4 and e["waves_per_frame"] == 4050.0
    assert e["list_pass"]["waves"] == 2048.0 and 0.0 < e["list_pass"]["issue_cycles_share"] < 0.05
    assert 75.0 < e["valu_issue_bound_us_per_frame"] < 90.0
    assert 49.9e6 < e["hbm_bytes_per_frame"] < 55e6
    x = k["extract_kernel<8>"]
    assert x["valu_instr_per_wave"] == 3608.2 and "list_pass" not in x


def test_valu_embed16(tmp_path):
    e = _valu(tmp_path, 16)["embed_kernel<16>"]
    assert e["valu_instr_per_wave"] == 39033.4 and "list_pass" not in e
