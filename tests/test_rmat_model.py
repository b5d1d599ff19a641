"""tools/rmat_model.py (the R-MAT byte-and-time model behind DESIGN.md §4.12) runs on a small
graph and prices every design it reports: kernel 9 per launch, its floor, and the two
structural alternatives with their gate verdicts (CPU only)."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def test_rmat_model_small_scale(tmp_path):
    out = tmp_path / "m.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rmat_model.py"), "--scale", "14",
                    "--out", str(out)], check=True, capture_output=True, text=True, timeout=300)
    rep = json.loads(out.read_text())
    assert rep["n"] == 1 << 14 and rep["E"] > 0
    assert abs(sum(c["edge_share"] for c in rep["classes"].values()) - 1.0) < 1e-9
    assert all(v["GB"] >= 0 for v in rep["kernel9_model"].values())  # no mega hubs at this scale
    assert rep["kernel9_model"]["k_stage"]["GB"] > 0 and rep["kernel9_model"]["k_transpose"]["GB"] > 0
    assert 0 < rep["kernel9_floor"]["GB"] <= rep["kernel9_model_total_GB"]
    alts = [k for k in rep if k.startswith("alt_")]
    assert len(alts) >= 2 and set(rep["verdict"]) == set(alts)  # rows of 257-8192 edges at least
    for k in alts:
        assert rep[k]["GB"] > 0 and rep[k]["ms"] > 0
