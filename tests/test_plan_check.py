"""The host-side launch plans (csrc/fu_plan.cpp: tile lists, row classes, kernel 8 slice
layouts, kernel 9 staging / transpose tables, the kernel-9 launch partition) against a CPU
replay of every kernel's index arithmetic (tools/plan_check.cpp), built with AddressSanitizer
and UndefinedBehaviorSanitizer. No GPU: this runs in the CPU suite.

Covers every golden fixture graph (CA:105-128 on those graphs is pinned bitwise by the GPU
suite) and R-MAT scales 9-15, both node numberings, mega-hub thresholds 64 / 300 / 8192, the
forced heavy path and a rank's view with ghost slots: each table index in range, each row computed
by exactly one launch, each flow written once, each edge's pre-gathered estimate its own
neighbour's."""
import os
import subprocess

import numpy as np
import pytest

import fu
from conftest import ROOT, ca_sync_fixtures, load_npz

BIN = os.path.join(ROOT, "tools", "bin", "plan_check")
MEGAS = ["--mega", "64", "--mega", "300", "--mega", "8192"]


@pytest.fixture(scope="module")
def plan_check():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), "bin/plan_check"], check=True)
    return BIN


def _write_csr(path, rowptr, col):
    with open(path, "wb") as f:
        np.array([len(rowptr) - 1, int(rowptr[-1])], dtype=np.int64).tofile(f)
        np.asarray(rowptr, dtype=np.int64).tofile(f)
        np.asarray(col, dtype=np.int32).tofile(f)


def _run(binary, args):
    p = subprocess.run([binary] + args, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
                                UBSAN_OPTIONS="print_stacktrace=1"))
    assert p.returncode == 0, p.stdout + p.stderr[-4000:]
    assert "0 failed" in p.stdout, p.stdout
    return p.stdout


@pytest.mark.parametrize("layout", ["given", "degree"])
@pytest.mark.parametrize("name,meta", ca_sync_fixtures())
def test_fixture_graph_plans(plan_check, tmp_path, name, meta, layout):
    d = load_npz(meta["file"])
    f = str(tmp_path / "g.bin")
    _write_csr(f, d["rowptr"], d["col"])
    _run(plan_check, ["--csr", f, "--layout", layout, "--ht", "128", "--ht", "3"]
         + MEGAS)


@pytest.mark.parametrize("layout", ["given", "degree"])
@pytest.mark.parametrize("scale,ef", [(9, 8), (10, 16), (11, 16), (12, 16), (13, 16), (14, 16), (15, 16)])
def test_rmat_plans(plan_check, scale, ef, layout):
    hts = ["--ht", "128"] if scale >= 14 else ["--ht", "128", "--ht", "16"]
    _run(plan_check, ["--rmat", str(scale), str(ef), str(scale), "--layout", layout] + MEGAS + hts)


def test_er_plans(plan_check):
    """ER with > 64 slices per kernel 8 layout width (kernel 8 then builds only some layouts)."""
    _run(plan_check, ["--er", "200000", "800000", "5"])


def _edges_graph(n, src, dst):
    return fu.Graph.from_edges(n, np.asarray(src), np.asarray(dst))


@pytest.mark.parametrize("tail", ["heavy_hub", "hub_iso_heavy", "iso_end"])
def test_isolated_rows_before_heavy_rows(plan_check, tmp_path, tail):
    """The iso_rows case (fixed in round 5): trailing degree-0 light tiles right before a heavy
    row and a mega hub (layout "given") must stay light tiles; k_isolated takes only the
    trailing run of degree-0 rows."""
    rng = np.random.default_rng(21)
    n_leaf, n_iso = 12000, 700
    base = rng.integers(0, n_leaf, size=(3 * n_leaf, 2))
    if tail == "heavy_hub":
        heavy, hub = n_leaf + n_iso, n_leaf + n_iso + 1
    elif tail == "hub_iso_heavy":
        hub, heavy = n_leaf, n_leaf + 1 + n_iso
    else:
        heavy, hub = n_leaf, n_leaf + 1
    n = n_leaf + n_iso + 2
    g = _edges_graph(n, np.concatenate([base[:, 0], np.full(300, heavy), np.full(9000, hub)]),
                     np.concatenate([base[:, 1], rng.choice(n_leaf, 300, replace=False),
                                     rng.choice(n_leaf, 9000, replace=False)]))
    f = str(tmp_path / "g.bin")
    _write_csr(f, g.rowptr, g.col)
    _run(plan_check, ["--csr", f] + MEGAS)


@pytest.mark.parametrize("case", ["single", "pair", "star", "path_iso", "two_hubs"])
def test_tiny_graph_plans(plan_check, tmp_path, case):
    """Graphs smaller than one transpose bucket, one stage piece, one tile (the kernel-9 case
    of the round-4 abort: rmat9_ef8 has 5,654 edges, under one 8,192-edge bucket)."""
    if case == "single":
        rp, col = np.array([0, 0]), np.array([], dtype=np.int32)
    elif case == "pair":
        rp, col = np.array([0, 1, 2]), np.array([1, 0])
    elif case == "star":
        g = _edges_graph(600, np.zeros(599, dtype=np.int32), np.arange(1, 600))
        rp, col = g.rowptr, g.col
    elif case == "path_iso":
        g = _edges_graph(50, np.arange(0, 20), np.arange(1, 21))
        rp, col = g.rowptr, g.col
    else:
        g = _edges_graph(1000, np.r_[np.zeros(400), np.full(500, 999)].astype(np.int32),
                         np.r_[np.arange(1, 401), np.arange(400, 900)])
        rp, col = g.rowptr, g.col
    f = str(tmp_path / "g.bin")
    _write_csr(f, rp, col)
    for layout in ("given", "degree"):
        _run(plan_check, ["--csr", f, "--layout", layout, "--ht", "128", "--ht", "3"]
             + MEGAS)


def test_autotune_pass_rounds_rank_independent(plan_check):
    """Multi-GPU: an autotune pass runs the same number of rounds on every rank whatever the
    rank-local state (forced candidate drops from its own timings, kernel 8 / 9 layouts missing
    on its graph): each round is a halo exchange, so a mismatch would hang RCCL at N > 1
    instead of failing (CA:74, CA:124). The engine asserts the same count at run time."""
    out = _run(plan_check, ["--tune"])
    assert "4096 rank states, 36 rounds per multi-GPU pass" in out


@pytest.mark.parametrize("args", [["--rmat", "12", "16", "3", "--ghosts", "1000"],
                                  ["--rmat", "14", "16", "3", "--ghosts", "4000", "--ht", "32", "--mega", "256"],
                                  ["--er", "100000", "400000", "5", "--ghosts", "20000"]])
def test_rank_view_plans(plan_check, args):
    """A multi-GPU rank's view (the last ids as ghost estimate slots, na > n): the boundary light
    tiles lead, the staging slices cover the ghost slots, kernel 9's transposes deliver ghost
    estimates to their edges (kernels 4, 8 and 9 all run partitioned)."""
    extra = [] if "--mega" in args else MEGAS
    _run(plan_check, args + extra)
