"""Mega hubs (rows above the "mega_hub" degree) with the parallel exact sums (hub_scan = 1)
and with the one-wave chain (hub_scan = 0, the default): both must give the bits of the
sequential left-to-right sums of avg_and_send (flowupdating-collectall.py:106, 110). The
value sets include adversarial ones for the speculation: dyadic values (exact zeros,
powers of two, rounding ties), a huge dynamic range, and values that cancel to ~0."""
import numpy as np
import pytest

import coracle
import fu

pytestmark = pytest.mark.gpu


def _star_er(n_er, leaves, seed):
    er = fu.Graph.erdos_renyi(n_er, 4 * n_er, seed=seed)
    src = np.repeat(np.arange(er.n), np.diff(er.rowptr))
    keep = src < er.col
    hub = n_er + leaves
    s = np.concatenate([src[keep], np.full(leaves, hub), [0]])
    d = np.concatenate([er.col[keep], n_er + np.arange(leaves), [hub]])
    return fu.Graph.from_edges(hub + 1, s, d)


def _values(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        return fu.uniform_values(n, seed=seed)
    if kind == "dyadic":  # small dyadic rationals: exact sums, exact zeros, ties
        return rng.integers(-4, 5, n).astype(np.float64) / 8.0
    if kind == "range":  # |v| from 1e-30 to 1e30, both signs
        return rng.choice([-1.0, 1.0], n) * 10.0 ** rng.uniform(-30, 30, n)
    if kind == "cancel":  # +-1 plus tiny noise: partial sums wander through ~0
        return rng.choice([-1.0, 1.0], n) * (1.0 + rng.uniform(0, 1e-12, n))
    raise ValueError(kind)


def _run(g, v, rounds, **opts):
    eng = fu.CollectAll(g, v, kernel="recon")
    for k, val in opts.items():
        eng.set_option(k, val)
    eng.run(rounds)
    info = eng.info()
    return eng.estimates(), eng.flows(), info


@pytest.mark.parametrize("kind", ["uniform", "dyadic", "range", "cancel"])
def test_star_hub_scan_bitwise(kind):
    g = _star_er(20_000, 60_000, seed=21)
    v = _values(kind, g.n, 21)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 30, nthreads=16)
    for scan in (1, 0):
        a, f, info = _run(g, v, 30, hub_scan=scan)
        assert np.array_equal(a, a_ref, equal_nan=True), (kind, scan)
        assert np.array_equal(f, f_ref, equal_nan=True), (kind, scan)
        assert info["mega_hubs"] == 1 and info["hub_pieces"] == 30
        if scan and kind == "uniform":  # the speculation mostly holds: few pieces redone
            # (the star's flow sums wander around zero: ~6% of the S steps change binade,
            # which overflows the boundary list of about a third of the S pieces)
            assert info["hub_pieces_redone"] < 0.4 * 30 * 2 * 29, info


@pytest.mark.parametrize("tile", [2048, 512])
def test_rmat_many_mega_hubs_scan_bitwise(tile):
    """Many mega hubs (threshold 300), packed rounds included, every piece boundary shape."""
    g = fu.Graph.rmat(15, 16, seed=9)
    v = fu.uniform_values(g.n, seed=9)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 120, nthreads=16)
    for scan in (1, 0):
        a, f, info = _run(g, v, 120, tile_edges=tile, mega_hub=300, hub_threshold=16, pack_every=4,
                          hub_scan=scan)
        assert info["mega_hubs"] > 10
        assert (info["hub_pieces_redone"] > 0) == (scan == 1)  # converged flow sums: some redone
        assert np.array_equal(a, a_ref)
        assert np.array_equal(f, f_ref)


def test_hub_scan_degree_layout():
    g = fu.Graph.rmat(16, 16, seed=4)
    v = fu.uniform_values(g.n, seed=4)
    eng = fu.CollectAll(g, v, kernel="recon", layout="degree")
    eng.set_option("mega_hub", 1000)
    eng.set_option("hub_scan", 1)
    eng.run(60)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 60, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


@pytest.mark.parametrize("fork", [1, 0])
@pytest.mark.parametrize("kind", ["all_heavy", "mixed"])
def test_heavy_light_split_launches(fork, kind):
    """Kernel 4 runs heavy tiles (hubs, heavy rows) as their own launch on a side stream and
    light tiles as a light-only launch (fork_heavy 1), or both in order on one stream
    (fork_heavy 0). Graphs with only heavy rows and with both must give the oracle's bits."""
    if kind == "all_heavy":  # K_300: every row has degree 299 > hub_threshold
        n = 300
        iu = np.triu_indices(n, 1)
        g = fu.Graph.from_edges(n, iu[0].astype(np.int32), iu[1].astype(np.int32))
    else:
        g = _star_er(5_000, 12_000, seed=5)
    v = fu.uniform_values(g.n, seed=5)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 40, nthreads=16)
    for tile in (2048, 1024, 512):
        a, f, _ = _run(g, v, 40, fork_heavy=fork, tile_edges=tile, mega_hub=256)
        assert np.array_equal(a, a_ref), (kind, fork, tile)
        assert np.array_equal(f, f_ref), (kind, fork, tile)
