"""Node relabelling (fu_graph_relabel, layout "degree"): rows move as blocks and keep their
neighbour order, the summation order of avg_and_send (flowupdating-collectall.py:106, 110),
so every node computes the same bits under any numbering. CPU tests run the C oracle on both
numberings; the GPU test runs the engine with layout "degree" against the C oracle on the
caller's numbering."""
import numpy as np
import pytest

import coracle
import fu


def _check_relabelled(g, h, perm):
    rp, col, rev = g.arrays()
    rp2, col2, rev2 = h.arrays()
    assert sorted(perm.tolist()) == list(range(g.n))
    for i in range(g.n):
        p = perm[i]
        assert np.array_equal(col2[rp2[p]:rp2[p + 1]], perm[col[rp[i]:rp[i + 1]]])
    k = np.arange(h.E)
    assert np.array_equal(rev2[rev2], k)
    src2 = np.repeat(np.arange(h.n), np.diff(rp2))
    assert np.array_equal(col2[rev2], src2)


@pytest.mark.parametrize("mk", [lambda: fu.Graph.rmat(10, 8, seed=5),
                                lambda: fu.Graph.erdos_renyi(3000, 9000, seed=5)])
def test_degree_relabel_structure(mk):
    g = mk()
    h, perm = g.relabel("degree")
    _check_relabelled(g, h, perm)
    d2 = h.degrees
    assert np.all(d2[:-1] >= d2[1:])  # degree descending
    assert h.max_deg == g.max_deg and h.E == g.E


def test_given_relabel_and_bad_permutation():
    g = fu.Graph.random_regular(500, 6, seed=2)
    perm = np.random.default_rng(0).permutation(g.n).astype(np.int32)
    h, p2 = g.relabel("given", perm)
    assert np.array_equal(p2, perm)
    _check_relabelled(g, h, perm)
    bad = perm.copy()
    bad[0] = bad[1]
    with pytest.raises(RuntimeError):
        g.relabel("given", bad)


def test_relabelled_rounds_are_bitwise_the_same():
    g = fu.Graph.rmat(11, 8, seed=7)
    v = fu.uniform_values(g.n, seed=7)
    h, perm = g.relabel("degree")
    v2 = np.empty_like(v)
    v2[perm] = v
    a, f = coracle.ca_sync(*g.arrays(), v, 40)
    a2, f2 = coracle.ca_sync(*h.arrays(), v2, 40)
    assert np.array_equal(a2[perm], a)
    rp, rp2 = g.rowptr, h.rowptr
    f_back = np.concatenate([f2[rp2[perm[i]]:rp2[perm[i] + 1]] for i in range(g.n)])
    assert np.array_equal(f_back, f)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["auto", "recon", "stage", "pregather"])
def test_gpu_degree_layout_matches_oracle(kernel):
    g = fu.Graph.rmat(14, 16, seed=3)
    v = fu.uniform_values(g.n, seed=3)
    eng = fu.CollectAll(g, v, kernel=kernel, layout="degree")
    eng.run(120)
    a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, 120, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    means, _ = fu.component_means(g.rowptr, g.col, v)
    eng.set_targets(means)
    assert eng.max_err() == np.max(np.abs(a_ref - means))
