"""GPU parity: the HIP kernels (through the C ABI) against the oracle and the golden
fixtures. Bit-exact everywhere: the kernels keep the reference's left-to-right fp64 sums
(flowupdating-collectall.py:106-113), so no tolerance is needed. Full-size checks use
properties (convergence to the component means, flow antisymmetry) and a bitwise
comparison against the C oracle on a prefix of the rounds."""
import io
import os

import numpy as np
import pytest

import coracle
import fu
from conftest import (ca_sync_fixtures, fixture_decl_csr, load_json, load_npz, tick_fixtures,
                      write_deployment_xml, write_platform_xml)

pytestmark = pytest.mark.gpu

# kernel 4 (recon: LDS tiles with flow reconstruction), kernel 8 (stage: LDS-staged slices +
# recon tiles) and kernel 9 (pregather: slice staging + per-bucket transpose, then recon
# tiles reading the pre-gathered estimates); "auto" switches between them mid-run
KERNELS = ["recon", "stage", "pregather"]


def _check_fixture(meta, kernel, hub_threshold=None):
    d = load_npz(meta["file"])
    rounds = [int(r) for r in d["rounds"]]
    eng = fu.CollectAll(rowptr=d["rowptr"], col=d["col"], values=d["values"], kernel=kernel,
                        hub_threshold=hub_threshold)
    done = 0
    for k, r in enumerate(rounds):
        eng.run(r + 1 - done)
        done = r + 1
        assert np.array_equal(eng.estimates(), d["last_avg"][k]), (meta["file"], kernel, r)
        assert np.array_equal(eng.flows(), d["flows"][k]), (meta["file"], kernel, r)
    eng.close()


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name,meta", ca_sync_fixtures())
def test_ca_sync_fixture_bitwise(name, meta, kernel):
    _check_fixture(meta, kernel)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", ["rmat9_ef8", "star_257", "star_1500", "er300_m450"])
def test_ca_sync_fixture_heavy_path(name, kernel):
    """hub_threshold=3 sends most nodes down the heavy (block-per-node) path."""
    meta = dict(ca_sync_fixtures())[name]
    _check_fixture(meta, kernel, hub_threshold=3)


@pytest.mark.parametrize("kernel", KERNELS + ["auto"])
def test_er_vs_c_oracle_bitwise(kernel):
    g = fu.Graph.erdos_renyi(200_000, 800_000, seed=5)
    v = fu.uniform_values(g.n, seed=1)
    eng = fu.CollectAll(g, v, kernel=kernel)
    eng.run(40)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 40, nthreads=8)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


@pytest.mark.parametrize("kernel", KERNELS)
def test_rmat_hubs_vs_c_oracle_bitwise(kernel):
    g = fu.Graph.rmat(15, 16, seed=2)
    assert g.max_deg > 2048  # exercises chunked heavy tiles
    v = fu.uniform_values(g.n, seed=4)
    eng = fu.CollectAll(g, v, kernel=kernel)
    eng.run(25)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 25, nthreads=8)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


def test_err_trace_and_max_err():
    g = fu.Graph.random_regular(4096, 8, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    tgt, _ = fu.component_means(g.rowptr, g.col, v)
    eng = fu.CollectAll(g, v)
    eng.set_targets(tgt)
    tr = eng.run(400, err_every=1)
    assert len(tr) == 400
    est = eng.estimates()
    assert tr[-1] == np.max(np.abs(est - tgt))
    assert eng.max_err() == tr[-1]
    first = int(np.argmax(tr < 1e-9)) + 1
    assert tr[first - 1] < 1e-9 and 150 < first < 260  # 187 rounds on RR-4096
    # same trace from a C-oracle run at a few rounds
    for r in (1, 10, 100):
        a_ref, _ = coracle.ca_sync(g.rowptr, g.col, g.rev, v, r)
        assert tr[r - 1] == np.max(np.abs(a_ref - tgt))


@pytest.mark.parametrize("kernel", KERNELS)
def test_first_rounds_flows_each_round(kernel):
    """Round 0 writes no flows and rounds 1-2 compute the old flows instead of reading them
    (fm): the flows read back after every one of the first rounds (f_0 materialised on
    demand) and before any round (all 0.0) equal the C oracle, also after a reset."""
    g = fu.Graph.rmat(12, 16, seed=4)
    v = fu.uniform_values(g.n, seed=4)
    eng = fu.CollectAll(g, v, kernel=kernel, hub_threshold=32)
    eng.set_option("mega_hub", 300)  # mega-hub chains and k_hub_stage / k_hub_flows too
    assert g.max_deg > 300
    for attempt in range(2):
        assert not np.any(eng.flows())
        for r in range(1, 6):
            eng.run(1)
            a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, r)
            assert np.array_equal(eng.estimates(), a_ref), (kernel, r)
            assert np.array_equal(eng.flows(), f_ref), (kernel, r)
        eng.reset()
    eng.close()


def test_mem_info_tracks_a_handle():
    """fu_mem_info: the device's HBM (288 GB on an MI355X), and a handle's device memory
    shows as used while it lives."""
    free0, total = fu.mem_info(0)
    assert 0 < free0 <= total and total > 200 * 2 ** 30
    g = fu.Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
    eng = fu.CollectAll(g, fu.uniform_values(g.n, seed=0))
    eng.run(2)
    free1, _ = fu.mem_info(0)
    assert free1 < free0 - 100 * 2 ** 20  # flows, estimates, tables: > 100 MB for ER-1M
    eng.close()
    with pytest.raises(fu.FuError, match="bad device"):
        fu.mem_info(99)


def test_nan_propagates_to_err():
    g = fu.Graph.random_regular(256, 4, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    v[17] = np.nan
    eng = fu.CollectAll(g, v)
    eng.set_targets(np.zeros(g.n))
    tr = eng.run(3, err_every=1)
    assert np.isnan(tr).all()


def test_isolated_and_empty():
    rp = np.array([0, 0, 1, 2, 2], dtype=np.int64)
    col = np.array([2, 1], dtype=np.int32)
    v = np.array([3.5, -0.0, 7.0, 1e-310])  # isolated nodes, signed zero, subnormal
    eng = fu.CollectAll(rowptr=rp, col=col, values=v)
    eng.run(5)
    a_ref, f_ref = coracle.ca_sync(rp, col, np.array([1, 0], dtype=np.int32), v, 5)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    assert eng.estimates()[3] == 1e-310


def test_option_errors():
    g = fu.Graph.random_regular(64, 4, seed=1)
    eng = fu.CollectAll(g, np.ones(g.n))
    for k in (1, 2, 3, 5, 6, 7, 10, 11):  # removed variants / out of range
        with pytest.raises(fu.FuError, match="kernel must be"):
            eng.set_option("kernel", k)
    for key in ("nope", "bins", "hub_scan", "pipe_bpc", "wave_edges", "diag", "hub_multi", "hub_blocks", "fuse",
                "tr_pipe", "hub_prio", "side_tiles", "split_tr", "hub_cus", "hub_cu_stride", "st_split", "tr_hot", "nt", "g56"):
        with pytest.raises(fu.FuError):
            eng.set_option(key, 1)
    for key, val in (("tr_nt", 2), ("tr_nt", -1)):
        with pytest.raises(fu.FuError):
            eng.set_option(key, val)
    with pytest.raises(fu.FuError):
        eng.run(5, err_every=1)  # no targets
    eng.run(2)
    with pytest.raises(fu.FuError):
        eng.set_option("kernel", 8)  # after rounds ran
    eng.reset()
    eng.set_option("kernel", 8)
    eng.run(1)
    eng.reset()
    eng.set_option("kernel", 9)
    eng.run(2)


@pytest.mark.parametrize("persistent", [False, True, "noreg"])
@pytest.mark.parametrize("name,fn", tick_fixtures())
def test_replay_matches_reference_snapshots(name, fn, persistent):
    d = load_json(fn)
    names, vals, rp, col = fixture_decl_csr(d)
    tr = fu.Trace(rp, col, "collectall" if d["mode"] == "ca" else "pairwise", d["ticks"],
                  d["order"])
    rep = fu.Replay(tr, vals, persistent=bool(persistent), registers=persistent != "noreg")
    snaps = rep.run(d["ticks"], snapshot_ticks=range(d["ticks"]))
    for t in range(d["ticks"]):
        keys = d["snap_keys"][t]
        assert [float(snaps[t][i]) for i in keys] == d["snap_vals"][t], (name, t)
    last, flows, est = rep.state()
    a = tr.arrays()
    for i in range(tr.n):
        assert list(flows[a["rowptr"][i]:a["rowptr"][i + 1]]) == d["flows"][i]
        assert list(est[a["rowptr"][i]:a["rowptr"][i + 1]]) == d["estimates"][i]


@pytest.mark.parametrize("persistent", [False, True, "noreg"])
@pytest.mark.parametrize("mode", ["collectall", "pairwise"])
def test_replay_rr64k_vs_c_oracle(mode, persistent):
    """BASELINE config 3: pairwise on a 64K-node random regular graph (and collect-all)."""
    g = fu.Graph.random_regular(65536, 8, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    tr = fu.Trace(g.rowptr, g.col, mode, 160, "rand:3")
    a = tr.arrays()
    rep = fu.Replay(tr, v, persistent=bool(persistent), registers=persistent != "noreg")
    snaps = rep.run(160, snapshot_ticks=[60, 120, 159])
    last, flows, est = rep.state()
    l_ref, f_ref, e_ref, s_ref = coracle.replay(a["rowptr"], v, a["tick_task_off"], a["tasks"],
                                                a["events"], a["out_ids"], tr.n_msgs,
                                                [60, 120, 159])
    assert np.array_equal(last, l_ref)
    assert np.array_equal(flows, f_ref)
    assert np.array_equal(est, e_ref)
    for t in (60, 120, 159):
        assert np.array_equal(snaps[t], s_ref[t])


def test_headline_window_bitwise():
    """The driver's N = 1 headline exactly as bench.py runs it: ER-1M, bench.prepare (one
    autotune pass, 5 warmup rounds, fu_reset), then bench.timed_rounds (rounds 0-19 with
    the HIP event marks); estimates and flows equal the C oracle's after 20 rounds, then
    config2_1000's prefix (reset, the 400-round untimed pass, reset, 1000 timed rounds)."""
    import bench

    g = fu.Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    eng = fu.CollectAll(g, v)
    bench.prepare(eng, "auto", 5)
    bench.timed_rounds(eng, 20)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 20, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    eng.reset()
    bench.prepare(eng, "auto", 400, [], tune=False)
    bench.timed_rounds(eng, 1000)
    coracle.ca_rounds(g.rowptr, g.col, g.rev, v, 980, a_ref, f_ref, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    eng.close()


@pytest.mark.parametrize("bounds", [[0, 1, 7], [0, 3, 7], [0, 0, 2, 7]])
def test_marked_window_matches_plain_rounds(bounds):
    """fu_run_collectall_marked (bench.py's timed window): marks at the bounds, round 0's
    marks from k_round0's own start / stop events when the window starts at round 0; the
    state equals plain rounds bitwise, every interval is a positive device time, and a second
    window (not from round 0) records its marks as plain events."""
    g = fu.Graph.erdos_renyi(20000, 80000, seed=5)
    v = fu.uniform_values(g.n, seed=2)
    eng = fu.CollectAll(g, v)
    eng.run_marked(np.asarray(bounds, dtype=np.int32))
    eng.synchronize()
    for k in range(len(bounds) - 1):
        if bounds[k + 1] > bounds[k]:
            assert eng.elapsed(k, k + 1) > 0.0, k
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, bounds[-1], nthreads=8)
    assert np.array_equal(eng.estimates(), a_ref) and np.array_equal(eng.flows(), f_ref)
    eng.run_marked(np.asarray([0, 2], dtype=np.int32))
    assert eng.elapsed(0, 1) > 0.0
    coracle.ca_rounds(g.rowptr, g.col, g.rev, v, 2, a_ref, f_ref, nthreads=8)
    assert np.array_equal(eng.estimates(), a_ref)
    eng.close()


def test_pairwise_unit_window_bitwise():
    """BASELINE config 3 exactly as `pairwise_unit` times it: RR-64K pairwise, tie order
    rand:3, the default persistent register kernel run to tick 101, then ticks 101-500
    through fu_replay_run_timed; the final last_avg, flows and estimate caches equal the C
    oracle's replay of ticks 0-500 (PW:93-117 every event)."""
    g = fu.Graph.random_regular(65536, 8, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    tr = fu.Trace(g.rowptr, g.col, "pairwise", 501, "rand:3")
    a = tr.arrays()
    rep = fu.Replay(tr, v, persistent=True)
    rep.run(101)
    assert rep.run_timed(501) > 0
    last, flows, est = rep.state()
    rep.close()
    l_ref, f_ref, e_ref, _ = coracle.replay(a["rowptr"], v, a["tick_task_off"], a["tasks"], a["events"],
                                            a["out_ids"], tr.n_msgs)
    assert np.array_equal(last, l_ref)
    assert np.array_equal(flows, f_ref)
    assert np.array_equal(est, e_ref)


@pytest.mark.parametrize("mode,tag", [("ca", "fwd"), ("pw", "fwd"), ("ca", "rev"), ("pw", "rand7")])
def test_engine_small_platform_watcher_lines(tmp_path, mode, tag):
    """The drop-in Engine on the reference inputs prints the watcher's lines (CA:134-142)
    with the reference's values at t = 10, 20, ..., 1000."""
    d = load_json(f"tick_small_platform_{mode}_{tag}.json")
    plat = tmp_path / "small_platform.xml"
    dep = tmp_path / "actors.xml"
    write_platform_xml(plat)
    write_deployment_xml(dep, d["actors"])
    order = d["order"]
    e, res = fu.run_reference_main("collectall" if mode == "ca" else "pairwise", str(plat),
                                   str(dep), 1000.0, 10.0, order=order, out=io.StringIO())
    names = d["names"]
    watch = [ln for ln in e.lines if ":watcher:" in ln and ("last_avg{" in ln or "value{" in ln)]
    by_t = {}
    for ln in watch:
        t = float(ln.split()[1].rstrip("]"))
        by_t.setdefault(t, []).append(ln.split("] ", 2)[2])
    for t in range(10, 1001, 10):
        la = {names[k]: v for k, v in zip(d["snap_keys"][t], d["snap_vals"][t])}
        vd = {nm: float(a[1]) for nm, a in zip(names, d["actors"])}
        want = [f"value{vd}"] + ([f"last_avg{la}"] if la else [])
        assert by_t[float(t)] == want, t
    assert np.max(np.abs(res["last_avg"] - 190 / 6)) / (190 / 6) < 1e-12


@pytest.mark.parametrize("mode", ["ca", "pw"])
def test_cli_reference_inputs_watcher_lines(tmp_path, monkeypatch, capsys, mode):
    """`python -m fu collectall|pairwise` run where the reference runs (./platforms/
    small_platform.xml, ./actors.xml: CA:154,157) prints the reference's watcher lines
    (CA:134-142) at t = 10 ... 1000; `--sync` and `bench-graph` run too."""
    from fu.__main__ import main

    d = load_json(f"tick_small_platform_{mode}_fwd.json")
    (tmp_path / "platforms").mkdir()
    write_platform_xml(tmp_path / "platforms" / "small_platform.xml")
    write_deployment_xml(tmp_path / "actors.xml", d["actors"])
    monkeypatch.chdir(tmp_path)
    assert main(["collectall" if mode == "ca" else "pairwise"]) == 0
    out = capsys.readouterr().out.splitlines()
    watch = [ln for ln in out if ":watcher:" in ln and ("last_avg{" in ln or "value{" in ln)]
    by_t = {}
    for ln in watch:
        by_t.setdefault(float(ln.split()[1].rstrip("]")), []).append(ln.split("] ", 2)[2])
    names = d["names"]
    vd = {nm: float(a[1]) for nm, a in zip(names, d["actors"])}
    for t in range(10, 1001, 10):
        la = {names[k]: v for k, v in zip(d["snap_keys"][t], d["snap_vals"][t])}
        assert by_t[float(t)] == [f"value{vd}"] + ([f"last_avg{la}"] if la else []), t
    if mode == "ca":
        assert main(["collectall", "--sync", "--rounds", "200"]) == 0
        assert "last_avg{" in capsys.readouterr().out
        assert main(["bench-graph", "rr:n=4096,d=8", "--rounds", "50"]) == 0
        line = capsys.readouterr().out
        assert "n=4096" in line and "edge_updates/s=" in line and "max_err=" in line


def test_full_size_er1m_convergence_and_prefix_parity():
    """BASELINE config 2 at full size: ER n=1e6 m=4e6. Bitwise vs the C oracle for 60 rounds,
    then the 1000-round run converges to the per-component means (< 1e-9)."""
    g = fu.Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    eng = fu.CollectAll(g, v)
    eng.run(60)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 60, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    tgt, comp = fu.component_means(g.rowptr, g.col, v)
    eng.set_targets(tgt)
    tr = eng.run(940, err_every=10)
    assert tr[-1] < 1e-9
    assert np.all(np.diff(tr[5:]) <= 0) or tr[-1] < 1e-12  # settles monotonically


def test_config2_as_written_1000_rounds_bitwise():
    """BASELINE config 2 as written, the whole job bitwise: ER n=1e6 m=4e6, 1000 rounds from
    the zero state on the default engine (kernel auto, autotuned at every packing width it
    reaches; the estimate table packs to 32, 16 and 8 bits on the way), estimates and flows
    equal to the C oracle's after rounds 150, 400 and 1000 (CA:105-128 every round)."""
    g = fu.Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    eng = fu.CollectAll(g, v)
    a_ref, f_ref = None, None
    widths = set()
    for done, k in ((150, 150), (400, 250), (1000, 600)):
        for _ in range(0, k, 50):  # the host sees each plan's width between calls (autotune per width)
            eng.run(50)
            widths.add(eng.pack_widths()[2])
        if a_ref is None:
            a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, done, nthreads=16)
        else:
            coracle.ca_rounds(g.rowptr, g.col, g.rev, v, k, a_ref, f_ref, nthreads=16)
        assert np.array_equal(eng.estimates(), a_ref), done
        assert np.array_equal(eng.flows(), f_ref), done
    assert {32, 16, 8} <= widths, widths  # every packed width ran
    assert eng.info()["rounds"] == 1000
    eng.close()


def test_dist_single_rank_rccl_matches_engine():
    """fu_dist_create + RCCL communicator at world size 1 (the only size one GPU box can
    run): no ghosts, the per-round halo hook runs with empty send lists. Ghost slots are
    exercised by the local-transport tests below."""
    from fu.dist import DistCollectAll, partition, unique_id

    g = fu.Graph.random_geometric(50_000, avg_deg=8, seed=3)
    v = fu.uniform_values(g.n, seed=1)
    plan = partition(g.rowptr, g.col, g.rev, 1, 0)
    d = DistCollectAll(plan, v, unique_id(), kernel="recon")
    d.run(30)
    eng = fu.CollectAll(g, v)
    eng.run(30)
    assert np.array_equal(d.estimates(), eng.estimates())
    assert np.array_equal(d.flows(), eng.flows())
    tgt, _ = fu.component_means(g.rowptr, g.col, v)
    d.set_targets(tgt)
    tr = d.run(10, err_every=5)
    assert len(tr) == 2 and np.isfinite(tr).all()
    d.close()
    d8 = DistCollectAll(plan, v, unique_id(), kernel="stage")  # kernel 8 at one RCCL rank
    d8.run(30)
    assert np.array_equal(d8.estimates(), eng.estimates())
    assert np.array_equal(d8.flows(), eng.flows())
    d8.close()


@pytest.mark.parametrize("kernel", ["recon", "stage"])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", ["rgg", "er"])
def test_dist_ghost_slots_local_transport_bitwise(world, kind, kernel):
    """Every rank of a partitioned graph as its own handle on GPU 0, the halo moved by the
    in-process transport through the RCCL path's comm-stream / event chain (pack on the comm
    stream behind the boundary tiles, copies into the peers' ghost slots beside the interior
    tiles, the next round behind ev_halo), 100 rounds queued with no host sync. Estimates and
    flows equal the C oracle bitwise. ER cuts most edges (every rank talks to every rank).
    kernel "stage": kernel 8, the ghost slots staged as slices of their own (boundary light
    tiles first, then the halo beside the interior tiles)."""
    from fu.dist import DistCollectAll, partition, run_local

    if kind == "rgg":
        g = fu.Graph.random_geometric(200_000, avg_deg=8, seed=21)
    else:
        g = fu.Graph.erdos_renyi(60_000, 240_000, seed=21)
    v = fu.uniform_values(g.n, seed=21)
    plans = [partition(g.rowptr, g.col, g.rev, world, r) for r in range(world)]
    assert all(p.n_ghost_a > 0 and len(p.send_a_idx) > 0 for p in plans)
    engs = [DistCollectAll(p, v[p.lo:p.hi], None, kernel=kernel) for p in plans]
    assert all(e.info()["kernel"] == kernel for e in engs)
    rounds = 100
    run_local(engs, rounds)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, rounds, nthreads=16)
    for p, e in zip(plans, engs):
        assert np.array_equal(e.estimates(), a_ref[p.lo:p.hi]), p.rank
        assert np.array_equal(e.flows(), f_ref[g.rowptr[p.lo]:g.rowptr[p.hi]]), p.rank
    for e in engs:
        e.close()


def test_dist_autotune_never_runs_kernel_9():
    """Kernel 9 runs on partitioned handles when asked for (test_dist_kernel9_rmat_ghosts_bitwise),
    but the autotuner never makes it a candidate there: whether it has a staging layout may
    differ between ranks, and every rank must run the same rounds (FP::tune_steps). One RCCL
    rank (a pass needs many rounds in one call; the in-process transport runs one at a time),
    R-MAT where kernel 9 would win on one GPU; kernel 9 explicitly at one rank, bitwise."""
    from fu.dist import DistCollectAll, partition, unique_id

    g = fu.Graph.rmat(15, 16, seed=12)
    v = fu.uniform_values(g.n, seed=12)
    plan = partition(g.rowptr, g.col, g.rev, 1, 0)
    d = DistCollectAll(plan, v, unique_id(), kernel="auto")
    d.run(120)
    info = d.info()
    assert info["autotune"] == "done" and info["kernel"] in ("recon", "stage"), info
    assert info["tune_us_per_round"]["pregather"] == 0.0
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 120, nthreads=16)
    assert np.array_equal(d.estimates(), a_ref) and np.array_equal(d.flows(), f_ref)
    d.close()
    d9 = DistCollectAll(plan, v, unique_id(), kernel="pregather")
    d9.run(40)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 40, nthreads=16)
    assert np.array_equal(d9.estimates(), a_ref) and np.array_equal(d9.flows(), f_ref)
    d9.close()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("geo", [(1024, 0), (2048, 0), (512, 0)])
def test_dist_rmat_heavy_rows_and_hubs_with_ghosts_bitwise(world, geo):
    """Partitioned R-MAT (scale 14) on the in-process transport with hub_threshold 32 and
    mega_hub 256: hundreds of heavy rows and mega hubs per rank have ghost columns, so the
    heavy tiles, k_hub_stage (gathers through col into ghost slots), the hub chains and
    k_hub_flows all read halo estimates. 100 rounds bitwise against the C oracle."""
    from fu.dist import DistCollectAll, partition, run_local

    g = fu.Graph.rmat(14, 16, seed=3)
    v = fu.uniform_values(g.n, seed=4)
    plans = [partition(g.rowptr, g.col, g.rev, world, r) for r in range(world)]
    engs = []
    for p in plans:
        e = DistCollectAll(p, v[p.lo:p.hi], None)
        for key, val in (("hub_threshold", 32), ("mega_hub", 256), ("tile_edges", geo[0])):
            fu._lib.call("fu_set_option", e._h, key.encode(), val)
        ld = np.diff(p.rowptr)
        ghost = [(p.col[p.rowptr[i]:p.rowptr[i + 1]] >= p.n_local).any() for i in range(p.n_local)]
        assert sum(1 for i in range(p.n_local) if ld[i] > 256 and ghost[i]) > 50  # mega hubs at the cut
        engs.append(e)
    assert all(e.info()["mega_hubs"] > 0 for e in engs)
    rounds = 100
    run_local(engs, rounds)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, rounds, nthreads=16)
    for p, e in zip(plans, engs):
        assert np.array_equal(e.estimates(), a_ref[p.lo:p.hi]), p.rank
        assert np.array_equal(e.flows(), f_ref[g.rowptr[p.lo]:g.rowptr[p.hi]]), p.rank
    for e in engs:
        e.close()


@pytest.mark.parametrize("world", [2, 3])
def test_dist_kernel9_rmat_ghosts_bitwise(world):
    """Kernel 9 on a partitioned R-MAT (in-process transport): the staging slices cover the
    ghost estimate slots, the transposes deliver halo estimates to heavy rows, mega hubs and
    light tiles, and the halo goes out after the round (boundary rows sit in every row class).
    60 rounds with lag, bitwise against the C oracle; then a switch to kernel 4 after a reset."""
    from fu.dist import DistCollectAll, partition, run_local

    g = fu.Graph.rmat(14, 16, seed=5)
    v = fu.uniform_values(g.n, seed=6)
    plans = [partition(g.rowptr, g.col, g.rev, world, r) for r in range(world)]
    engs = []
    for p in plans:
        e = DistCollectAll(p, v[p.lo:p.hi], None, kernel="pregather")
        for key, val in (("hub_threshold", 32), ("mega_hub", 256)):
            fu._lib.call("fu_set_option", e._h, key.encode(), val)
        engs.append(e)
    assert all(e.info()["kernel"] == "pregather" and e.info()["mega_hubs"] > 0 for e in engs)
    for rounds in (7, 60):
        run_local(engs, rounds - (7 if rounds == 60 else 0))
        a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, rounds, nthreads=16)
        for p, e in zip(plans, engs):
            assert np.array_equal(e.estimates(), a_ref[p.lo:p.hi]), (p.rank, rounds)
            assert np.array_equal(e.flows(), f_ref[g.rowptr[p.lo]:g.rowptr[p.hi]]), (p.rank, rounds)
    for e in engs:
        e.reset()
        fu._lib.call("fu_set_option", e._h, b"kernel", 4)
    run_local(engs, 5)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 5, nthreads=16)
    for p, e in zip(plans, engs):
        assert np.array_equal(e.estimates(), a_ref[p.lo:p.hi]), p.rank
    for e in engs:
        e.close()


def test_dist_exchange_local_checks_round_counts():
    """fu_dist_exchange_local refuses ranks that ran different numbers of rounds, no round,
    or a round whose halo was already exchanged (it would copy into the wrong generation)."""
    import ctypes

    from fu.dist import DistCollectAll, partition

    g = fu.Graph.erdos_renyi(20_000, 80_000, seed=2)
    v = fu.uniform_values(g.n, seed=2)
    plans = [partition(g.rowptr, g.col, g.rev, 2, r) for r in range(2)]
    engs = [DistCollectAll(p, v[p.lo:p.hi], None) for p in plans]
    arr = (ctypes.c_void_p * 2)(*[e._h.value for e in engs])
    with pytest.raises(fu.FuError, match="different numbers of rounds"):
        fu._lib.call("fu_dist_exchange_local", arr, 2)  # no round yet
    engs[0].run(1)
    with pytest.raises(fu.FuError, match="different numbers of rounds"):
        fu._lib.call("fu_dist_exchange_local", arr, 2)
    with pytest.raises(fu.FuError, match="no halo exchanged yet"):
        engs[0].halo_ms()  # packed, never exchanged
    engs[1].run(1)
    fu._lib.call("fu_dist_exchange_local", arr, 2)
    with pytest.raises(fu.FuError, match="no packed halo pending"):
        fu._lib.call("fu_dist_exchange_local", arr, 2)
    assert engs[0].halo_ms() > 0 and engs[1].halo_ms() > 0
    # a reset restarts the round bookkeeping: exactly one round, reset, one round again
    for e in engs:
        e.reset()
    with pytest.raises(fu.FuError, match="no halo exchanged yet"):
        engs[0].halo_ms()
    from fu.dist import run_local

    run_local(engs, 1)
    engs[0].run(1)  # round 1 launched on rank 0 only: its halo is packed, not exchanged
    with pytest.raises(fu.FuError, match="packed but not exchanged"):
        engs[0].halo_ms()
    engs[1].run(1)
    fu._lib.call("fu_dist_exchange_local", arr, 2)
    assert engs[0].halo_ms() > 0
    run_local(engs, 3)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 5, nthreads=16)
    for p, e in zip(plans, engs):
        assert np.array_equal(e.estimates(), a_ref[p.lo:p.hi]), p.rank
        assert np.array_equal(e.flows(), f_ref[g.rowptr[p.lo]:g.rowptr[p.hi]]), p.rank
    for e in engs:
        e.close()


def test_dist_rgg_slabs_local_transport_bitwise():
    """The native slab generator's halo plans (fu_part_gen_rgg, 3 parts) on the local
    transport equal the single-GPU engine on the global graph."""
    from fu.dist import DistCollectAll, RggPart, run_local

    n, world = 300_000, 3
    parts = [RggPart(n, avg_deg=8.0, seed=7, nparts=world, part=r) for r in range(world)]
    engs = [DistCollectAll(p.to_plan(), p.values(seed=3), None) for p in parts]
    run_local(engs, 20)
    g = fu.Graph.random_geometric(n, avg_deg=8.0, seed=7)
    v = fu.uniform_values(g.n, seed=3)
    eng = fu.CollectAll(g, v)
    eng.run(20)
    a, f = eng.estimates(), eng.flows()
    for p, e in zip(parts, engs):
        assert np.array_equal(e.estimates(), a[p.lo:p.hi])
        assert np.array_equal(e.flows(), f[g.rowptr[p.lo]:g.rowptr[p.hi]])
    for e in engs:
        e.close()


@pytest.mark.parametrize("persistent", [False, True, "noreg"])
def test_replay_with_faults_vs_c_oracle(persistent):
    """Fault-injected pairwise trace (drops + delays) replayed on the GPU == C oracle."""
    g = fu.Graph.random_regular(4096, 6, seed=2)
    v = fu.uniform_values(g.n, seed=5)
    tr = fu.Trace(g.rowptr, g.col, "pairwise", 300, "rand:1", faults="drop=0.1,delay=4:0.1,seed=3")
    a = tr.arrays()
    rep = fu.Replay(tr, v, persistent=bool(persistent), registers=persistent != "noreg")
    snaps = rep.run(150, snapshot_ticks=[60, 149])
    snaps.update(rep.run(300, snapshot_ticks=[299]))
    l_ref, f_ref, e_ref, s_ref = coracle.replay(a["rowptr"], v, a["tick_task_off"], a["tasks"],
                                                a["events"], a["out_ids"], tr.n_msgs, [60, 149, 299])
    last, flows, est = rep.state()
    assert np.array_equal(last, l_ref) and np.array_equal(flows, f_ref)
    for t in (60, 149, 299):
        assert np.array_equal(snaps[t], s_ref[t])


def test_dist_rgg_slab_estimates_only_halo_matches_engine():
    """The native slab generator + estimates-only halo at world size 1 (RCCL) equals the
    single-GPU engine on the global graph, bitwise."""
    from fu.dist import DistCollectAll, RggPart, unique_id

    n = 200_000
    part = RggPart(n, avg_deg=8.0, seed=5, nparts=1, part=0)
    v = part.values(seed=2)
    d = DistCollectAll(part.to_plan(), v, unique_id())
    d.run(40)
    g = fu.Graph.random_geometric(n, avg_deg=8.0, seed=5)
    eng = fu.CollectAll(g, v)
    eng.run(40)
    assert np.array_equal(d.estimates(), eng.estimates())
    assert np.array_equal(d.flows(), eng.flows())


def test_autotune_switches_kernels_bitwise():
    """kernel="auto" times kernel 4 (three tile geometries) and kernel 8 on real rounds and
    keeps the fastest; the switch happens mid-run and must not change a single bit."""
    g = fu.Graph.erdos_renyi(300_000, 1_200_000, seed=8)
    v = fu.uniform_values(g.n, seed=8)
    eng = fu.CollectAll(g, v)
    assert eng.info()["autotune"] == "pending"
    eng.run(64)
    info = eng.info()
    assert info["autotune"] == "done" and info["rounds"] == 64
    assert all(t > 0 for t in info["tune_us_per_round"].values())
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 64, nthreads=8)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


def test_autotune_width_cache_across_reset_bitwise():
    """The autotuner re-times the candidates when the packing width changes, keeps each
    width's winner, and after fu_reset reuses them (no new pass); the kernel switches at
    every width change must leave the bits untouched."""
    g = fu.Graph.erdos_renyi(200_000, 800_000, seed=12)
    v = fu.uniform_values(g.n, seed=12)
    eng = fu.CollectAll(g, v)
    eng.set_option("pack_every", 4)
    for _ in range(7):  # the host sees each plan's width once the stream has passed it
        eng.run(64)
        eng.synchronize()
    passes = eng.info()["tune_passes"]
    assert passes >= 3
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 448, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    eng.reset()
    for _ in range(7):
        eng.run(64)
        eng.synchronize()
    # widths tuned before the reset reuse their winner; a width whose change the host first
    # saw while a pass was pending (asynchronous width copies) may still need one pass
    assert eng.info()["tune_passes"] - passes <= 1
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


def test_reset_drops_a_width_pass_left_pending():
    """Calls too short for an autotune pass (bench.prepare's settle: 16 rounds each) see the
    packing width change and leave a pass pending for that width. fu_reset returns to the
    unpacked table, whose winner is cached, so the pending pass is dropped: the next call
    runs no pass at width 0 again, and the bits stay the oracle's."""
    g = fu.Graph.erdos_renyi(200_000, 800_000, seed=13)
    v = fu.uniform_values(g.n, seed=13)
    eng = fu.CollectAll(g, v)
    eng.set_option("pack_every", 4)
    eng.tune()
    passes = eng.info()["tune_passes"]
    assert passes == 1 and eng.info()["autotune"] == "done"
    for _ in range(30):
        eng.run(16)
        eng.synchronize()
    assert eng.pack_widths()[2] > 0
    assert eng.info()["autotune"] == "pending"
    assert eng.info()["tune_passes"] == passes
    eng.reset()
    assert eng.info()["autotune"] == "done"
    eng.run(64)
    eng.synchronize()
    assert eng.info()["tune_passes"] == passes
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 64, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    # a pass armed by the kernel option is not dropped by a reset
    eng.reset()
    eng.set_option("kernel", 0)
    eng.reset()
    assert eng.info()["autotune"] == "pending"


def _er_with_outlier_pairs(n, m, pairs, seed):
    """ER(n, m) plus `pairs` disjoint 2-node components whose values are far from the giant
    component's mean: their estimates never enter the packed window, so every gather of
    them goes through the escape code."""
    g = fu.Graph.erdos_renyi(n, m, seed=seed)
    src = np.repeat(np.arange(g.n), np.diff(g.rowptr))
    keep = src < g.col
    ps = n + 2 * np.arange(pairs)
    s = np.concatenate([src[keep], ps])
    d = np.concatenate([g.col[keep], ps + 1])
    v = np.concatenate([fu.uniform_values(n, seed=seed), 1e6 + np.arange(2 * pairs, dtype=np.float64)])
    return fu.Graph.from_edges(n + 2 * pairs, s, d), v


@pytest.mark.parametrize("kind,kernel", [("er", "recon"), ("rmat", "recon"), ("er", "stage"),
                                         ("rmat", "stage"), ("er", "pregather"), ("rmat", "pregather")])
def test_packed_gather_long_run_bitwise(kind, kernel):
    """The packed estimate table (8/16/32-bit lossless codes + escapes) switches on as the
    estimates converge; 300 rounds must still equal the C oracle bit for bit, and equal the
    same run with packing off."""
    if kind == "er":
        g, v = _er_with_outlier_pairs(100_000, 400_000, 64, seed=3)
    else:
        g = fu.Graph.rmat(13, 16, seed=3)
        v = fu.uniform_values(g.n, seed=3)
    rounds = 300
    eng = fu.CollectAll(g, v, kernel=kernel, hub_threshold=16)
    eng.set_option("pack_every", 4)
    seen = set()
    for _ in range(rounds // 25):
        eng.run(25)
        seen.update(eng.pack_widths())
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, rounds, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    assert seen & {8, 16, 32}, seen  # packing was actually exercised
    off = fu.CollectAll(g, v, kernel="recon", hub_threshold=16)
    off.set_option("pack", 0)
    off.run(rounds)
    assert off.pack_widths() == (0, 0, 0)
    assert np.array_equal(off.estimates(), a_ref)


@pytest.mark.parametrize("opts", [{"staged_lo": 0}, {"staged_lo": 0, "pack": 0}, {"tr_bpx": 0},
                                  {"tr_bpx": 3}, {"tr_bpx": 3, "tr_nt": 0}])
def test_load_order_and_transpose_options_bitwise(opts):
    """The A/B options of this round (kernel 8's interleaved load order; kernel 9's
    one-block-per-bucket transpose) give the C oracle's bits over a 300-round run with packing
    and escapes."""
    g, v = _er_with_outlier_pairs(100_000, 400_000, 64, seed=5)
    rounds = 300
    eng = fu.CollectAll(g, v, kernel="pregather" if "tr_bpx" in opts else "stage",
                        hub_threshold=16)
    eng.set_option("pack_every", 4)
    for k, val in opts.items():
        eng.set_option(k, val)
    eng.run(rounds)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, rounds, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


def test_packed_gather_with_kernel_switches():
    """recon, stage and auto (which switches kernels and geometries mid-run, re-tuning at each
    packing width) give the same bits over a run long enough for packing to engage."""
    g = fu.Graph.erdos_renyi(50_000, 200_000, seed=9)
    v = fu.uniform_values(g.n, seed=9)
    ref = None
    for kernel in ("recon", "stage", "pregather", "auto"):
        eng = fu.CollectAll(g, v, kernel=kernel)
        eng.set_option("pack_every", 2)
        eng.run(260)
        got = (eng.estimates(), eng.flows())
        if ref is None:
            ref = got
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), kernel


@pytest.mark.parametrize("kernel,opts", [("recon", {"tile_edges": 2048}),
                                         ("recon", {"tile_edges": 1024}),
                                         ("recon", {"tile_edges": 1024, "tile_nodes": 256}),
                                         ("recon", {"tile_edges": 512})])
@pytest.mark.parametrize("kind", ["er", "rmat", "rgg"])
def test_tile_geometries_bitwise(kernel, opts, kind):
    """Every kernel 4 tile geometry the autotuner may pick, with heavy rows (hub_threshold 16
    on R-MAT), against the C oracle."""
    if kind == "er":
        g = fu.Graph.erdos_renyi(200_000, 800_000, seed=6)
    elif kind == "rgg":  # narrow tiles: 2-byte column offsets (c16)
        g = fu.Graph.random_geometric(200_000, avg_deg=8, seed=6)
    else:
        g = fu.Graph.rmat(14, 16, seed=6)
    v = fu.uniform_values(g.n, seed=6)
    eng = fu.CollectAll(g, v, kernel=kernel, hub_threshold=16 if kind == "rmat" else None)
    for k, val in opts.items():
        eng.set_option(k, val)
    eng.run(30)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 30, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


@pytest.mark.parametrize("layout", [0, 1, 2, 3])
def test_stage_forced_layouts_bitwise(layout):
    """Kernel 8 with each slice layout forced (1/2/4/8-byte elements) over a run in which the
    table goes from doubles to 32/16/8-bit codes: a table wider than the layout is gathered
    from global memory by the stage launch, a narrower one sits in LDS; escapes (far-off
    2-node components) read the double through the edge's column. Heavy rows (R-MAT part)
    run as kernel 4 heavy tiles."""
    g, v = _er_with_outlier_pairs(60_000, 240_000, 32, seed=11)
    eng = fu.CollectAll(g, v, kernel="stage", hub_threshold=16)
    eng.set_option("stage_layout", layout)
    eng.set_option("pack_every", 4)
    seen = set()
    for _ in range(12):
        eng.run(25)
        seen.update(eng.pack_widths())
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 300, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    assert seen & {8, 16, 32}, seen


@pytest.mark.parametrize("mega", [64, 300, 8192])
def test_pregather_heavy_rows_and_mega_hubs_bitwise(mega):
    """Kernel 9 on R-MAT with heavy rows (hub_threshold 16) and mega hubs above `mega`
    (k_hub_stage reading the pre-gathered estimates), packed rounds included; several
    buckets and slices (n > 16K nodes, E > 16K edges)."""
    g = fu.Graph.rmat(15, 16, seed=15)
    v = fu.uniform_values(g.n, seed=15)
    eng = fu.CollectAll(g, v, kernel="pregather", hub_threshold=16)
    eng.set_option("mega_hub", mega)
    eng.set_option("pack_every", 4)
    eng.run(60)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 60, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


@pytest.mark.parametrize("multi", [1, 0, "mid0", "nolag", "iso0", "short0", "short_nolag", "trnt0", "bpx3"])
@pytest.mark.parametrize("ht,mega", [(16, 8192), (4, 700), (64, 100000)])
def test_pregather_multi_row_chains_bitwise(multi, ht, mega):
    """Kernel 9's heavy rows of more than 256 edges as k_heavy_multi blocks (16 rows per
    block, one wave running all 32 chains) against the C oracle, with rounds 1-2 (no flow
    reads), the error check on every round (CHECK), packing every 4 rounds, rows of every
    length from the threshold to the mega hubs (ragged ends of the last chunk), and the
    one-row-per-wave path (multi_heavy 0) and the rows of 257-1024 edges in registers
    (multi_mid 0) for A/B."""
    g = fu.Graph.rmat(15, 16, seed=33)
    v = fu.uniform_values(g.n, seed=33)
    eng = fu.CollectAll(g, v, kernel="pregather", hub_threshold=ht, layout="degree")
    eng.set_option("mega_hub", mega)
    if multi == "mid0":
        eng.set_option("multi_mid", 0)
    elif multi == "nolag":  # the two-pass heavy rows (lag is the default)
        eng.set_option("lag", 0)
    elif multi == "bpx3":  # three transpose blocks per XCD, each looping over many buckets
        eng.set_option("tr_bpx", 3)
    elif multi == "iso0":  # the trailing isolated rows as light tiles (k_isolated is the default)
        eng.set_option("iso_rows", 0)
    elif multi == "trnt0":  # plain G_A loads / G_B stores in the transposes (tr_nt is the default)
        eng.set_option("tr_nt", 0)
    elif multi == "short0":  # the rows of 129-256 edges one per wave (multi_short is the default)
        eng.set_option("multi_short", 0)
    elif multi == "short_nolag":
        for key, val in (("multi_short", 1), ("lag", 0)):
            eng.set_option(key, val)
    else:
        eng.set_option("multi_heavy", multi)
    eng.set_option("pack_every", 4)
    tgt, _ = fu.component_means(g.rowptr, g.col, v)
    eng.set_targets(tgt)
    tr = eng.run(45, err_every=1)
    a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, 45, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    assert np.max(np.abs(a_ref - tgt)) == tr[-1]


@pytest.mark.parametrize("mega", [100, 1000])
def test_pregather_degree_layout_hub_buckets_first(mega):
    """Kernel 9 under the degree layout: the mega hubs are the first rows, so their buckets
    are transposed first and their chains (reading the pre-gathered estimates and the old
    flows) and k_hub_flows overlap the other buckets' transpose and the other tiles."""
    g = fu.Graph.rmat(15, 16, seed=21)
    v = fu.uniform_values(g.n, seed=21)
    eng = fu.CollectAll(g, v, kernel="pregather", layout="degree")
    eng.set_option("mega_hub", mega)
    assert eng.info()["mega_hubs"] > 0
    eng.run(40)
    a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, 40, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


@pytest.mark.parametrize("tile", [2048, 1024, 512])
@pytest.mark.parametrize("mega", [64, 300, 8192])
def test_mega_hub_staged_chain_bitwise(tile, mega):
    """Kernel 4's mega-hub path (k_hub_stage + a chain-only block) on R-MAT rows above the
    threshold, every tile geometry, unpacked and packed rounds, against the C oracle."""
    g = fu.Graph.rmat(14, 16, seed=12)
    v = fu.uniform_values(g.n, seed=12)
    eng = fu.CollectAll(g, v, kernel="recon")
    eng.set_option("tile_edges", tile)
    eng.set_option("mega_hub", mega)
    eng.set_option("pack_every", 4)
    eng.run(60)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 60, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


def test_star_hub_above_default_mega_threshold():
    """A 20000-leaf star (one row far above the default 8192 threshold) joined to an ER graph."""
    n_er, leaves = 30_000, 20_000
    er = fu.Graph.erdos_renyi(n_er, 120_000, seed=13)
    src = np.repeat(np.arange(er.n), np.diff(er.rowptr))
    keep = src < er.col
    hub = n_er + leaves
    s = np.concatenate([src[keep], np.full(leaves, hub), [0]])
    d = np.concatenate([er.col[keep], n_er + np.arange(leaves), [hub]])
    g = fu.Graph.from_edges(hub + 1, s, d)
    assert g.max_deg > 8192
    v = fu.uniform_values(g.n, seed=13)
    eng = fu.CollectAll(g, v, kernel="recon")
    eng.run(40)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 40, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


@pytest.mark.parametrize("wave_heavy", [0, 1])
@pytest.mark.parametrize("tile", [2048, 1024, 512])
def test_heavy_rows_wave_and_block_paths_bitwise(tile, wave_heavy):
    """Kernel 4's heavy rows (degree > hub_threshold) one per wave (default) or one per block,
    with mega hubs above 300 in the staged path, every geometry, packed rounds included."""
    g = fu.Graph.rmat(14, 16, seed=14)
    v = fu.uniform_values(g.n, seed=14)
    eng = fu.CollectAll(g, v, kernel="recon", hub_threshold=16)
    eng.set_option("tile_edges", tile)
    eng.set_option("wave_heavy", wave_heavy)
    eng.set_option("mega_hub", 300)
    eng.set_option("pack_every", 4)
    eng.run(80)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 80, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


def test_round0_flows_sparse_rows_and_hubs():
    """Round 0's per-block row search: long runs of isolated nodes between edges (a block's
    rows span more than its LDS window) and a hub whose edges fill whole blocks."""
    n = 300_000
    rng = np.random.default_rng(3)
    hub = 5
    leaves = rng.choice(np.arange(10, n), size=5000, replace=False)
    s = np.concatenate([np.full(len(leaves), hub), rng.integers(0, n, 3000)])
    d = np.concatenate([leaves, rng.integers(0, n, 3000)])
    g = fu.Graph.from_edges(n, s, d)
    v = fu.uniform_values(g.n, seed=4)
    for kernel in KERNELS:
        eng = fu.CollectAll(g, v, kernel=kernel)
        for r in (1, 2, 3):
            eng.run(1)
            a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, r)
            assert np.array_equal(eng.estimates(), a_ref), (kernel, r)
            assert np.array_equal(eng.flows(), f_ref), (kernel, r)


def test_stage_layout_slices_and_unbuildable_graphs():
    """Kernel 8's layouts: ER-1M builds all four (1-byte codes: 16 slices of 64K nodes, the
    u16 offset limit; doubles: 62 slices of 16K), each tile within the 64 runs the u16
    index addresses."""
    g = fu.Graph.erdos_renyi(1_000_000, 4_000_000, seed=1)
    eng = fu.CollectAll(g, fu.uniform_values(g.n, seed=0), kernel="stage")
    assert eng.info()["stage_slices"] == [16, 16, 31, 62]
    eng.close()


def _check_flow_bookkeeping(g, v, a, f):
    """Each node's estimate after its average equals its value minus its outgoing flows
    (CA:107 with CA:117: Σ_j f_new = Σ fr + d·a - Σ er = v - a), so Σ a + Σ f = Σ v: the
    mass in flight is the flow sum. Both hold to rounding: per node within 4 (d + 2) u of
    |v| + Σ|f| + (d + 1)|a| + 1 (u = 2^-53; d + 2 roundings of the row's flows, its average
    and numpy's sum; the C oracle's R-MAT 18-20 outputs reach 0.44 of (d + 2) u of it, so
    the test holds at any row length, where a flat 1e-12 failed on R-MAT-24's 20th round at
    1.8e-12, a row of ~10^5 edges)."""
    idx = np.minimum(g.rowptr[:-1], g.E - 1)  # reduceat needs indices < len; empty rows -> 0
    d = np.diff(g.rowptr)
    empty = d == 0
    out = np.add.reduceat(f, idx)
    out[empty] = 0.0
    absout = np.add.reduceat(np.abs(f), idx)
    absout[empty] = 0.0
    scale = np.abs(v) + absout + (d + 1) * np.abs(a) + 1.0
    assert np.max(np.abs(a - (v - out)) / ((d + 2) * 2.0 ** -53 * scale)) < 4.0
    tot = np.sum(np.abs(v)) + np.sum(np.abs(f))
    assert abs(np.sum(a) + np.sum(f) - np.sum(v)) / tot < 1e-12


@pytest.mark.timeout(900)
def test_rmat24_degree_layout_bitwise():
    """BASELINE config 4 at full size: R-MAT scale 24 (edge factor 16; E = 5.2e8, max degree
    406,598: mega hubs, heavy rows) with the degree layout and the autotuned kernel on one
    MI355X. Rounds 0-19 (the window `rmat24_unit` times) bitwise against the C oracle (16
    threads), and the flow bookkeeping."""
    g = fu.Graph.rmat(24, 16, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    eng = fu.CollectAll(g, v, layout="degree")
    eng.run(20)
    a, f = eng.estimates(), eng.flows()
    eng.close()
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 20, nthreads=16)
    assert np.array_equal(a, a_ref)
    assert np.array_equal(f, f_ref)
    del a_ref, f_ref
    _check_flow_bookkeeping(g, v, a, f)


def test_rgg_2pow23_partition_unit_bitwise():
    """BASELINE config 5's weak-scaling unit: RggPart(2^23) at world size 1 (native slab
    generator, RCCL communicator), rounds 0-19 (the window `weak_scaling_unit` times) bitwise
    against the C oracle on the same graph."""
    from fu.dist import DistCollectAll, RggPart, unique_id

    n = 1 << 23
    part = RggPart(n, avg_deg=8.0, seed=1, nparts=1, part=0)
    v = part.values(seed=0)
    d = DistCollectAll(part.to_plan(), v, unique_id())
    d.run(20)
    g = fu.Graph.random_geometric(n, avg_deg=8.0, seed=1)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 20, nthreads=16)
    assert np.array_equal(d.estimates(), a_ref)
    assert np.array_equal(d.flows(), f_ref)
    d.close()


@pytest.mark.timeout(1100)
@pytest.mark.skipif(not os.environ.get("FU_BIG_GRAPH"), reason="set FU_BIG_GRAPH=1 (several minutes, ~90 GB of host memory)")
def test_rgg_2pow28_two_partitions_one_gpu_bitwise():
    """A graph beyond one handle's 2^31 directed edges on one MI355X: RGG 2^28 at average
    degree 9 (2.4e9 directed edges; at degree 8 it has 2,147,384,282, just under 2^31) as two
    in-process x-slab partitions (fu_part_gen_rgg, fu_dist_create_local,
    fu_dist_run_local: the halo copied into the neighbour's ghost slots every round), rounds
    0-19 bitwise against the C oracle (16 threads, 64-bit reverse index) on the global graph,
    assembled from the slabs' rows in global numbering (the slab generator's rows are the
    global generator's, test_dist_rgg_slabs_local_transport_bitwise)."""
    from fu.dist import DistCollectAll, RggPart, run_local

    import threading
    import time

    stop = threading.Event()

    def beat():  # a line every 30 s: the oracle's C calls run for minutes (ctypes drops the GIL)
        t0 = time.time()
        while not stop.wait(30):
            print(f"[big] {time.time() - t0:.0f} s", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    n, k, rounds = 1 << 28, 2, 20
    parts = [RggPart(n, avg_deg=9.0, seed=1, nparts=k, part=r) for r in range(k)]
    E = sum(p.e_local for p in parts)
    assert E > 2 ** 31 - 1
    print(f"[big] {k} slabs, E = {E}", flush=True)  # progress lines: the run takes minutes
    engs = [DistCollectAll(p.to_plan(), p.values(seed=0), None) for p in parts]
    run_local(engs, rounds)
    print("[big] rounds queued", flush=True)
    got = [(p.lo, p.hi, e.estimates(), e.flows()) for p, e in zip(parts, engs)]
    for e in engs:
        e.close()
    del engs
    print("[big] estimates and flows read back", flush=True)
    rowptr = np.empty(n + 1, dtype=np.int64)
    col = np.empty(E, dtype=np.int32)
    v = np.empty(n)
    off = 0
    for p in parts:
        rowptr[p.lo:p.hi] = p.rowptr[:-1] + off
        col[off:off + p.e_local] = p.global_col()
        v[p.lo:p.hi] = p.values(seed=0)
        off += p.e_local
    rowptr[n] = off
    del parts
    rev = coracle.rev64(rowptr, col, 16)
    print("[big] global CSR and reverse index built", flush=True)
    a_ref, f_ref = coracle.ca_sync64(rowptr, col, rev, v, rounds, nthreads=16)
    print("[big] C oracle done", flush=True)
    stop.set()
    for lo, hi, a, f in got:
        assert np.array_equal(a, a_ref[lo:hi])
        assert np.array_equal(f, f_ref[rowptr[lo]:rowptr[hi]])


@pytest.mark.timeout(900)
def test_rgg64m_single_gpu_properties():
    """BASELINE config 5's graph at full size on one GPU (2^26 nodes, E = 5.4e8): 10 rounds
    on the single-GPU engine bitwise against the C oracle, with finite estimates, the flow
    bookkeeping (Σ a + Σ f = Σ v: mass conserved counting the flows in flight) and the mean of
    the values recovered to 1e-9; then rounds 0-19 through the partitioned path at one rank
    (the `--workload rgg-dist --strong` line: slab generator, RCCL communicator) bitwise."""
    import math

    from fu.dist import DistCollectAll, RggPart, unique_id

    n = 1 << 26
    g = fu.Graph.random_geometric(n, avg_deg=8.0, seed=1)
    v = fu.uniform_values(g.n, seed=0)
    eng = fu.CollectAll(g, v)
    eng.run(10)
    a, f = eng.estimates(), eng.flows()
    eng.close()
    assert np.isfinite(a).all() and np.isfinite(f).all()
    _check_flow_bookkeeping(g, v, a, f)
    mean_v = math.fsum(v.tolist()) / n
    mass = (math.fsum(a.tolist()) + float(np.sum(f))) / n
    assert abs(mass - mean_v) < 1e-9 * mean_v
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 10, nthreads=16)
    assert np.array_equal(a, a_ref)
    assert np.array_equal(f, f_ref)
    del a, f
    part = RggPart(n, avg_deg=8.0, seed=1, nparts=1, part=0)
    d = DistCollectAll(part.to_plan(), part.values(seed=0), unique_id())
    d.run(20)
    coracle.ca_rounds(g.rowptr, g.col, g.rev, v, 10, a_ref, f_ref, nthreads=16)
    assert np.array_equal(d.estimates(), a_ref)
    assert np.array_equal(d.flows(), f_ref)
    d.close()


@pytest.mark.parametrize("seed", range(12))
def test_random_configurations_bitwise(seed):
    """Seeded random mix of graph family, size, layout, round kernel, the heavy-row / mega-hub
    thresholds and kernel 4's tile geometry (switched between runs), against the C oracle:
    every kernel and path must give the same bits."""
    rng = np.random.default_rng(1000 + seed)
    fam = rng.choice(["er", "rmat", "rr", "rgg"])
    if fam == "er":
        n = int(rng.integers(500, 40000))
        g = fu.Graph.erdos_renyi(n, int(n * rng.uniform(1, 6)), seed=seed)
    elif fam == "rmat":
        g = fu.Graph.rmat(int(rng.integers(9, 15)), int(rng.choice([4, 8, 16])), seed=seed)
    elif fam == "rr":
        g = fu.Graph.random_regular(int(rng.integers(64, 20000)) * 2, int(rng.choice([2, 4, 8])), seed=seed)
    else:
        g = fu.Graph.random_geometric(int(rng.integers(1000, 30000)), avg_deg=float(rng.uniform(3, 12)), seed=seed)
    v = fu.uniform_values(g.n, seed=seed)
    layout = str(rng.choice(["given", "degree"]))
    eng = fu.CollectAll(g, v, kernel="recon", layout=layout)
    eng.set_option("hub_threshold", int(rng.choice([16, 64, 128, 512])))
    eng.set_option("mega_hub", int(rng.choice([64, 300, 2000, 8192])))
    eng.set_option("pack_every", int(rng.choice([4, 16])))
    kern = str(rng.choice(["recon", "stage", "pregather"]))
    try:
        eng.set_option("kernel", fu.engine.KERNELS[kern])
    except fu.FuError:
        eng.set_option("kernel", 4)  # kernel 8 needs a slice layout the graph admits
    rounds = 0
    for _ in range(3):  # switch the kernel-4 tile geometry between runs (same state, same bits)
        eng.set_option("tile_edges", int(rng.choice([2048, 1024, 512])))
        k = int(rng.integers(3, 12))
        eng.run(k)
        rounds += k
    a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, rounds, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref), (fam, layout)
    assert np.array_equal(eng.flows(), f_ref), (fam, layout)


@pytest.mark.parametrize("tile", [2048, 1024, 512])
def test_c16_narrow_and_wide_tiles_bitwise(tile):
    """Kernel 4's 2-byte column offsets: an RGG (every 1024-edge block narrow) joined to an ER
    block with random columns (wide) and a few long-range edges inside the RGG part (one wide
    block among narrow ones), c16 on and off, against the C oracle."""
    import numpy as np
    a = fu.Graph.random_geometric(60_000, avg_deg=8, seed=8)
    b = fu.Graph.erdos_renyi(20_000, 80_000, seed=8)
    n = a.n + b.n
    src = [np.repeat(np.arange(a.n), np.diff(a.rowptr)), np.repeat(np.arange(b.n), np.diff(b.rowptr)) + a.n]
    dst = [np.asarray(a.col, dtype=np.int64), np.asarray(b.col, dtype=np.int64) + a.n]
    far = np.array([[5, 45_000], [100, 79_000], [30_000, 70_123]], dtype=np.int64)  # long-range edges
    s_ = np.concatenate(src + [far[:, 0], far[:, 1]])
    d_ = np.concatenate(dst + [far[:, 1], far[:, 0]])
    g = fu.Graph.from_edges(n, s_, d_)
    v = fu.uniform_values(g.n, seed=8)
    a_ref, f_ref = coracle.ca_sync(g.rowptr, g.col, g.rev, v, 25, nthreads=16)
    for c16 in (1, 0):
        eng = fu.CollectAll(g, v, kernel="recon")
        eng.set_option("tile_edges", tile)
        eng.set_option("c16", c16)
        eng.run(25)
        assert np.array_equal(eng.estimates(), a_ref), c16
        assert np.array_equal(eng.flows(), f_ref), c16
        eng.close()


def test_bench_rccl_two_ranks_parity_and_convergence():
    """bench.py --gpus 2 (rgg-dist, small slabs): the RCCL halo's parity check against the
    single-GPU engine reports "bitwise", and the line carries the error reached against the
    per-component means. Two RCCL ranks need two GPUs (RCCL refuses two ranks on one)."""
    import json
    import subprocess
    import sys

    if fu.device_count() < 2:
        pytest.skip("two RCCL ranks need two GPUs (this box has one)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--workload", "rgg-dist",
                        "--n", "262144", "--steps", "5", "--warmup", "2", "--conv-rounds", "60"],
                       capture_output=True, text=True, timeout=110, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["rccl_parity"] == "bitwise"
    assert line["err_after_conv_rounds"] is not None and line["components"] >= 1


def test_bench_rccl_parity_arrays_one_rank():
    """bench.py's RCCL correctness check, end to end at one RCCL rank (the only size one GPU
    allows): the slab run through fu_dist_create + RCCL, rank 0's single-GPU reference on
    the global RGG and the bitwise verdict. The N > 1 gather and the slab order are the
    ones test_dist_rgg_slabs_local_transport_bitwise pins on three in-process ranks."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from fu.dist import unique_id

    arrs = bench.rccl_parity_arrays(1, 0, 0, None, unique_id, n=1 << 16, rounds=12)
    assert bench.parity_verdict(*arrs) == (True, "bitwise")


def test_copy_bandwidth_plausible():
    """bench.py's roofline.copy_GBs: a float4 copy of 256 MB reads as an HBM-class rate."""
    gbs = fu.copy_bandwidth(0, 256 << 20, 3)
    assert 1000.0 < gbs < 20000.0, gbs
    with pytest.raises(fu.FuError, match="bad arguments"):
        fu.copy_bandwidth(0, 8, 1)


def test_lag_flows_every_round_and_switches():
    """Kernel 9's lag (the multi-row heavy rows leave f_r to round r + 2): the flows read
    after every round (fu_get_flows writes the lagged ones first) and the rounds that continue
    after each read, a staging-layout rebuild mid-run, the option switched off and on, the
    lagged set changed mid-run (its flows are written first), and fu_reset, all bitwise
    against the C oracle."""
    g = fu.Graph.rmat(14, 16, seed=8)
    v = fu.uniform_values(g.n, seed=8)
    eng = fu.CollectAll(g, v, kernel="pregather", hub_threshold=16, layout="given")
    eng.set_option("mega_hub", 600)
    eng.set_option("lag", 1)
    for r in range(1, 12):  # rounds 0 .. r-1 run: compare after each
        eng.run(1)
        a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, r, nthreads=16)
        assert np.array_equal(eng.estimates(), a_ref), r
        assert np.array_equal(eng.flows(), f_ref), r
    eng.run(5)
    eng.set_option("mega_hub", 700)  # tiles and staging layout rebuilt: the lagged flows are written first
    eng.run(4)
    eng.set_option("lag", 0)
    eng.run(3)
    eng.set_option("lag", 1)
    eng.set_option("multi_mid", 0)  # the lagged set shrinks between two rounds of one parity
    eng.run(7)
    a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, 11 + 5 + 4 + 3 + 7, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)
    eng.reset()
    eng.run(9)
    a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, 9, nthreads=16)
    assert np.array_equal(eng.flows(), f_ref) and np.array_equal(eng.estimates(), a_ref)


def test_lag_with_autotune_kernel_switches():
    """kernel "auto" with lag on: the autotune passes run kernel 9 (lagged) and then other
    kernels, which read F as f_{r-2}: the lagged rows' flows are written before each switch.
    200 rounds with packing every 4 rounds (re-tunes at every width), bitwise."""
    g = fu.Graph.rmat(15, 16, seed=9)
    v = fu.uniform_values(g.n, seed=9)
    eng = fu.CollectAll(g, v, kernel="auto", hub_threshold=16, layout="degree")
    eng.set_option("mega_hub", 2000)
    eng.set_option("lag", 1)
    eng.set_option("pack_every", 4)
    eng.run(200)
    a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, 200, nthreads=16)
    assert np.array_equal(eng.estimates(), a_ref)
    assert np.array_equal(eng.flows(), f_ref)


CLASS_EDGE_DEGREES = [0, 1, 2, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1023, 1024,
                      1025, 2047, 2048, 2049, 4095, 4096, 4097, 8191, 8192, 8193, 12000]


def _class_edge_graph(seed):
    """Star centres of exactly the degrees above (each row class's first and last degree: heavy
    rows at > 128, multi-row blocks at > 256, the register launch's 1024, the mega hubs at >
    8192), their leaves drawn from a random background graph that never touches a centre."""
    rng = np.random.default_rng(seed)
    k, n_leaf = len(CLASS_EDGE_DEGREES), 16000
    n = k + n_leaf
    src, dst = [], []
    for c, d in enumerate(CLASS_EDGE_DEGREES):
        leaves = k + rng.choice(n_leaf, size=d, replace=False)
        src.append(np.full(d, c))
        dst.append(leaves)
    m = 3 * n_leaf
    src.append(k + rng.integers(0, n_leaf, m))
    dst.append(k + rng.integers(0, n_leaf, m))
    g = fu.Graph.from_edges(n, np.concatenate(src), np.concatenate(dst))
    assert [int(x) for x in g.degrees[:k]] == CLASS_EDGE_DEGREES
    return g


def _isolated_then_heavy_graph(tail):
    """Layout "given" with runs of isolated rows right before a heavy row and a mega hub:
    tail = "heavy_hub" puts [..., isolated x 700, heavy (300 edges), mega hub (9000 edges)] at
    the end, "hub_iso_heavy" [..., mega hub, isolated x 700, heavy], "iso_end" keeps the
    isolated run last (the k_isolated case)."""
    rng = np.random.default_rng(21)
    n_leaf, n_iso = 12000, 700
    base = rng.integers(0, n_leaf, size=(3 * n_leaf, 2))
    src, dst = [base[:, 0]], [base[:, 1]]
    if tail == "heavy_hub":
        iso0, heavy, hub = n_leaf, n_leaf + n_iso, n_leaf + n_iso + 1
    elif tail == "hub_iso_heavy":
        hub, iso0, heavy = n_leaf, n_leaf + 1, n_leaf + 1 + n_iso
    else:
        heavy, hub, iso0 = n_leaf, n_leaf + 1, n_leaf + 2
    n = n_leaf + n_iso + 2
    src += [np.full(300, heavy), np.full(9000, hub)]
    dst += [rng.choice(n_leaf, 300, replace=False), rng.choice(n_leaf, 9000, replace=False)]
    g = fu.Graph.from_edges(n, np.concatenate(src), np.concatenate(dst))
    deg = g.degrees
    assert deg[heavy] == 300 and deg[hub] == 9000 and not deg[iso0:iso0 + n_iso].any()
    return g


@pytest.mark.parametrize("tail", ["heavy_hub", "hub_iso_heavy", "iso_end"])
@pytest.mark.parametrize("opts", [{}, {"lag": 0}, {"iso_rows": 0}, {"multi_short": 0}])
def test_isolated_rows_before_heavy_rows_given_layout_bitwise(tail, opts):
    """Kernel 9's k_isolated must not cover a heavy row or a mega hub that follows the
    trailing run of edge-less light tiles (layout "given", CollectAll's default): every row
    computed by exactly one launch, bitwise against the C oracle (CA:106-113)."""
    g = _isolated_then_heavy_graph(tail)
    v = fu.uniform_values(g.n, seed=8)
    eng = fu.CollectAll(g, v, kernel="pregather", layout="given")
    for key, val in opts.items():
        eng.set_option(key, val)
    done = 0
    for k in (1, 2, 4, 9):
        eng.run(k)
        done += k
        a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, done, nthreads=16)
        assert np.array_equal(eng.estimates(), a_ref), done
        assert np.array_equal(eng.flows(), f_ref), done
    eng.close()


@pytest.mark.parametrize("layout", ["given", "degree"])
@pytest.mark.parametrize("kernel,opts", [("recon", {}), ("recon", {"wave_heavy": 0}), ("stage", {}),
                                         ("pregather", {}), ("pregather", {"lag": 0}),
                                         ("pregather", {"multi_mid": 0}),
                                         ("pregather", {"iso_rows": 0}), ("pregather", {"tr_nt": 0, "lag": 0}),
                                         ("pregather", {"multi_short": 0}),
                                         ("pregather", {"multi_short": 1, "multi_heavy": 0})])
def test_row_class_boundaries_bitwise(kernel, opts, layout):
    """Rows of exactly the degree where each row class starts or ends, at the default
    thresholds, every kernel, against the C oracle after every few rounds (the lagged flows
    read back in between)."""
    g = _class_edge_graph(7)
    v = fu.uniform_values(g.n, seed=3)
    eng = fu.CollectAll(g, v, kernel=kernel, layout=layout)
    for key, val in opts.items():
        eng.set_option(key, val)
    done = 0
    for k in (1, 2, 5, 9):
        eng.run(k)
        done += k
        a_ref, f_ref = coracle.ca_sync(*g.arrays(), v, done, nthreads=16)
        assert np.array_equal(eng.estimates(), a_ref), done
        assert np.array_equal(eng.flows(), f_ref), done
