"""The oracle (oracle/) against the golden fixtures produced from the reference's own Peer
arithmetic (tests/golden/make_golden.py). This pins the oracle before anything trusts it."""
import numpy as np
import pytest

import coracle
import oracle
from conftest import ca_sync_fixtures, load_json, load_npz, tick_fixtures


@pytest.mark.parametrize("name,meta", ca_sync_fixtures())
def test_python_oracle_ca_sync(name, meta):
    d = load_npz(meta["file"])
    rounds = [int(r) for r in d["rounds"]]
    snaps = oracle.ca_sync(d["rowptr"], d["col"], d["values"], max(rounds) + 1,
                           snapshot_rounds=rounds)
    for k, r in enumerate(rounds):
        assert np.array_equal(snaps[r][0], d["last_avg"][k]), (name, r)
        assert np.array_equal(snaps[r][1], d["flows"][k]), (name, r)


@pytest.mark.parametrize("name,meta", ca_sync_fixtures())
@pytest.mark.parametrize("threads", [1, 4])
def test_c_oracle_ca_sync(name, meta, threads):
    d = load_npz(meta["file"])
    rev = oracle.build_rev(d["rowptr"], d["col"])
    for k, r in enumerate(int(x) for x in d["rounds"]):
        a, f = coracle.ca_sync(d["rowptr"], d["col"], rev, d["values"], r + 1, threads)
        assert np.array_equal(a, d["last_avg"][k]), (name, r)
        assert np.array_equal(f, d["flows"][k]), (name, r)


@pytest.mark.parametrize("name,meta", ca_sync_fixtures())
def test_c_oracle_ca_sync64(name, meta):
    """The 64-bit reverse-index variant (graphs of 2^31 or more directed edges): its index
    equals build_rev's and its rounds the same fixtures bitwise."""
    d = load_npz(meta["file"])
    rev = coracle.rev64(d["rowptr"], d["col"], 4)
    assert np.array_equal(rev, oracle.build_rev(d["rowptr"], d["col"]).astype(np.int64))
    for k, r in enumerate(int(x) for x in d["rounds"]):
        a, f = coracle.ca_sync64(d["rowptr"], d["col"], rev, d["values"], r + 1, 4)
        assert np.array_equal(a, d["last_avg"][k]), (name, r)
        assert np.array_equal(f, d["flows"][k]), (name, r)


@pytest.mark.parametrize("name,fn", tick_fixtures())
def test_tick_emulator(name, fn):
    d = load_json(fn)
    em = oracle.TickEmulator(d["actors"], d["mode"])
    keys, vals = [], []

    def cb(t, e):
        it = e.last_avg_items()
        keys.append([k for k, _ in it])
        vals.append([v for _, v in it])

    em.run(d["ticks"], d["order"], on_tick=cb)
    assert [list(x) for x in em.events] == d["events"]
    assert em.fires == d["fires"]
    assert keys == d["snap_keys"]
    assert vals == d["snap_vals"]  # bitwise (JSON floats round-trip exactly)
    assert [[em.idx[x] for x in nd.nbrs] for nd in em.nodes] == d["neighbors"]
    assert [[nd.flows.get(x, 0.0) for x in nd.nbrs] for nd in em.nodes] == d["flows"]
    assert em.errors == d["errors_logged"]


def test_known_answers_small_platform():
    """first collect-all average v/(deg+1), first pairwise fire v/2^deg,
    and convergence to 190/6 by t=1000 within 1e-12 relative in every tie order."""
    ca = load_json("tick_small_platform_ca_fwd.json")
    first = {}
    em = oracle.TickEmulator(ca["actors"], "ca")

    def cb(t, e):
        for i, v in e.last_avg_items():
            first.setdefault(i, v)

    em.run(50, "fwd", on_tick=cb)
    assert [first[i] for i in range(6)] == [3.75, 3.3333333333333335, 6.666666666666667, 20.0,
                                            26.666666666666668, 1.25]
    pw = oracle.TickEmulator(ca["actors"], "pw").run(52, "fwd")
    assert [pw.nodes[i].last_avg for i in range(6)] == [1.875, 2.5, 5.0, 15.0, 20.0, 0.625]
    mean = 190 / 6
    for mode in ("ca", "pw"):
        for tag in ("fwd", "rev", "rand7"):
            d = load_json(f"tick_small_platform_{mode}_{tag}.json")
            final = d["snap_vals"][1000]
            assert max(abs(x - mean) / mean for x in final) < 1e-12, (mode, tag)


def test_replay_oracle_matches_emulator_small():
    """oracle.replay_trace on an emulator-derived trace == the emulator (self-consistency of
    the event format)."""
    from conftest import fixture_decl_csr
    import fu

    d = load_json("tick_small_platform_pw_fwd.json")
    names, vals, rp, col = fixture_decl_csr(d)
    tr = fu.Trace(rp, col, "pairwise", d["ticks"], d["order"])
    a = tr.arrays()
    last, flow, est, snaps = oracle.replay_trace(a["rowptr"], vals, a["tick_task_off"],
                                                 a["tasks"], a["events"], a["out_ids"],
                                                 tr.n_msgs, snapshot_ticks=[1000])
    order = tr.last_avg_order()
    assert [float(snaps[1000][i]) for i in order] == d["snap_vals"][1000]
