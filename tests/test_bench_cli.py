"""bench.py's multi-GPU contract, on the CPU: `--gpus N` without a launcher starts N rank
processes itself, and a node with fewer visible GPUs than ranks is an error (never a silent
one-GPU line). Also the timed-region chunking and the pairwise byte model."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_gpus2_forks_two_ranks_and_fails_without_gpus():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "0", "--no-conv", "--cpu-seconds", "0"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert "[bench] rank 0/2" in p.stderr and "[bench] rank 1/2" in p.stderr
    assert "need 2 GPU(s), 0 visible" in p.stderr
    assert '"metric"' not in p.stdout  # no JSON line for GPUs that do not exist


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode == 2 and "WORLD_SIZE=1 but --gpus 4" in p.stderr


@pytest.mark.parametrize("steps", [1, 2, 5, 20, 1000])
def test_chunk_bounds(steps):
    b = bench.chunk_bounds(steps)
    assert b[0] == 0 and b[-1] == steps and all(x < y for x, y in zip(b, b[1:]))
    if steps > 1:
        assert b[1] == 1  # round 0 timed alone
        assert len(b) - 2 <= (1 if steps <= 100 else 10)


def test_pairwise_bytes_model():
    # RECV, FIRE_PW over 8 flows, FIRE_CA over 3 neighbours
    ev = np.array([[0, 1, 5, 0], [2, 1, 8, 7], [1, 3, 0, 0]], dtype=np.int32)
    assert bench.pairwise_bytes(ev, None, None) == 32 + (8 * 8 + 56) + (48 * 3 + 16)
    # receive + pairwise fire at degree 8 = SURVEY §8(d)'s 136 B per exchange (+16 B of state)
    assert 32 + 8 * 8 + 56 == 152


def test_dist_line_schema():
    """The N > 1 (rgg-dist) line is self-contained: halo bytes inside the per-GPU roofline
    bytes, the halo's measured share of the round, no number read from a committed file,
    cpu_baseline left to the N = 1 line."""
    kinfo = {"kernel": "recon", "tile": (1024, 128)}
    line = bench.dist_line(world=4, steps=20, warmup=5, wall=0.01, dev1_ms=6.0, e_tot=4 * 67_000_000,
                           n_tot=4 * 8_388_608, halo=4 * 40_000, n_total=4 * 8_388_608, per=8_388_608,
                           kinfo=kinfo, halo_us=12.0, round_us=6.0e3 / 19, t_gen=1.0,
                           conv={"rounds_to_1e-9": None, "conv_note": "x"})
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "cpu_baseline", "halo", "rounds_to_1e-9"):
        assert key in line, key
    assert line["n_gpus"] == 4 and line["scaling"] == "weak"
    assert line["value"] == 4 * 67_000_000 * 20 / 0.01
    roof = line["roofline"]
    assert roof["alg_bytes_per_launch"] == (24 * 67_000_000 + 28 * 8_388_608 + 8 * 40_000)
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-12
    assert roof["avg_launch_us"] == 6.0e3 / 19
    assert line["config"]["halo_bytes_per_round"] == 8 * 4 * 40_000
    assert abs(line["halo"]["share_of_round"] - 12.0 / (6.0e3 / 19)) < 1e-12
    assert line["cpu_baseline"] is None and "one_rank_reference" not in line
    json_text = __import__("json").dumps(line)
    assert "profiles/" not in json_text  # nothing read from committed files


def test_weak_unit_flag():
    """The default N = 1 line measures config 5's per-GPU unit beside the headline (on the
    GPU); --no-unit skips it."""
    assert bench.parse([]).no_unit is False
    assert bench.parse(["--no-unit"]).no_unit is True


def test_dist_line_strong_scaling():
    """--strong (BASELINE config 5 as written: 2^26 nodes split over the ranks) is labelled."""
    kinfo = {"kernel": "recon", "tile": (1024, 128)}
    line = bench.dist_line(world=8, steps=20, warmup=5, wall=0.01, dev1_ms=6.0, e_tot=8 * 67_000_000,
                           n_tot=1 << 26, halo=8 * 40_000, n_total=1 << 26, per=(1 << 26) // 8,
                           kinfo=kinfo, halo_us=12.0, round_us=6.0e3 / 19, t_gen=1.0,
                           conv={"rounds_to_1e-9": None}, strong=True)
    assert line["scaling"] == "strong" and "strong scaling" in line["config"]["workload"]
    assert bench.parse(["--strong"]).strong is True and bench.parse([]).strong is False


def test_dist_line_rccl_parity_and_traffic_fields():
    """N > 1 lines carry the RCCL halo's correctness bit and the per-GPU PMC traffic."""
    kinfo = {"kernel": "recon", "tile": (1024, 128)}
    chk = {"status": "bitwise", "graph": "rgg", "rounds": 30, "against": "x"}
    line = bench.dist_line(world=2, steps=20, warmup=5, wall=0.01, dev1_ms=6.0, e_tot=2 * 67_000_000,
                           n_tot=2 * 8_388_608, halo=2 * 40_000, n_total=2 * 8_388_608, per=8_388_608,
                           kinfo=kinfo, halo_us=12.0, round_us=6.0e3 / 19, t_gen=1.0,
                           conv={"rounds_to_1e-9": None, "err_after_conv_rounds": 0.6}, rccl_parity=chk,
                           traffic=1.7e9)
    assert line["rccl_parity"] == "bitwise" and line["rccl_parity_check"] == chk
    assert line["roofline"]["traffic"] == 1.7e9
    assert line["err_after_conv_rounds"] == 0.6
    one = bench.dist_line(world=1, steps=20, warmup=5, wall=0.01, dev1_ms=6.0, e_tot=67_000_000,
                          n_tot=8_388_608, halo=0, n_total=8_388_608, per=8_388_608, kinfo=kinfo,
                          halo_us=1.0, round_us=300.0, t_gen=1.0, conv={})
    assert one["rccl_parity"].startswith("n/a")


def test_parity_verdict():
    a = np.arange(10, dtype=np.float64)
    f = np.linspace(-1, 1, 40)
    assert bench.parity_verdict([a[:4], a[4:]], [f[:15], f[15:]], a, f) == (True, "bitwise")
    a2 = a.copy()
    a2[3] = np.nextafter(a2[3], 10.0)  # one ulp
    ok, why = bench.parity_verdict([a2[:4], a2[4:]], [f], a, f)
    assert not ok and "1 estimates and 0 flows" in why
    z = np.array([0.0])
    assert not bench.parity_verdict([np.array([-0.0])], [f], z, f)[0]  # signed zero counts
    assert not bench.parity_verdict([a[:4]], [f], a, f)[0]


def test_rccl_parity_mismatch_exits_nonzero(monkeypatch, capsys):
    """A wrong halo must not produce a fast, plausible line: rank 0's mismatch ends the run
    with status 5 (every rank, through the broadcast verdict)."""
    a = np.arange(6, dtype=np.float64)
    f = np.arange(12, dtype=np.float64)
    bad = a.copy()
    bad[5] += 1.0
    monkeypatch.setattr(bench, "rccl_parity_arrays", lambda *x, **k: ([bad[:3], bad[3:]], [f], a, f))
    with pytest.raises(SystemExit) as ex:
        bench.rccl_parity(2, 0, 0, None, lambda: b"")
    assert ex.value.code == 5
    assert "RCCL parity FAILED" in capsys.readouterr().err
    monkeypatch.setattr(bench, "rccl_parity_arrays", lambda *x, **k: ([a[:3], a[3:]], [f], a, f))
    assert bench.rccl_parity(2, 0, 0, None, lambda: b"")["status"] == "bitwise"


def test_pmc_traffic_per_gpu_record(tmp_path, monkeypatch):
    import json

    rec = [{"n": 8388608, "E": 67000000, "kernel_selected": "rgg-dist", "rounds_timed": 20,
            "bytes_per_launch": 1.8e9}]
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_traffic(8388608, None, "rgg-dist", 20, per_gpu=True) == 1.8e9
    assert bench.pmc_traffic(8388608, None, "rgg-dist", 21, per_gpu=True) is None
    assert bench.pmc_traffic(8388608, 5, "rgg-dist", 20) is None


class _FakeGraph:
    def __init__(self, n, E):
        self.n, self.E, self.max_deg = n, E, 8
        self.rowptr = np.zeros(n + 1, dtype=np.int64)
        self.col = np.zeros(0, dtype=np.int32)


class _FakeEngine:
    """A CollectAll stand-in for the bench's control flow on the CPU: rounds advance a
    counter, every round 'takes' 50 us, the packing plan narrows at rounds 110/150/200."""
    def __init__(self, g, v, device=0, kernel="auto", layout="given"):
        self.r, self.marks, self.kernel = 0, {}, kernel

    def tune(self):
        pass

    def run(self, k, err_every=0):
        self.r += k
        return np.zeros(max(k // err_every, 1)) if err_every else None

    def synchronize(self):
        pass

    def estimates(self):
        return np.zeros(4)

    def pack_widths(self):
        w = 8 if self.r >= 200 else 16 if self.r >= 150 else 32 if self.r >= 110 else 0
        return (w, w, w)

    def reset(self):
        self.r = 0

    def mark(self, slot):
        self.marks[slot] = self.r

    def run_marked(self, b):
        base = self.r
        for k, x in enumerate(b):
            self.marks[k] = base + x
        self.r = base + b[-1]

    def elapsed(self, a, b):
        return (self.marks[b] - self.marks[a]) * 0.05

    def info(self):
        return {"kernel": "stage", "tile": (1024, 128), "tune_passes": 1,
                "tune_us_per_round": {"stage": 50.0}, "tune_winner_by_width": {0: "stage"}}

    def close(self):
        pass


class _FakeReplay:
    def __init__(self, tr, v, device=0, persistent=False):
        self.tr = tr

    def run(self, tick_end, snapshot_ticks=()):
        return {}

    def run_timed(self, tick_end):
        return 0.5

    def close(self):
        pass


def test_n1_line_carries_config2_rmat24_pairwise_units(monkeypatch, capsys):
    """The driver's N = 1 command (--steps 20 --warmup 5) measures BASELINE configs 2 (as
    written: 1000 rounds), 4 (R-MAT-24) and 3 (pairwise RR-64K, ticks 101-500) beside the
    headline, each guarded so that a failure keeps the headline line (CPU: fake engines)."""
    import json

    import fu

    graphs = {"er": _FakeGraph(1_000_000, 7_999_972), "rmat": _FakeGraph(1 << 24, 520_761_504)}
    monkeypatch.setattr(bench, "make_graph", lambda wl, n, m: (graphs[wl], f"{wl} fake"))
    monkeypatch.setattr(fu, "CollectAll", _FakeEngine)
    monkeypatch.setattr(fu, "Replay", _FakeReplay)
    monkeypatch.setattr(fu, "uniform_values", lambda n, seed=0: np.zeros(n))
    monkeypatch.setattr(fu, "copy_bandwidth", lambda *a: 5500.0)
    monkeypatch.setattr(bench, "measure_dist", lambda *a: {
        "config": {"workload": "rgg", "E_directed": 1, "kernel_selected": "recon", "tile_selected": (1024, 128)},
        "value": 1.0, "unit": "edge-updates/s", "ms_per_step": 1.0,
        "roofline": {"frac": 0.7, "avg_launch_us": 300.0}})
    args = bench.parse(["--steps", "20", "--warmup", "5", "--no-conv", "--cpu-seconds", "0"])
    bench.run_single(args, "er")
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["steps"] == 20 and line["roofline"]["copy_GBs"] == 5500.0
    st = line["config"]["settle"]  # untimed rounds right before the window (>= 25 ms)
    assert st["ms"] == 25.0 and st["rounds"] >= 16 and st["rounds"] % 16 == 0
    io = line["host_io"]  # the PCIe-inclusive rate, beside (never as) the value
    assert io["host_bytes_in"] == 8 * 1_000_001 + 4 * 7_999_972 + 8 * 1_000_000
    assert 0 < io["value_with_create_and_download"] <= line["value"]
    c2 = line["config2_1000"]
    assert "error" not in c2, c2
    assert abs(c2["avg_round_us"] - 50.0) < 1e-9 and len(c2["phases"]) == 11
    assert abs(c2["frac"] - (24 * 7_999_972 + 28 * 1_000_000) / 50e-6 / 1e9 / 8000.0) < 1e-9
    assert [p["width"] for p in c2["pack_width_schedule"]] == [0, 32, 16, 8]
    rm = line["rmat24_unit"]
    assert "error" not in rm, rm
    assert rm["E_directed"] == 520_761_504 and rm["steps"] == 20
    assert abs(rm["frac"] - (24 * 520_761_504 + 28 * (1 << 24)) / 50e-6 / 1e9 / 8000.0) < 1e-9
    pw = line["pairwise_unit"]
    assert "error" not in pw, pw
    assert "ticks 101-500" in pw["workload"] and abs(pw["us_per_tick"] - 0.5e3 / 400) < 1e-3
    assert line["weak_scaling_unit"]["roofline_frac"] == 0.7
    # a failing companion keeps the headline
    monkeypatch.setattr(bench, "rmat24_unit", lambda a: 1 / 0)
    bench.run_single(args, "er")
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert "ZeroDivisionError" in line["rmat24_unit"]["error"] and line["value"] > 0


def test_window_stats_lookup(tmp_path, monkeypatch):
    import json

    d = tmp_path / "profiles" / "r05"
    d.mkdir(parents=True)
    rec = {"n": 10, "E": 40, "kernel_selected": "stage", "rounds_timed": 20, "avg_round_us": 60.0, "frac": 0.45,
           "per_kernel_per_round": {"k_stage": 17.0}}
    (d / "x_window_stats.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    ws = bench.window_stats(10, 40, "stage", 20)
    assert ws["file"] == os.path.join("profiles", "r05", "x_window_stats.json") and ws["frac"] == 0.45
    assert bench.window_stats(10, 40, "stage", 21) is None


def _replica_rank(rank, port, outdir):
    import contextlib
    import io
    import json

    import torch.distributed as dist

    import fu

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", world_size=2, rank=rank)
    fu.Replay = _FakeReplay
    args = bench.parse(["--gpus", "2", "--workload", "pairwise", "--steps", "40", "--warmup", "10", "--n", "4096",
                        "--cpu-seconds", "0"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.run_pairwise_replicas(args, 2, rank, rank, dist)
    with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
        f.write(buf.getvalue())


def test_pairwise_replicas_at_two_ranks(tmp_path):
    """--workload pairwise at N > 1 runs replicas (the replay does not shard):
    rank 0's line sums the replicas' updates over the slowest rank's wall time (gloo, two
    processes on the CPU; the trace is real, the replay faked)."""
    import json

    import torch.multiprocessing as mp

    mp.spawn(_replica_rank, args=(bench._free_port(), str(tmp_path)), nprocs=2, join=True)
    line = json.loads((tmp_path / "r0.txt").read_text().strip().splitlines()[-1])
    assert (tmp_path / "r1.txt").read_text().strip() == ""
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and "replicas x2" in line["config"]["parallelism"]
    assert abs(line["value"] - 2 * line["value_per_gpu"]) < 1e-6 * line["value"]
    assert line["cpu_baseline"] is None


class _RecordingDist:
    """A DistCollectAll stand-in that records, in order, every call of bench.py's N > 1
    sequence that moves rounds (each round is one halo exchange) or runs a collective (the
    kernel option, the error all-reduce): a rank whose sequence differs would hang RCCL. Its
    autotune pass runs the rounds FP::tune_rounds_fixed gives for this rank's own state
    (tools/plan_check --tune-rank), which the test makes differ from rank to rank."""
    log = None
    tune_rounds = None

    def __init__(self, plan, values, uid, device=0, kernel="auto"):
        self.n, self.E = plan.n_local, plan.e_local
        self.log.append(["create", kernel])

    def tune(self):
        self.log.append(["rounds", self.tune_rounds, "tune"])

    def run(self, rounds, err_every=0):
        self.log.append(["rounds", int(rounds), "err" if err_every else ""])
        return np.zeros(max(rounds // err_every, 1)) if err_every else None

    def run_marked(self, b):
        self.log.append(["rounds", int(b[-1]), "marked"])

    def reset(self):
        self.log.append(["reset"])

    def synchronize(self):
        pass

    def set_targets(self, t):
        pass

    def halo_ms(self):
        return 0.01

    def elapsed(self, a, b):
        return 0.3

    def estimates(self):
        return np.zeros(self.n)

    def flows(self):
        return np.zeros(self.E)

    def info(self):
        return {"kernel": "recon", "tile": (1024, 128)}

    def close(self):
        pass


class _RefEngine:
    def __init__(self, g, v, device=0, **k):
        self.n, self.E = g.n, g.E

    def run(self, rounds, err_every=0):
        pass

    def estimates(self):
        return np.zeros(self.n)

    def flows(self):
        return np.zeros(self.E)

    def close(self):
        pass


def _dist_sequence_rank(rank, world, port, outdir, table):
    import json

    import torch.distributed as dist

    import fu
    import fu.dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", world_size=world, rank=rank)
    log = []
    _RecordingDist.log = log
    # this rank's autotune state: kernel 8 / 9 layouts and candidate drops differ by rank
    _RecordingDist.tune_rounds = table[rank]
    fu.dist.DistCollectAll = _RecordingDist
    fu.dist.unique_id = lambda: bytes(128)
    fu.CollectAll = _RefEngine
    monkey = bench.RCCL_PARITY_N
    bench.RCCL_PARITY_N = 1 << 14
    try:
        args = bench.parse(["--gpus", str(world), "--workload", "rgg-dist", "--steps", "20", "--warmup", "5",
                            "--n", str(1 << 13), "--conv-rounds", "300", "--cpu-seconds", "0"])
        line = bench.measure_dist(args, world, rank, rank, dist)
    finally:
        bench.RCCL_PARITY_N = monkey
    with open(os.path.join(outdir, f"seq{rank}.json"), "w") as f:
        json.dump({"log": log, "line": line}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dist_sequence_identical_on_every_rank(tmp_path, world):
    """bench.py --gpus N (N = 2, 4, 8): every rank runs the same sequence of round counts and
    collectives -- the RCCL parity prelude (30 rounds), the kernel option, the autotune pass,
    the warmup, the fixed 80-round settle, the timed window, the halo samples and the
    convergence run with its per-round error all-reduce -- although the ranks' own autotune
    states differ (kernel 8 / 9 layouts present or not, candidates dropped on their own
    timings): the pass's round count comes from FP::tune_rounds_fixed for each rank's state
    (tools/plan_check --tune-rank). A rank whose count differed would hang RCCL instead of
    failing (CA:74, CA:124). gloo on the CPU, engines recorded, graphs and plans real."""
    import json
    import subprocess

    import torch.multiprocessing as mp

    from conftest import ROOT

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), "bin/plan_check"], check=True)
    pc = os.path.join(ROOT, "tools", "bin", "plan_check")
    table = []
    for rank in range(world):
        k8, k9, code = int(rank % 2 == 0), int(rank % 3 == 0), (rank * 77) % 256
        out = subprocess.run([pc, "--tune-rank", "0", str(k8), str(k9), str(code)], check=True,
                             capture_output=True, text=True).stdout.split()
        table.append(int(out[1]))
    mp.spawn(_dist_sequence_rank, args=(world, bench._free_port(), str(tmp_path), table), nprocs=world, join=True)
    seqs = [json.loads((tmp_path / f"seq{r}.json").read_text()) for r in range(world)]
    for r in range(1, world):
        assert seqs[r]["log"] == seqs[0]["log"], r
    log = seqs[0]["log"]
    rounds = [e for e in log if e[0] == "rounds"]
    assert rounds[0] == ["rounds", bench.RCCL_PARITY_ROUNDS, ""]          # the parity prelude
    assert ["rounds", table[0], "tune"] in rounds and table[0] == 36      # one pass, FP::tune_rounds_fixed
    assert ["rounds", 5, ""] in rounds and ["rounds", 80, ""] in rounds   # warmup, settle
    assert ["rounds", 20, "marked"] in rounds and ["rounds", 300, "err"] in rounds
    line = seqs[0]["line"]
    assert line["config"]["settle_rounds"] == 80 and line["rccl_parity"] == "bitwise"
    assert all(s["line"] is None for s in seqs[1:])
