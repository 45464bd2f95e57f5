"""bench.py's host-side pieces that need no GPU: the live launch timer's statistics and the
ppo_adam_banks_t mirror the chained update passes through the C ABI."""
import ctypes

import pytest


class _Ev:
    """Stand-in for a torch.cuda.Event pair member: elapsed_time(other) returns a fixed value."""

    def __init__(self, ms):
        self.ms = ms

    def elapsed_time(self, other):
        return self.ms


def test_kernel_timer_median_minus_empty_pair():
    bench = pytest.importorskip("bench")
    kt = bench.KernelTimer(spin_cycles=0)
    # 5 launches, one of them a cold outlier; the median ignores it
    kt.pairs = [(_Ev(v), None) for v in (0.030, 0.031, 0.090, 0.029, 0.030)]
    kt.empty = [(_Ev(v), None) for v in (0.005, 0.006, 0.005, 0.005, 0.004)]
    assert kt.raw_ms() == pytest.approx(0.030)
    assert kt.overhead_ms() == pytest.approx(0.005)
    assert kt.mean_ms() == pytest.approx(0.025)
    kt.pairs = [(_Ev(v), None) for v in (0.010, 0.020)]
    assert kt.raw_ms() == pytest.approx(0.015)   # even count: mean of the middle two
    assert bench.KernelTimer().raw_ms() != bench.KernelTimer().raw_ms()   # NaN without launches


def test_adam_banks_struct_matches_header():
    from omniisaacgymenvs_loop_amd._abi import PpoAdamBanks
    names = [f[0] for f in PpoAdamBanks._fields_]
    assert names == ["params", "m", "v", "opt"]
    assert ctypes.sizeof(PpoAdamBanks) == 7 * ctypes.sizeof(ctypes.c_void_p)
    b = PpoAdamBanks()
    b.params[0], b.params[1] = 16, 32
    assert (b.params[0], b.params[1]) == (16, 32)


class _At:
    """An event at a fixed time: a.elapsed_time(b) = b.t - a.t."""

    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def test_phase_split_from_timed_epoch_events():
    """The rollout / update split of the timed epochs (events recorded inside them): means, the epochs named,
    and host_gap_ms = ms_per_step - rollout - update (>= 0 whenever the events lie inside the timed epochs)."""
    bench = pytest.importorskip("bench")
    ev = [(_At(0.0), _At(10.0), _At(60.0)), (_At(100.0), _At(112.0), _At(164.0))]
    ph = bench.phase_split(ev, 65.0, 2048, 30)
    assert ph["rollout_ms"] == pytest.approx(11.0) and ph["update_ms"] == pytest.approx(51.0)
    assert ph["host_gap_ms"] == pytest.approx(3.0) and ph["host_gap_ms"] >= 0
    assert ph["update_us_per_minibatch"] == pytest.approx(51.0e3 / 2048)
    assert ph["rollout_ms_min_max"] == [10.0, 12.0] and "epochs 29-30" in ph["phase_method"]
    assert bench.phase_split([], 65.0, 2048, 30) == {}


def test_multi_rank_line_fields_under_torchrun_gloo(tmp_path):
    """A two-rank torchrun (gloo, CPU): the line's config.exchange, extra.dp_selftest per rank and extra.ranks with
    each rank's device, task, epoch ms and minibatch update time, gathered in rank order."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = 29000 + os.getpid() % 2000
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(root, "tests", "_bench_ranks_worker.py")],
                         capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["config"]["exchange"] == "peer"
    assert line["extra"]["dp_selftest"] == {"0": "pass", "1": "pass"}
    ranks = line["extra"]["ranks"]
    assert [r["rank"] for r in ranks] == [0, 1]
    assert [r["task"] for r in ranks] == ["GoToPose", "TrackXYOVelocity"]
    assert ranks[1]["epoch_ms"] == pytest.approx(65.0) and ranks[0]["epoch_ms"] == pytest.approx(60.0)
    assert [r["update_us_per_minibatch"] for r in ranks] == [25.0, 26.0]
    assert all(r["device"].endswith("/cpu") for r in ranks)


def test_dp_fields_names_a_mixed_exchange():
    bench = pytest.importorskip("bench")
    recs = [{"rank": 0, "exchange": "peer", "selftest": "pass"},
            {"rank": 1, "exchange": "collective", "selftest": "fail"}]
    ex, extra = bench.dp_fields(recs)
    assert ex == "mixed: collective, peer" and extra["dp_selftest"] == {"0": "pass", "1": "fail"}
