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
