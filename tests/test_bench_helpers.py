"""CPU: bench.py's helpers that shape the measurement (no GPU): the ring
passes of equal size, the per-launch statistic by rate
(launches of different sizes compared per byte), and the CPU-baseline pinning
(one hardware thread per core, within the process's affinity)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_even_ring_equal_passes():
    assert bench.even_ring(100000, 10240) == 10000          # 10 x 10 000, not 9 x 10 240 + 7 840
    assert bench.even_ring(10000, 10240) == 10000
    assert bench.even_ring(12500, 10240) == 6250
    assert bench.even_ring(7, 0) == 1
    for n, cap in ((100000, 10240), (99999, 777), (5, 3), (1, 1)):
        r = bench.even_ring(n, cap)
        passes = -(-n // r)
        assert r <= max(1, cap) and passes == -(-n // max(1, min(n, cap)))
        assert r * passes - n < passes                       # passes differ by at most one object


def test_launch_distribution_per_byte():
    # two launch sizes: a 7 840-object tail is not a slow launch by time
    big, small = 10240 * 8 << 20, 7840 * 8 << 20
    ms = [11.2] * 9 + [11.2 * small / big]
    d = bench.launch_distribution(ms, [big] * 9 + [small], per_step=10)
    assert d["slow_share_rate_below_p90_over_1.06"] == 0.0
    assert d["launch_bytes"] == sorted({big, small})
    # one launch 10 % slower per byte is counted, with its index and position
    ms2 = [11.2] * 19 + [12.4]
    d2 = bench.launch_distribution(ms2, [big] * 20, per_step=10)
    assert d2["slow_share_rate_below_p90_over_1.06"] == 0.05
    assert d2["slow_launch_indices"] == [19] and d2["slow_by_position_in_step"][9] == 1


def test_pin_cpus_within_affinity_one_per_core():
    aff = sorted(os.sched_getaffinity(0))
    n = min(4, len(aff))
    cpus = bench.pin_cpus(0, n)
    assert len(cpus) == n and len(set(cpus)) == n and set(cpus) <= set(aff)
    for policy in ("local", "any"):
        assert set(bench.pin_cpus(0, n, policy)) <= set(aff)


def test_pcie_link_without_a_gpu_is_none():
    """The D2H sample's link probe never raises: no GPU (or no sysfs) -> None."""
    import torch
    assert bench.pcie_link(torch, 0) is None or all(isinstance(s, str) for s in bench.pcie_link(torch, 0))

    class NoCuda:
        class cuda:
            @staticmethod
            def get_device_properties(dev):
                raise RuntimeError("no GPU")
    assert bench.pcie_link(NoCuda, 0) is None
