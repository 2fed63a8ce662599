"""Host logic of bench.py (no GPU): the oracle row check attached to the CPU baseline, and
the batch sizing of the timed frames."""
import numpy as np

import bench


def test_oracle_rows_check():
    rng = np.random.default_rng(0)
    gpu = rng.random((40, 16, 3), dtype=np.float32) * 4000
    cpu = gpu.copy()
    r = bench.oracle_rows_check(gpu, cpu, [0, 5, 39])
    assert r["ok"] and r["all_bit_exact"] and r["max_abs_diff"] == 0.0 and r["pixels"] == 48
    cpu[5, 3, 1] = np.nextafter(cpu[5, 3, 1], np.float32(np.inf))  # one ulp at ~4000: 2.4e-4
    r = bench.oracle_rows_check(gpu, cpu, [0, 5, 39])
    assert not r["ok"] and r["max_abs_diff"] > 1e-4 and abs(r["bit_exact_pixel_frac"] - 47 / 48) < 1e-6
    r = bench.oracle_rows_check(gpu, cpu, [0, 39])  # the differing row not sampled
    assert r["ok"]
    cpu = gpu.copy()
    cpu[0, 0, 0] = np.nan
    r = bench.oracle_rows_check(gpu, cpu, [0])
    assert not r["ok"] and not r["nan_pattern_equal"]
    gpu[0, 0, 0] = np.nan
    assert bench.oracle_rows_check(gpu, cpu, [0])["ok"]
