"""Offline LDS bank-conflict checks of kernel tile layouts (bench/lds_sim.py, the
MI355X_MICROARCH.md LDS banking model): no GPU needed."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))


def test_conv_halo_swizzle_conflict_free():
    import lds_sim
    # conv_halo.hip fwd/dgrad A and B fragment reads: 4 LDS cycles per ds_read_b128 = no conflict
    assert lds_sim.check_halo(4) == 4
    assert lds_sim.check_halo(8) == 4


def test_gemm_kc_swap_conflict_free():
    import lds_gemm_kc as m
    # gemm.hip K-contiguous images at 48-element rows: odd-row block swap -> 1 cycle per group
    assert m.store(48, True, False) == 1 and m.store(48, True, True) == 1
    assert all(m.read(48, True, r0) == 1 for r0 in (0, 16, 32, 48))
    assert m.store(48, False, False) == 2


def test_gemm256_swizzles_conflict_free():
    import lds_gemm256 as m
    # gemm256.hip LDS-DMA images: linear would be 4-way (KC b128) / 8-way (MN tr_b16)
    assert m.kc_worst(lambda r: 0) == 4 and m.mn_worst(lambda r: 0) == 8
    assert m.kc_worst(m.kc_swz) == 1 and m.mn_worst(m.mn_swz) == 1
