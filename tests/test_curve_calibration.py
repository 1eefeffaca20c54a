"""The fp32 loss-curve bars of tests/test_gpu_golden.py (CAL_*) against the
calibration population they were set from (CPU, fixture only): every one of
the seven independent fp32 samples of the 100 steps (oracle/make_golden.py
curvecal4 / curvecal16) passes when judged against the envelope of the other
six -- the bars admit every legitimate fp32 summation order sampled -- and a
curve that stops training (a broken backward) fails them."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

CAL_MIN_FRAC, CAL_MAX_X, CAL_L1_X = 0.80, 3.0, 3.0


def _judge(dev, pdev):
    n = dev.size
    env = pdev.max(0)
    local = np.array([env[max(0, i - 2):i + 3].max() for i in range(n)])
    return (np.mean(dev <= 3 * local + 1e-4) >= CAL_MIN_FRAC and dev.max() <= CAL_MAX_X * env.max()
            and dev.sum() <= CAL_L1_X * pdev.sum(1).max())


@pytest.mark.parametrize("batch", [4, 16])
def test_every_fp32_sample_passes_against_the_others(batch):
    gd = np.load(os.path.join(GOLDEN, f"loss_curve_res299_b{batch}.npz"))
    ref = gd["losses"]
    pop = np.vstack([gd["losses_fp32_cpu"][None], gd["losses_fp32_cal"]])
    assert len(pop) >= 7
    pdev = np.abs(pop - ref)
    for k in range(len(pop)):
        assert _judge(pdev[k], np.delete(pdev, k, 0)), k
    # a run that stops learning after step 10 (e.g. a dropped gradient term)
    stalled = np.concatenate([ref[:10], np.full(len(ref) - 10, ref[9])])
    assert not _judge(np.abs(stalled - ref), pdev)


def test_calibration_bars_match_the_gpu_test():
    import test_gpu_golden as T
    assert (T.CAL_MIN_FRAC, T.CAL_MAX_X, T.CAL_L1_X) == (CAL_MIN_FRAC, CAL_MAX_X, CAL_L1_X)
