"""P2: the GPU's counter-keyed RNG streams ("ctr" mode) estimate the same image as the
reference's own scheme ("ref" mode: per-thread xoroshiro streams, split_work_tasks sample split,
merge_planes order, rendering.rs:121-252), up to Monte Carlo noise.  Both modes run the same
restated render loop in the oracle, so the comparison isolates the RNG scheme."""
import numpy as np
import pytest

from oracle import pyoracle as O

import raytracinginaweekend_amd as R


@pytest.mark.parametrize("name,size,spp", [("final_scene1", (32, 18), 512), ("cornell_box", (20, 20), 256)])
def test_ctr_and_ref_modes_agree_statistically(worlds, name, size, spp):
    w = worlds(name)
    p1 = R.render_params(R.Size2i(*size), spp, 50, seed=1)
    p2 = R.render_params(R.Size2i(*size), spp, 50, seed=2)
    ctr1 = O.render(w, p1, O.RNG_CTR, 8)
    ctr2 = O.render(w, p2, O.RNG_CTR, 8)
    ref = O.render(w, p1, O.RNG_REF, 3)  # thread_count 3: unequal sample split, merge_planes weights
    ok = np.isfinite(ctr1).all(1) & np.isfinite(ctr2).all(1) & np.isfinite(ref).all(1)
    noise = np.sqrt(np.mean((ctr1[ok] - ctr2[ok]) ** 2))  # two independent estimates of the same image
    diff = np.sqrt(np.mean((ctr1[ok] - ref[ok]) ** 2))
    assert diff < 1.5 * noise + 1e-6, (diff, noise)
    # image means: the difference must be within 4 standard errors of the per-pixel noise
    n = int(ok.sum())
    se = np.sqrt(np.mean((ctr1[ok] - ctr2[ok]) ** 2, axis=0) / n)
    m_ctr, m_ref = ctr1[ok].mean(0), ref[ok].mean(0)
    assert np.all(np.abs(m_ctr - m_ref) <= 4.0 * se + 1e-6), (m_ctr, m_ref, se)
