"""computeR on the device (csrc/graph_dev.hip: one thread per mesh vertex, the Jacobi SVD restated in
csrc/procrustes.h) against the host loop: a context with a device builds the graph with the kernel,
a host-only context with the host loop, and every descriptor array must be bit-identical (both
sides one rounding per operation: no FMA contraction, IEEE fp64 division and square root)."""
import numpy as np
import pytest

from deftri import capi, sim

pytestmark = pytest.mark.gpu

FIELDS = ("points", "tg", "scales", "cam_kb8", "cam_pose", "rep_point", "rep_cam", "rep_obs", "rep_info",
          "dep_point", "dep_scale", "dep_cam", "dep_meas", "dep_info", "arap_pts", "arap_pair", "arap_rot",
          "arap_w", "rot", "pair_area", "pair_info", "order_xy", "point_ids")


def both(m, *w):
    with capi.Context(-1) as h, capi.Context(0) as d:
        return h.build_graph(m, *w), d.build_graph(m, *w)


@pytest.mark.parametrize("n,seed", [(3000, 1), (20000, 2)])
def test_device_compute_r_two_view(n, seed):
    m, _ = sim.simulate_two_view(n=n, seed=seed, scale_scene=True, compact=True)
    ph, pd = both(m, 1.0, 2e5, np.float32(0.003))
    for f in FIELDS:
        assert np.array_equal(getattr(ph, f), getattr(pd, f)), f
    assert not np.array_equal(pd.rot.reshape(-1, 9), np.tile(np.eye(3).ravel(), (pd.rot.size // 9, 1)))


def test_device_compute_r_multi_view():
    m = sim.multi_view_arrays(n=2000, k=5, seed=3)
    ph, pd = both(m, 1.0, 1e7, np.float32(0.3))
    for f in FIELDS:
        assert np.array_equal(getattr(ph, f), getattr(pd, f)), f
