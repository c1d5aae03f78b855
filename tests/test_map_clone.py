"""Map::clone (deftri/mapmodel.py Map.__deepcopy__): the weight search clones the map for every
objective evaluation (nloptOptimization.cc: pData->pMap->clone()).  The direct clone must equal the
generic object-walking copy.deepcopy — same keyframe order, slots, observation / covisibility tables,
positions, scales and global transformations — and be independent of the original."""
import copy

import numpy as np

from deftri import mapmodel, sim


def _generic_deepcopy(m):
    saved = mapmodel.Map.__deepcopy__
    try:
        del mapmodel.Map.__deepcopy__
        return copy.deepcopy(m)
    finally:
        mapmodel.Map.__deepcopy__ = saved


def test_map_clone_equals_generic_deepcopy_and_is_independent():
    m, _ = sim.simulate_two_view(n=2000, seed=3, scale_scene=True, compact=True)
    m.insert_global_T(0, 1, mapmodel.SE3f(t=np.array([0.1, 0.2, 0.3], np.float32)))
    fast, ref = copy.deepcopy(m), _generic_deepcopy(m)
    assert list(fast.keyframes) == list(ref.keyframes) and list(fast.map_points) == list(ref.map_points)
    assert fast.kf_obs == ref.kf_obs and fast.mp_obs == ref.mp_obs and fast.covis == ref.covis
    assert fast.min_common_obs == ref.min_common_obs
    for k in ref.global_T:
        assert np.array_equal(fast.global_T[k].as7(), ref.global_T[k].as7())
    _, ka = fast.to_c()
    _, kb = ref.to_c()
    for x, y in zip(ka["arrays"], kb["arrays"]):
        for u, v in zip(x[1:], y[1:]):
            assert np.array_equal(u, v)
    for kid, kf in fast.keyframes.items():           # slots point at the clone's own MapPoints
        for mp in kf.map_points:
            if mp is not None:
                assert fast.map_points[mp.id] is mp and m.map_points[mp.id] is not mp
        assert kf.keypoints is not m.keyframes[kid].keypoints
    pid = next(iter(fast.map_points))
    before = m.map_points[pid].position.copy()
    fast.map_points[pid].position[0] += 1.0
    fast.keyframes[next(iter(fast.keyframes))].estimated_depth_scale = 7.0
    fast.kf_obs[next(iter(fast.kf_obs))].clear()
    assert np.array_equal(m.map_points[pid].position, before)
    assert m.keyframes[next(iter(m.keyframes))].estimated_depth_scale != 7.0
    assert all(len(v) > 0 for v in m.kf_obs.values())
