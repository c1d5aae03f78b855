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


def test_keyframe_iteration_order_is_libstdcxx_unordered_map():
    """Map::mKeyFrames_ is a std::unordered_map<ID, KeyFrame_>; every reference loop over keyframes
    follows its iteration order.  deftri_keyframe_order evaluates it with the same container: reverse
    insertion up to 13 keyframes (13 buckets), interleaved after the rehash to 29 (C5's 20 keyframes:
    19..13 first, then 0..12)."""
    from deftri.capi import keyframe_order
    assert keyframe_order([0, 1]) == [1, 0]
    assert keyframe_order(list(range(8))) == list(range(7, -1, -1))
    assert keyframe_order(list(range(20))) == [19, 18, 17, 16, 15, 14, 13] + list(range(13))
    # Map::clone re-inserts in the source's iteration order
    assert keyframe_order([0, 1], clones=1) == [0, 1]
    assert keyframe_order([0, 1], clones=2) == [1, 0]
    assert keyframe_order(list(range(20)), clones=1) == keyframe_order(keyframe_order(list(range(20))))


def test_reference_clone_semantics():
    """Map.clone() is Map::clone (Map.cc:30-58): the keyframes re-inserted in the source's iteration
    order, so a two-view clone iterates (0, 1) where the map iterates (1, 0) and the clone of that
    clone (the weight search's evaluation maps, g2oBundleAdjustment.cc:499 + nloptOptimization.cc:13)
    iterates (1, 0) again; and no global-transformation table (mGTransformation_ is not copied)."""
    m, _ = sim.simulate_two_view(n=500, seed=3, scale_scene=True, compact=True)
    m.insert_global_T(0, 1, mapmodel.SE3f(t=np.array([0.1, 0.2, 0.3], np.float32)))
    c1 = m.clone()
    c2 = c1.clone()
    assert m.kf_order() == [1, 0] and c1.kf_order() == [0, 1] and c2.kf_order() == [1, 0]
    assert len(m.global_T) == 2 and c1.global_T == {} and c2.global_T == {}
    mc, _ = c2.to_c()
    assert mc.n_global == 0 and list(mc.global_t) == [0, 0, 0, 1, 0, 0, 0]
    for kid in m.keyframes:
        for a, b in zip(m.keyframes[kid].map_points, c2.keyframes[kid].map_points):
            assert (a is None) == (b is None)
            if a is not None:
                assert a is not b and np.array_equal(a.position, b.position)
