"""Graph construction parity: the product's C++ builder (csrc/graph_builder.cpp, reached through
deftri_arap_build_graph) against the oracle restatement (oracle/graph_ref.py, scipy qhull) of the
reference's arapOptimization graph build (g2oBundleAdjustment.cc:640-953).
Index arrays must be bit-exact; floats within rounding (summation order differs)."""
import json

import numpy as np
import pytest
from scipy.spatial import ConvexHull, Delaunay

from conftest import GOLDEN
from deftri import capi, sim
from deftri.problem import Problem
from oracle import graph_ref

INT_FIELDS = ["rep_point", "rep_cam", "dep_point", "dep_scale", "dep_cam", "arap_pts", "arap_pair", "arap_rot"]
F_FIELDS = ["points", "scales", "tg", "rep_obs", "rep_info", "dep_meas", "dep_info", "arap_w", "rot", "pair_area",
            "pair_info", "cam_pose"]


def compare(pr, pc, rtol=1e-12):
    for k in INT_FIELDS:
        a, b = getattr(pr, k), getattr(pc, k)
        assert a.shape == b.shape, k
        assert np.array_equal(a, b), k
    for k in F_FIELDS:
        a, b = getattr(pr, k), getattr(pc, k)
        assert a.shape == b.shape, k
        if a.size:
            assert np.abs(a - b).max() <= rtol * max(1.0, np.abs(a).max()), k
    assert np.array_equal(pr.cam_kb8, pc.cam_kb8)
    assert pr.huber_delta == pc.huber_delta


@pytest.fixture(scope="module")
def host():
    return capi.Context(-1)


def test_golden_graphs_reproduced(host, golden_cases):
    import importlib, sys
    sys.path.insert(0, str(GOLDEN))
    mg = importlib.import_module("make_golden")
    for name in golden_cases:
        m, st, sigma = mg.scene(name)
        pg = Problem.load(GOLDEN / name / "problem.npz")
        pc = host.build_graph(m, st.rep, st.arap, sigma)
        compare(pg, pc)
        kw, info = graph_ref.build_arap_graph(m, st.rep, st.arap, sigma)
        compare(Problem(**kw), pg, rtol=0)                  # oracle is deterministic


@pytest.mark.parametrize("n,seed", [(300, 3), (1500, 4)])
def test_builder_matches_oracle_sim(host, n, seed):
    m, _ = sim.simulate_two_view(n=n, seed=seed)
    kw, info = graph_ref.build_arap_graph(m, 1.0, 2e5, np.float32(0.003))
    compare(Problem(**kw), host.build_graph(m, 1.0, 2e5, np.float32(0.003)))


def test_null_slot_quirk(host):
    """Null slots: the reference uses the KF slot index as a position index and the position
    index as a slot index.  Both builders must reproduce that."""
    m, _ = sim.simulate_two_view(n=200, seed=5)
    kf0, kf1 = m.keyframes[0], m.keyframes[1]
    for s in (3, 40, 41, 150):                  # drop correspondences -> null slots in both KFs
        for kf in (kf0, kf1):
            mp = kf.map_points[s]
            kf.map_points[s] = None
            m.kf_obs[kf.id].pop(mp.id, None)
    kw, info = graph_ref.build_arap_graph(m, 1.0, 2e5, np.float32(0.003))
    pr = Problem(**kw)
    compare(pr, host.build_graph(m, 1.0, 2e5, np.float32(0.003)))
    # the quirk really changes the graph: some ARAP edges join non-adjacent slots
    assert len(pr.arap_pair) > 0


def test_triangle_count_is_qhull_facet_count():
    rng = np.random.default_rng(9)
    for n in (10, 120, 1000):
        xy = rng.normal(size=(n, 2))
        lifted = np.c_[xy, (xy * xy).sum(1)]
        T = len(ConvexHull(lifted).simplices)
        assert T == 2 * n - 4
        lower = len(Delaunay(xy).simplices)
        h = len(ConvexHull(xy).vertices)
        assert lower == 2 * n - 2 - h


def test_eigen_jacobi_svd_restatement():
    rng = np.random.default_rng(10)
    for _ in range(50):
        S = rng.normal(size=(3, 3)) * 10.0 ** rng.uniform(-6, 2)
        U, s, V = graph_ref.eigen_jacobi_svd3(S)
        assert np.allclose(U @ np.diag(s) @ V.T, S, atol=1e-12 * np.abs(S).max())
        assert np.allclose(s, np.linalg.svd(S)[1], rtol=1e-10)
        assert np.allclose(U.T @ U, np.eye(3), atol=1e-12)
        R = graph_ref.procrustes(S)
        assert np.isclose(np.linalg.det(R), 1.0) and np.allclose(R.T @ R, np.eye(3), atol=1e-12)


def test_problem_roundtrip(tmp_path, golden_cases):
    p = Problem.load(GOLDEN / golden_cases[0] / "problem.npz")
    p.save(tmp_path / "p.npz")
    q = Problem.load(tmp_path / "p.npz")
    compare(p, q, rtol=0)


def test_graph_errors(host):
    m, _ = sim.simulate_two_view(n=2, seed=1)
    with pytest.raises(capi.DeftriError) as e:
        host.build_graph(m, 1.0, 2e5, np.float32(0.003))
    assert e.value.code == -6


def test_global_transform_lookup_per_pair(host):
    """Every KF pair starts from getGlobalKeyFramesTransformation(kf1.id, kf2.id)
    (g2oBundleAdjustment.cc:664, Map.cc:332-343): T for the stored (0, 1) entry, its fp32 inverse for
    (1, 0), identity otherwise.  With 3 KFs in reverse-insertion order the pair holding the stored T
    is the last one, so a first-pair-only lookup would start it from identity."""
    from deftri.mapmodel import SE3f, mat_from_quat
    m, _ = sim.simulate_multi_view(n=150, k=3, seed=6)
    q = np.array([0.02, -0.01, 0.03, 1.0]); q /= np.linalg.norm(q)
    m.insert_global_T(0, 1, SE3f(mat_from_quat(q).astype(np.float32), np.array([0.004, -0.002, 0.001], np.float32)))
    for _round in range(2):          # second round: the map carries the written-back T
        kw, info = graph_ref.build_arap_graph(m, 1.0, 2e5, np.float32(0.003))
        pr = Problem(**kw)
        pc = host.build_graph(m, 1.0, 2e5, np.float32(0.003))
        compare(pr, pc)
        ident = np.array([0, 0, 0, 1, 0, 0, 0], float)
        non_identity = [not np.allclose(t, ident) for t in pc.tg.reshape(-1, 7)]
        assert sum(non_identity) == 1, non_identity        # only the pair (KF 1, KF 0) has a stored T
        t_new = pc.tg.reshape(-1, 7)[int(np.argmax(non_identity))] * np.r_[1, 1, 1, 1, 1.5, 1.5, 1.5]
        m.insert_global_T(0, 1, SE3f.from7(t_new))


def _equal_problems(a, b):
    for k in INT_FIELDS + F_FIELDS + ["cam_kb8", "order_xy", "point_ids"]:
        x, y = getattr(a, k), getattr(b, k)
        assert np.array_equal(x, y), k


def test_graph_memo_same_map_other_weights():
    """A repeated call on an unchanged map (NLopt's clones, nloptOptimization.cc:4-37) is answered
    from the graph memo; only the weights' entries are recomputed — bit-identical to a fresh build."""
    import copy
    m, _ = sim.simulate_two_view(n=1200, seed=11)
    with capi.Context(-1) as c:
        c.build_graph(m, 1.0, 2e5, np.float32(0.003))
        for w in ((2.0, 3e4, np.float32(0.01)), (1.0, 2e5, np.float32(0.003))):
            got = c.build_graph(copy.deepcopy(m), *w)
            with capi.Context(-1) as f:
                _equal_problems(got, f.build_graph(m, *w))


def test_graph_memo_miss_on_moved_point():
    """Any input change (here one MapPoint moved, as after a write-back) rebuilds the graph."""
    m, _ = sim.simulate_two_view(n=1200, seed=12)
    with capi.Context(-1) as c:
        p0 = c.build_graph(m, 1.0, 2e5, np.float32(0.003))
        mc, keep = m.to_c()
        kf = mc.keyframes[0]
        s = next(i for i in range(kf.n_slots) if kf.point_id[i] >= 0)
        kf.point_pos[3 * s] += 1e-3
        m.from_c(mc, keep)
        p1 = c.build_graph(m, 1.0, 2e5, np.float32(0.003))
        with capi.Context(-1) as f:
            _equal_problems(p1, f.build_graph(m, 1.0, 2e5, np.float32(0.003)))
        assert not np.array_equal(p0.points, p1.points)


FIELDS_ALL = ("points", "tg", "scales", "cam_kb8", "cam_pose", "rep_point", "rep_cam", "rep_obs", "rep_info",
              "dep_point", "dep_scale", "dep_cam", "dep_meas", "dep_info", "arap_pts", "arap_pair", "arap_rot",
              "arap_w", "rot", "pair_area", "pair_info", "order_xy", "point_ids")


def _same(pa, pb, skip=()):
    for f in FIELDS_ALL:
        if f in skip:
            continue
        a, b = getattr(pa, f), getattr(pb, f)
        assert a.shape == b.shape and np.array_equal(a, b), f


@pytest.mark.parametrize("n,seed,k", [(3000, 5, 2), (800, 6, 4)])
def test_next_round_fast_path_is_a_full_build(n, seed, k):
    """deformationOptimization's next round (g2oBundleAdjustment.cc:482): the written-back map has
    moved points, depth scales and T_g but the same structure.  When every pair's previous Delaunay
    triangulation is still THE Delaunay triangulation of the moved points, the structure memo
    refreshes the values in place — the descriptor must equal a fresh context's full build bit for
    bit (except the ordering hint order_xy, kept from the structure's first build so the device plan
    is reused); when the motion flips an edge it must fall back to the full build (then all equal)."""
    import copy
    from deftri import metrics
    if k == 2:
        m, _ = sim.simulate_two_view(n=n, seed=seed, scale_scene=True, compact=True)
    else:
        m = sim.multi_view_arrays(n=n, k=k, seed=seed)
    rng = np.random.default_rng(seed)
    with capi.Context(-1) as a:
        p0 = a.build_graph(m, 1.0, 2e5, np.float32(0.003))
        order0 = p0.order_xy
        ext = np.abs(p0.points).max()
        for step, (scale, expect_fast) in enumerate([(1e-9, True), (3e-9, True), (3e-2, False)]):
            m2 = copy.deepcopy(m)
            pts = p0.points + rng.normal(0.0, scale * ext, p0.points.shape)
            if k == 2:
                metrics.apply_solution(m2, list(p0.point_ids), pts)
                for kf in m2.keyframes.values():
                    kf.estimated_depth_scale = 1.0 + 1e-6 * (step + 1)
            else:                           # ArrayMap: MapPoint id = keyframe id * n + slot
                for pid, x in zip(p0.point_ids, pts):
                    kf = m2.kfs[int(pid) // n]
                    kf["pos"][int(pid) % n] = np.asarray(x, np.float32)
            before = a.graph_stats()[1]
            pa = a.build_graph(m2, 1.5, 1e5, np.float32(0.004))
            fast = a.graph_stats()[1] > before
            with capi.Context(-1) as b:
                pb = b.build_graph(m2, 1.5, 1e5, np.float32(0.004))
            if expect_fast:
                # order_xy (the plan's ordering hint) stays that of the structure's first build
                assert fast, (step, scale)
                _same(pa, pb, skip=("order_xy",))
                assert np.array_equal(pa.order_xy, order0)
            else:
                assert not fast, (step, scale)
                _same(pa, pb)
                order0 = pa.order_xy
            m = m2
            p0 = pa


@pytest.mark.parametrize("case", ["octave_first", "obs_only"])
def test_graph_observation_errors_first_pair_wins(host, case):
    """A bad observation index or keypoint octave fails the build (the reference would read out of
    bounds): the pairs' slot scans run in parallel, and the error reported is the one the sequential
    walk meets first — the earliest pair's first bad slot."""
    m = sim.multi_view_arrays(n=200, k=4, seed=2)

    class Corrupted:
        def to_c(self):
            mc, keep = m.to_c()
            last = mc.keyframes[mc.n_keyframes - 1]     # only in pairs (a, K-1): after pair (0, 1)
            last.obs_index[3] = last.n_obs + 3
            if case == "octave_first":
                first = mc.keyframes[0]                  # in pair (0, 1), the first pair
                first.kp_octave[first.obs_index[7]] = 99
            return mc, keep

    with pytest.raises(capi.DeftriError) as e:
        host.build_graph(Corrupted(), 1.0, 1e7, np.float32(0.3))
    want = "keypoint octave out of range" if case == "octave_first" else "observation index out of range"
    assert want in str(e.value)
    host.build_graph(m, 1.0, 1e7, np.float32(0.3))      # the context builds a good map afterwards


@pytest.mark.parametrize("rel", [1e-6, 1e-5])
def test_next_round_mesh_repair_equals_new_triangulation(rel, monkeypatch):
    """A full build after the points moved (the structure memo's triangulations no longer Delaunay):
    the keyframe's previous triangulation is repaired by Lawson flips (delaunay.cpp delaunay_repair,
    exact predicates, accepted only when the strict uniqueness check passes) — the descriptor must equal
    a fresh context's build (a new triangulation) field for field."""
    import copy
    from deftri import metrics
    monkeypatch.setenv("DEFTRI_DELAUNAY_REPAIR", "1")          # (opt-in: graph_builder.cpp build_mesh)
    m, _ = sim.simulate_two_view(n=3000, seed=5, scale_scene=True, compact=True)
    rng = np.random.default_rng(11)
    with capi.Context(-1) as a:
        p0 = a.build_graph(m, 1.0, 2e5, np.float32(0.003))
        ext = np.abs(p0.points).max()
        m2 = copy.deepcopy(m)
        metrics.apply_solution(m2, list(p0.point_ids), p0.points + rng.normal(0.0, rel * ext, p0.points.shape))
        r0 = a.graph_repairs()
        pa = a.build_graph(m2, 1.5, 1e5, np.float32(0.004))
        r1 = a.graph_repairs()
        assert r1[0] == r0[0] + 1 and r1[1] > r0[1], (r0, r1)      # repaired, with flips
        monkeypatch.delenv("DEFTRI_DELAUNAY_REPAIR")              # the fresh build: a new triangulation
        with capi.Context(-1) as b:
            _same(pa, b.build_graph(m2, 1.5, 1e5, np.float32(0.004)))
