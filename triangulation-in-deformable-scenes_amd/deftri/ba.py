"""Bundle adjustment: the reference's BA entry points over the device solver.

  bundleAdjustment(pMap)                  g2oBundleAdjustment.cc:38-138
  localBundleAdjustment(pMap, kfId)       g2oBundleAdjustment.cc:245-444
  poseOnlyOptimization(frame)             g2oBundleAdjustment.cc:140-243

Each builds the same g2o graph as the reference (pose vertices in KeyFrame iteration order, KF 0
fixed, map points marginalized, EdgeSE3ProjectXYZ with info = invSigma2(octave) * I2 and Huber
(float)sqrt(5.99)), hands it to the device (`capi.BAContext`: deftri_ba_*), and replays the
reference's control flow around `optimize()` (outlier levels, robust-kernel removal, write-back in
fp32).  `BAProblem` is the flat graph; `BAProblem.shard` splits it by points for the multi-GPU
path (every rank keeps every pose).
"""
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from .mapmodel import KeyFrame, Map, MapPoint, SE3f, quat_from_mat
from .sim import DRUNKARD_KB8, generate_points, inv_sigma2_table, kb8_project, look_at

TH_HUBER_2D = float(np.float32(np.sqrt(5.99)))     # const float thHuber2D = sqrt(5.99)
CHI2_OUTLIER = 5.991


@dataclass
class BAProblem:
    poses: np.ndarray                 # [K,7] T_cw qx qy qz qw tx ty tz
    pose_kb8: np.ndarray              # [K,8] f32
    points: np.ndarray                # [P,3]
    edge_point: np.ndarray            # [E] i32
    edge_pose: np.ndarray             # [E] i32
    edge_obs: np.ndarray              # [E,2]
    edge_info: np.ndarray             # [E]
    pose_fixed: np.ndarray = None     # [K] u8
    point_fixed: np.ndarray = None    # [P] u8
    edge_level: np.ndarray = None     # [E] u8
    edge_robust: np.ndarray = None    # [E] u8
    huber_delta: float = TH_HUBER_2D
    _keep: list = field(default_factory=list, repr=False)

    def __post_init__(self):
        f64 = lambda a: np.ascontiguousarray(a, np.float64)
        i32 = lambda a: np.ascontiguousarray(a, np.int32)
        u8 = lambda a: None if a is None else np.ascontiguousarray(a, np.uint8)
        self.poses = f64(self.poses).reshape(-1, 7)
        self.pose_kb8 = np.ascontiguousarray(self.pose_kb8, np.float32).reshape(-1, 8)
        self.points = f64(self.points).reshape(-1, 3)
        self.edge_point, self.edge_pose = i32(self.edge_point), i32(self.edge_pose)
        self.edge_obs = f64(self.edge_obs).reshape(-1, 2)
        self.edge_info = f64(self.edge_info)
        self.pose_fixed = u8(self.pose_fixed) if self.pose_fixed is not None else np.zeros(self.n_poses, np.uint8)
        self.point_fixed = u8(self.point_fixed)
        self.edge_level = u8(self.edge_level) if self.edge_level is not None else np.zeros(self.n_edges, np.uint8)
        self.edge_robust = u8(self.edge_robust) if self.edge_robust is not None else np.ones(self.n_edges, np.uint8)

    @property
    def n_poses(self): return int(self.poses.shape[0])

    @property
    def n_points(self): return int(self.points.shape[0])

    @property
    def n_edges(self): return int(self.edge_point.shape[0])

    def to_desc(self):
        d = _abi.BADesc()
        d.n_poses, d.n_points, d.n_edges = self.n_poses, self.n_points, self.n_edges
        P, u8 = _abi.ptr, _abi.C.c_uint8
        d.poses, d.pose_fixed, d.pose_kb8 = P(self.poses, _abi.f64), P(self.pose_fixed, u8), P(self.pose_kb8, _abi.f32)
        d.points, d.point_fixed = P(self.points, _abi.f64), P(self.point_fixed, u8)
        d.edge_point, d.edge_pose = P(self.edge_point, _abi.i32), P(self.edge_pose, _abi.i32)
        d.edge_obs, d.edge_info = P(self.edge_obs, _abi.f64), P(self.edge_info, _abi.f64)
        d.edge_level, d.edge_robust = P(self.edge_level, u8), P(self.edge_robust, u8)
        d.huber_delta = self.huber_delta
        return d

    def shard(self, rank, nranks):
        """Point shard `rank` of `nranks` (contiguous point ranges): every pose, the shard's points
        and the edges on them.  Returns (sub-problem, point index range, edge indices)."""
        lo = (self.n_points * rank) // nranks
        hi = (self.n_points * (rank + 1)) // nranks
        sel = np.nonzero((self.edge_point >= lo) & (self.edge_point < hi))[0]
        sub = BAProblem(self.poses, self.pose_kb8, self.points[lo:hi], self.edge_point[sel] - lo, self.edge_pose[sel],
                        self.edge_obs[sel], self.edge_info[sel], pose_fixed=self.pose_fixed,
                        point_fixed=None if self.point_fixed is None else self.point_fixed[lo:hi],
                        edge_level=self.edge_level[sel], edge_robust=self.edge_robust[sel],
                        huber_delta=self.huber_delta)
        return sub, (lo, hi), sel


# ------------------------------------------------------------------------------------------
# synthetic scenes
# ------------------------------------------------------------------------------------------
def _small_rotation(rng, sigma):
    w = rng.normal(0, sigma, 3)
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def simulate_ba_map(n=500, k=4, seed=0, kb8=DRUNKARD_KB8, radius=0.12, rep_error=1.0, decimals=1,
                    noise3d=0.002, pose_rot=0.01, pose_t=0.003, visibility=1.0, outliers=0.0, n_octaves=8,
                    min_common_obs=15):
    """Rigid BA scene: K keyframes on an arc around one cloud (the reference's simulated cloud,
    create_data.py recipe), each slot i of a keyframe observing MapPoint i when visible.  Keypoints
    = KB8 projection + N(0, rep_error) px rounded to `decimals` (SLAM.cc:281-319) at a random
    octave; a fraction `outliers` of observations is displaced by 20-40 px.  Initial MapPoints =
    truth + N(0, noise3d); initial poses of KFs > 0 are perturbed (KF 0 is the fixed gauge)."""
    rng = np.random.default_rng(seed + 11)
    base, _ = generate_points(n, rigid=0.0, gaussian=0.0, seed=seed)
    inv_s2 = inv_sigma2_table(n_octaves, 1.2)
    m = Map(min_common_obs=min_common_obs)
    center = base.mean(0)
    init = (base + rng.normal(0, noise3d, base.shape)).astype(np.float32)
    mps = [MapPoint(init[i], i) for i in range(n)]
    for mp in mps:
        m.insert_map_point(mp)
    truth = {}
    for kk in range(k):
        ang = np.deg2rad(-30 + 60 * kk / max(k - 1, 1))
        cpos = center + np.array([radius * np.sin(ang), 0.0, -radius * np.cos(ang)])
        R = look_at(cpos, center)
        Tcw = SE3f(R.T, -(R.T @ cpos.astype(np.float32)))
        truth[kk] = Tcw
        pc = Tcw * base.astype(np.float32)
        uv = kb8_project(kb8, pc).astype(np.float64)
        octv = rng.integers(0, n_octaves, n).astype(np.int32)
        uv = uv + rng.normal(0, rep_error, uv.shape)
        if outliers > 0:
            bad = rng.random(n) < outliers
            uv[bad] += rng.choice([-1, 1], (bad.sum(), 2)) * rng.uniform(20, 40, (bad.sum(), 2))
        uv = (np.round(uv * 10 ** decimals) / 10 ** decimals).astype(np.float32)
        if kk == 0:
            T0 = Tcw
        else:
            dR = _small_rotation(rng, pose_rot).astype(np.float32)
            T0 = SE3f(dR @ Tcw.R, Tcw.t + rng.normal(0, pose_t, 3).astype(np.float32))
        kf = KeyFrame(kk, T0, kb8, n, inv_s2, uv, octv, pc[:, 2].copy())
        m.insert_keyframe(kf)
        vis = rng.random(n) < visibility if kk > 0 else np.ones(n, bool)
        for i in range(n):
            if vis[i] and pc[i, 2] > 0:
                kf.map_points[i] = mps[i]
                m.add_observation(kk, i, i)
    return m, {"points": base, "poses": truth}


def make_ba_problem(n=50000, k=8, seed=0, kb8=DRUNKARD_KB8, radius=0.12, rep_error=1.0, noise3d=0.002,
                    pose_rot=0.01, pose_t=0.003, visibility=1.0, outliers=0.01):
    """Flat BAProblem of the same scene family at bench sizes (vectorised; no Map objects).
    Point order is the Morton order of the cloud's (x, y) so contiguous point shards are compact."""
    rng = np.random.default_rng(seed + 13)
    base, _ = generate_points(n, rigid=0.0, gaussian=0.0, seed=seed)
    xy = base[:, :2]
    q = ((xy - xy.min(0)) / (np.ptp(xy, 0) + 1e-12) * 65535).astype(np.uint32)

    def spread(v):
        v = v.astype(np.uint64)
        v = (v | (v << 8)) & 0x00FF00FF
        v = (v | (v << 4)) & 0x0F0F0F0F
        v = (v | (v << 2)) & 0x33333333
        v = (v | (v << 1)) & 0x55555555
        return v
    order = np.argsort(spread(q[:, 0]) | (spread(q[:, 1]) << np.uint64(1)), kind="stable")
    base = base[order]
    center = base.mean(0)
    inv_s2 = inv_sigma2_table(8, 1.2)
    poses, kbs, ep, eo, obs, info = [], [], [], [], [], []
    for kk in range(k):
        ang = np.deg2rad(-30 + 60 * kk / max(k - 1, 1))
        cpos = center + np.array([radius * np.sin(ang), 0.0, -radius * np.cos(ang)])
        R = look_at(cpos, center)
        Tcw = SE3f(R.T, -(R.T @ cpos.astype(np.float32)))
        pc = Tcw * base.astype(np.float32)
        uv = kb8_project(kb8, pc).astype(np.float64) + rng.normal(0, rep_error, (n, 2))
        if outliers > 0:
            bad = rng.random(n) < outliers
            uv[bad] += rng.uniform(20, 40, (bad.sum(), 2))
        uv = np.round(uv * 10) / 10
        vis = (rng.random(n) < visibility) | (kk == 0)
        vis &= pc[:, 2] > 0
        idx = np.nonzero(vis)[0]
        ep.append(idx.astype(np.int32)); eo.append(np.full(len(idx), kk, np.int32))
        obs.append(uv[idx])
        info.append(inv_s2[rng.integers(0, 8, len(idx))].astype(np.float64))
        T0 = Tcw if kk == 0 else SE3f(_small_rotation(rng, pose_rot).astype(np.float32) @ Tcw.R,
                                      Tcw.t + rng.normal(0, pose_t, 3).astype(np.float32))
        poses.append(T0.as7()); kbs.append(kb8)
    # edges grouped by point (the reference adds them KF by KF; the device sorts by point anyway)
    ep = np.concatenate(ep); eo = np.concatenate(eo); obs = np.concatenate(obs); info = np.concatenate(info)
    srt = np.lexsort((eo, ep))
    pts0 = base + rng.normal(0, noise3d, base.shape)
    fixed = np.zeros(k, np.uint8); fixed[0] = 1
    return BAProblem(np.array(poses), np.array(kbs), pts0, ep[srt], eo[srt], obs[srt], info[srt], pose_fixed=fixed)


# ------------------------------------------------------------------------------------------
# graph construction from the map (reference graph-building loops)
# ------------------------------------------------------------------------------------------
def _edge_of(kf, slot):
    uv = kf.keypoints[slot]                                   # pKF->getKeyPoint(mpIndex).pt
    octave = int(kf.octaves[slot])
    return [float(uv[0]), float(uv[1])], float(kf.inv_sigma2[octave])   # getInvSigma2(octave)


def build_ba_graph(kfs_free, kfs_fixed=(), local_mps=None):
    """Vertices/edges as g2oBundleAdjustment.cc:58-117 (kfs_fixed empty) or :276-387 (local BA):
    poses in the given KF order (KF id 0 fixed), then fixed KFs whose edges only reach local points;
    points in order of first appearance.  Returns (BAProblem, meta)."""
    poses, kbs, fixed = [], [], []
    pt_index, pts, pt_objs = {}, [], []
    ep, eo, obs, info, edge_kf, edge_slot, edge_mp = [], [], [], [], [], [], []
    for is_fixed_set, kfs in ((False, kfs_free), (True, kfs_fixed)):
        for kf in kfs:
            kidx = len(poses)
            poses.append(kf.pose.as7()); kbs.append(kf.kb8)
            fixed.append(1 if (is_fixed_set or kf.id == 0) else 0)
            for slot, mp in enumerate(kf.map_points):
                if mp is None:
                    continue
                if is_fixed_set and (local_mps is None or mp.id not in local_mps):
                    continue
                if mp.id not in pt_index:
                    if is_fixed_set:
                        raise AssertionError("fixed KF observes a local point missing from the graph")
                    pt_index[mp.id] = len(pts)
                    pts.append(mp.position.astype(np.float64)); pt_objs.append(mp)
                uv, inf = _edge_of(kf, slot)
                ep.append(pt_index[mp.id]); eo.append(kidx); obs.append(uv); info.append(inf)
                edge_kf.append(kf.id); edge_slot.append(slot); edge_mp.append(mp.id)
    prob = BAProblem(np.array(poses).reshape(-1, 7), np.array(kbs).reshape(-1, 8), np.array(pts).reshape(-1, 3),
                     np.array(ep, np.int32), np.array(eo, np.int32), np.array(obs).reshape(-1, 2),
                     np.array(info), pose_fixed=np.array(fixed, np.uint8))
    meta = {"kfs": list(kfs_free) + list(kfs_fixed), "n_free_kfs": len(kfs_free), "points": pt_objs,
            "edge_kf": edge_kf, "edge_slot": edge_slot, "edge_mp": edge_mp}
    return prob, meta


def _writeback(meta, poses, pts, n_kfs=None):
    """Pose: SE3f(estimate().to_homogeneous_matrix().cast<float>()); point: estimate().cast<float>()."""
    n = meta["n_free_kfs"] if n_kfs is None else n_kfs
    for i, kf in enumerate(meta["kfs"][:n]):
        kf.pose = SE3f.from7(poses[i])
    for i, mp in enumerate(meta["points"]):
        mp.position = pts[i].astype(np.float32)


_ctx_cache = {}


def _ctx(device):
    from . import capi
    c = _ctx_cache.get(device)
    if c is None:
        c = capi.BAContext(device)
        _ctx_cache[device] = c
    return c


def bundleAdjustment(pMap, device=0, report=None, ctx=None):
    """g2oBundleAdjustment.cc:38-138: every KF (map iteration order), KF 0 fixed, optimize(20).
    `ctx` (tests only) replaces the device context with another object of the same interface."""
    kfs = [pMap.keyframes[k] for k in pMap.kf_order()]
    prob, meta = build_ba_graph(kfs)
    ctx = ctx or _ctx(device)
    ctx.upload(prob)
    rep = ctx.solve_lm(20)
    poses, pts = ctx.download()
    _writeback(meta, poses, pts)
    if isinstance(report, dict):
        report.update(rep)
    return rep


def localBundleAdjustment(pMap, currKeyFrameId, device=0, report=None, ctx=None):
    """g2oBundleAdjustment.cc:245-444: local KFs + fixed covisible KFs; optimize(5) with Huber,
    outliers (chi2 > 5.991 or depth <= 0) to level 1, robust kernels removed, optimize(10), outlier
    observations removed from the map, poses of local KFs and local points written back."""
    local_mps, local_kfs, fixed_kfs = pMap.get_local_map_of_keyframe(currKeyFrameId)
    lm = set(local_mps)
    for kid in local_kfs:
        for mp in pMap.keyframes[kid].map_points:
            if mp is not None:
                assert mp.id in lm        # assert(sLocalMapPoints.count(pMP->getId()) != 0)
    prob, meta = build_ba_graph([pMap.keyframes[k] for k in local_kfs], [pMap.keyframes[k] for k in fixed_kfs], lm)
    ctx = ctx or _ctx(device)
    ctx.upload(prob)
    r1 = ctx.solve_lm(5)
    chi, dpos = ctx.edge_chi2()
    level = np.where((chi > CHI2_OUTLIER) | ~dpos, 1, 0).astype(np.uint8)
    ctx.set_edge_flags(level=level, robust=np.zeros(prob.n_edges, np.uint8))
    r2 = ctx.solve_lm(10, level=0)
    chi, dpos = ctx.edge_chi2()
    bad = (chi > CHI2_OUTLIER) | ~dpos
    for e in np.nonzero(bad)[0]:
        kid, slot, mpid = meta["edge_kf"][e], meta["edge_slot"][e], meta["edge_mp"][e]
        pMap.keyframes[kid].map_points[slot] = None          # setMapPoint(idx, nullptr)
        pMap.remove_observation(kid, mpid)                     # removeObservation; checkKeyFrame is a no-op
    poses, pts = ctx.download()
    _writeback(meta, poses, pts)
    rep = {"first": r1, "second": r2, "outliers_removed": int(bad.sum())}
    if isinstance(report, dict):
        report.update(rep)
    return rep


def poseOnlyOptimization(currFrame, device=0, report=None, ctx=None):
    """g2oBundleAdjustment.cc:140-243: one pose vertex, EdgeSE3ProjectXYZOnlyPose per map point
    (Xworld fixed), 4 rounds of {reset the pose estimate, initializeOptimization(0), optimize(10),
    classify edges by chi2 > 5.991}, robust kernels dropped after round 2.  Keeps the reference's
    index quirk: the computeError() guard tests vInlier[round] instead of vInlier[j]
    (:196-197).  Outlier slots are set to null; returns the inlier count."""
    slots = [i for i, mp in enumerate(currFrame.map_points) if mp is not None]
    n_slots = currFrame.n_slots
    pts = np.array([currFrame.map_points[i].position.astype(np.float64) for i in slots]).reshape(-1, 3)
    obs, info = zip(*[_edge_of(currFrame, i) for i in slots]) if slots else ([], [])
    pose0 = currFrame.pose.as7()
    E = len(slots)
    prob = BAProblem(pose0[None], currFrame.kb8[None], pts, np.arange(E, dtype=np.int32), np.zeros(E, np.int32),
                     np.array(obs).reshape(-1, 2), np.array(info), point_fixed=np.ones(len(slots), np.uint8))
    ctx = ctx or _ctx(device)
    ctx.upload(prob)
    v_inlier = np.zeros(n_slots, bool)
    v_inlier[slots] = True
    level = np.zeros(E, np.uint8)
    robust = np.ones(E, np.uint8)
    edge_of_slot = {s: e for e, s in enumerate(slots)}
    reps = []
    for rnd in range(4):
        ctx.set_state(poses=pose0[None])
        ctx.set_edge_flags(level=level, robust=robust)
        reps.append(ctx.solve_lm(10, level=0))
        # guard for j <= rnd uses vInlier[rnd] before edge rnd is classified, j > rnd after
        c_old = not v_inlier[rnd] if rnd < n_slots else False
        mask_lo = np.array([s <= rnd for s in slots], bool)
        if c_old and mask_lo.any():
            ctx.compute_errors(mask_lo)
        chi, _ = ctx.edge_chi2()
        if rnd in edge_of_slot:
            inl_r = not (chi[edge_of_slot[rnd]] > CHI2_OUTLIER)
        else:
            inl_r = bool(v_inlier[rnd]) if rnd < n_slots else False
        c_new = not inl_r
        mask_hi = ~mask_lo
        if c_new and mask_hi.any():
            ctx.compute_errors(mask_hi)
            chi, _ = ctx.edge_chi2()
        for e, s in enumerate(slots):
            if chi[e] > CHI2_OUTLIER:
                v_inlier[s] = False
                level[e] = 1
            else:
                v_inlier[s] = True
                level[e] = 0
            if rnd == 2:
                robust[e] = 0
    n_good = 0
    for i in range(n_slots):
        if not v_inlier[i]:
            currFrame.map_points[i] = None
        else:
            n_good += 1
    poses, _ = ctx.download()
    currFrame.pose = SE3f.from7(poses[0])
    if isinstance(report, dict):
        report.update({"rounds": reps, "n_good": n_good})
    return n_good
