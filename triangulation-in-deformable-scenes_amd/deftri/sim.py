"""Synthetic scenes following the reference's simulation path (upstream producer of the hot path).

Recipe, per reference file:
  points      Data/Scripts/synthetic/create_data.py:27-66 (N(0,sigma) cloud, rigid/gaussian
              motion, Rz(45)·Ry(0)·Rx(-45) rotation, +0.2 m in z); extents scaled by sqrt(N/120)
              to keep density
  cameras     SLAM::setCameraPoses SLAM.cc:223-235 (T1w = (I, C1), T2w = (lookAt(C2, moved[0]), C2)),
              SLAM::lookAt SLAM.cc:340-351
  depth       SLAM::getSimulatedDepthMeasurements SLAM.cc:321-338 (d = z_c * scale + N(0, err/1000))
  keypoints   SLAM::createKeyPoints SLAM.cc:281-319 (KB8 projection + N(0, RepError), rounded to
              `decimals`), octave 0
  MapPoints   Mapping::triangulateSimulatedMapPoints Mapping.cc:280-349 with
              triangulateNRSLAM(..., "FarPoints") Geometry.cc:103-153 and isValidParallax
              Mapping.cc:351-364 (fp32 math)
  sigma table Frame.cc:61-75 (nScales, scale factor)
Noise streams: the keypoint and depth noise and the camera poses come from deftri_sim_two_view
(csrc/sim_host.cpp): libstdc++'s std::default_random_engine (minstd_rand0, seed 1) and
std::normal_distribution<float>, one fresh engine per function as in SLAM.cc, Sophus-style SE3f
(fp32 unit quaternion) poses — the reference's own numbers for the reference's inputs.  The point
clouds follow create_data.py, whose np.random is unseeded; here a seeded legacy RandomState drawn in
the script's order (x, y, z columns, then x, y, z motion noise per point).

Multi-keyframe scenes (configs C3-C5) extend the same recipe: K cameras on an arc, each observing
its own deformed copy of the cloud.
"""
import numpy as np

from .mapmodel import KeyFrame, Map, MapPoint, SE3f

SIM_KB8 = np.array([458.654, 457.296, 367.215, 248.375, 0, 0, 0, 0], np.float32)   # Simulation.yaml
DRUNKARD_KB8 = np.array([190.68, 190.68, 160, 160, 0, 0, 0, 0], np.float32)       # Drunkard.yaml
REALCOLON_KB8 = np.array([727.1851, 728.5954, 738.1817, 537.4003, -0.1311029, -0.005149247,
                          0.001512357, -6.998448e-05], np.float32)                 # Realcolon.yaml


def inv_sigma2_table(n_scales=8, factor=1.2):
    sf = np.ones(n_scales, np.float32)
    for i in range(1, n_scales):
        sf[i] = np.float32(sf[i - 1] * np.float32(factor))
    sig2 = (sf * sf).astype(np.float32)
    return (np.float32(1.0) / sig2).astype(np.float32)


def rotate_points(points, ax, ay, az):
    ax, ay, az = np.deg2rad([ax, ay, az])
    Rx = np.array([[1, 0, 0], [0, np.cos(ax), -np.sin(ax)], [0, np.sin(ax), np.cos(ax)]])
    Ry = np.array([[np.cos(ay), 0, np.sin(ay)], [0, 1, 0], [-np.sin(ay), 0, np.cos(ay)]])
    Rz = np.array([[np.cos(az), -np.sin(az), 0], [np.sin(az), np.cos(az), 0], [0, 0, 1]])
    return points @ (Rz @ Ry @ Rx).T


def generate_points(n, rigid=0.0025, gaussian=0.0025, seed=0, scale_density=True,
                    stds=(0.03, 0.001, 0.01), mean=(0.0, 0.0, 0.2), angles=(-45, 0, 45)):
    """create_data.py:27-66 (Planar motion along y), its draw order with np.random seeded: the three
    coordinate columns, then per point the rigid offset and N(0, gaussian) on x, y, z (drawn even at
    gaussian = 0, as np.random.normal(scale=0) is)."""
    rs = np.random.RandomState(seed)
    s = np.sqrt(n / 120.0) if scale_density else 1.0
    orig = np.zeros((n, 3))
    orig[:, 0] = rs.normal(0.0, stds[0] * s, n)
    orig[:, 1] = rs.normal(0.0, stds[1] * s, n)
    orig[:, 2] = rs.normal(0.0, stds[2] * s, n)
    moved = orig.copy()
    moved[:, 1] += rigid
    moved += rs.normal(0.0, gaussian, (n, 3))
    orig = rotate_points(orig, *angles) + np.asarray(mean)
    moved = rotate_points(moved, *angles) + np.asarray(mean)
    return orig, moved


def look_at(camera_pos, target_pos, up=np.array([0, 1, 0], np.float32)):
    """SLAM::lookAt (SLAM.cc:340-351), fp32."""
    c = np.asarray(camera_pos, np.float32)
    t = np.asarray(target_pos, np.float32)
    f = (t - c); f = (f / np.linalg.norm(f)).astype(np.float32)
    r = np.cross(up, f).astype(np.float32); r = (r / np.linalg.norm(r)).astype(np.float32)
    u = np.cross(f, r).astype(np.float32); u = (u / np.linalg.norm(u)).astype(np.float32)
    return np.stack([r, u, f], 1).astype(np.float32)


def kb8_project(kb8, pc):
    """KannalaBrandt8::project (fp32), vectorised."""
    pc = np.asarray(pc, np.float32)
    k = kb8.astype(np.float32)
    x2y2 = pc[:, 0] * pc[:, 0] + pc[:, 1] * pc[:, 1]
    theta = np.arctan2(np.sqrt(x2y2), pc[:, 2]).astype(np.float32)
    psi = np.arctan2(pc[:, 1], pc[:, 0]).astype(np.float32)
    t2 = theta * theta; t3 = theta * t2; t5 = t3 * t2; t7 = t5 * t2; t9 = t7 * t2
    r = theta + k[4] * t3 + k[5] * t5 + k[6] * t7 + k[7] * t9
    u = k[0] * r * np.cos(psi) + k[2]
    v = k[1] * r * np.sin(psi) + k[3]
    return np.stack([u, v], 1).astype(np.float32)


def kb8_unproject(kb8, uv, precision=1e-6):
    """KannalaBrandt8::unproject (KannalaBrandt8.cc:51-83), fp32."""
    k = kb8.astype(np.float32)
    uv = np.asarray(uv, np.float32)
    px = ((uv[:, 0] - k[2]) / k[0]).astype(np.float32)
    py = ((uv[:, 1] - k[3]) / k[1]).astype(np.float32)
    theta_d = np.sqrt(px * px + py * py).astype(np.float32)
    theta = theta_d.copy()
    for _ in range(10):
        t2 = theta * theta; t4 = t2 * t2; t6 = t4 * t2; t8 = t4 * t4
        fix = (theta * (1 + k[4] * t2 + k[5] * t4 + k[6] * t6 + k[7] * t8) - theta_d) / \
              (1 + 3 * k[4] * t2 + 5 * k[5] * t4 + 7 * k[6] * t6 + 9 * k[7] * t8)
        theta = (theta - fix).astype(np.float32)
        if np.all(np.abs(fix) < precision):
            break
    s = np.sin(theta) / theta_d
    return np.stack([s * px, s * py, np.cos(theta)], 1).astype(np.float32)


def triangulate_nrslam_far(xn1, xn2, T1w, T2w):
    """triangulateNRSLAM(..., "FarPoints") Geometry.cc:103-153, vectorised fp32."""
    f0 = xn1 / np.linalg.norm(xn1, axis=1, keepdims=True)
    f1 = xn2 / np.linalg.norm(xn2, axis=1, keepdims=True)
    T21 = T2w * T1w.inverse()
    t = T21.t; R = T21.R
    Rf0 = f0 @ R.T
    p = np.cross(Rf0, f1); q = np.cross(Rf0, t); r = np.cross(f1, t)
    pn = np.linalg.norm(p, axis=1); qn = np.linalg.norm(q, axis=1); rn = np.linalg.norm(r, axis=1)
    lam0 = rn / pn; lam1 = qn / pn
    point0 = lam0[:, None] * Rf0
    point1 = lam1[:, None] * f1
    x1 = (qn / (qn + rn))[:, None] * (t + (rn / pn)[:, None] * (Rf0 + f1))
    point0 = t + point0
    p3d1 = point0 + (point0 - x1)
    p3d2 = point1 + (point1 - x1)
    Ti = T2w.inverse()
    return (Ti * p3d1.astype(np.float32)), (Ti * p3d2.astype(np.float32))


def triangulate_simulated(kb8_1, kb8_2, uv1, uv2, T1w, T2w, min_cos=0.9998):
    """Mapping::triangulateSimulatedMapPoints (Mapping.cc:280-349; NRSLAM, FarPoints) with
    isValidParallax (:351-366), vectorised fp32 host restatement.  The device version is
    deftri_triangulate_nrslam.  Returns (x3d_1, x3d_2, valid)."""
    xn1 = kb8_unproject(kb8_1, uv1); xn2 = kb8_unproject(kb8_2, uv2)
    xn1 = xn1 / np.linalg.norm(xn1, axis=1, keepdims=True)
    xn2 = xn2 / np.linalg.norm(xn2, axis=1, keepdims=True)
    x3d1, x3d2 = triangulate_nrslam_far(xn1, xn2, T1w, T2w)
    z1 = (T1w * x3d1)[:, 2]; z2 = (T2w * x3d2)[:, 2]
    ray1 = xn1 @ T1w.inverse().R.T; ray2 = xn2 @ T2w.inverse().R.T
    ray1 /= np.linalg.norm(ray1, axis=1, keepdims=True); ray2 /= np.linalg.norm(ray2, axis=1, keepdims=True)
    cosp = (ray1 * ray2).sum(1) / (np.linalg.norm(ray1, axis=1) * np.linalg.norm(ray2, axis=1))
    valid = (z1 >= 0) & (z2 >= 0) & (cosp <= min_cos) & np.all(np.isfinite(x3d1), 1) & np.all(np.isfinite(x3d2), 1)
    return x3d1, x3d2, valid


def simulate_two_view(n=120, seed=0, orig=None, moved=None, c1=(-0.10, 0.02, 0.12),
                      c2=(0.14, 0.01, 0.06), kb8=SIM_KB8, rep_error=1.0, decimals=1,
                      depth_error=3.0, depth_scales=(0.4, 1.7), min_cos=0.9998, n_scales=8,
                      scale_factor=1.2, rigid=0.0025, gaussian=0.0025, scale_scene=False, compact=False):
    """The reference's Execution/simulation.cc flow up to deformationOptimization.

    scale_scene: for large n the cloud extents grow by sqrt(n/120) (generate_points); this also
      scales the camera positions and the 0.2 m depth offset, so the viewing geometry of the
      reference's 120-point scene is kept (otherwise points fall behind / beside the cameras).
    compact: drop correspondences that fail the triangulation checks before slots are assigned
      (the reference leaves null slots, which triggers its slot/position index quirk; see
      SURVEY Appendix B.2 — a compacted scene is the same as running the reference on the
      filtered point files).
    Returns (Map, ground_truth dict)."""
    if orig is None:
        sc = np.sqrt(n / 120.0) if scale_scene else 1.0
        orig, moved = generate_points(n, rigid=rigid, gaussian=gaussian, seed=seed,
                                      mean=(0.0, 0.0, 0.2 * sc))
        c1 = tuple(np.asarray(c1) * sc); c2 = tuple(np.asarray(c2) * sc)
    orig = np.asarray(orig, np.float32); moved = np.asarray(moved, np.float32)
    n = len(orig)
    # SLAM::setCameraPoses + getSimulatedDepthMeasurements + createKeyPoints (SLAM.cc:223-338): the
    # reference's noise streams and Sophus poses (host C++, deftri_sim_two_view)
    from . import capi
    uv1, uv2, d1, d2, q1, q2 = capi.sim_two_view(orig, moved, c1, c2, kb8, kb8, rep_error, decimals, depth_error,
                                                 depth_scales)
    T1w = SE3f(np.eye(3, dtype=np.float32), np.asarray(c1, np.float32), q=q1[:4])
    T2w = SE3f(look_at(c2, moved[0]), np.asarray(c2, np.float32), q=q2[:4])
    inv_s2 = inv_sigma2_table(n_scales, scale_factor)
    kf0 = KeyFrame(0, T1w, kb8, n, inv_s2, uv1, np.zeros(n, np.int32), d1)
    kf1 = KeyFrame(1, T2w, kb8, n, inv_s2, uv2, np.zeros(n, np.int32), d2)
    m = Map()
    m.insert_keyframe(kf0)
    m.insert_keyframe(kf1)
    x3d1, x3d2, valid = triangulate_simulated(kb8, kb8, uv1, uv2, T1w, T2w, min_cos)
    if compact and not valid.all():
        keep = np.where(valid)[0]
        return simulate_two_view(n=len(keep), seed=seed, orig=orig[keep], moved=moved[keep], c1=c1, c2=c2,
                                 kb8=kb8, rep_error=rep_error, decimals=decimals, depth_error=depth_error,
                                 depth_scales=depth_scales, min_cos=min_cos, n_scales=n_scales,
                                 scale_factor=scale_factor, compact=True)
    next_id = 0
    for i in range(n):
        if not valid[i]:
            continue
        mp1 = MapPoint(x3d1[i], next_id); mp2 = MapPoint(x3d2[i], next_id + 1)
        next_id += 2
        m.insert_map_point(mp1); m.insert_map_point(mp2)
        m.add_observation(0, mp1.id, i); m.add_observation(1, mp2.id, i)
        kf0.map_points[i] = mp1; kf1.map_points[i] = mp2
    gt = {"original": orig, "moved": moved, "valid": valid}
    return m, gt


def simulate_multi_view(n=1000, k=8, seed=0, kb8=DRUNKARD_KB8, radius=0.12, rep_error=1.0,
                        decimals=1, depth_error=3.0, deform=0.0025, noise3d=0.004):
    """K-keyframe extension (configs C3-C5): K cameras on an arc around the cloud, each KF holding
    its own copy of the correspondences (slot i in every KF), deformed per KF.  Initial MapPoints
    are the ground truth plus N(0, noise3d) (the triangulation step is two-view only in the
    reference, Mapping.cc:100-103)."""
    rng = np.random.default_rng(seed + 7)
    base, _ = generate_points(n, rigid=0.0, gaussian=0.0, seed=seed)
    inv_s2 = inv_sigma2_table(8, 1.2)
    m = Map()
    next_id = 0
    center = base.mean(0)
    for kk in range(k):
        ang = np.deg2rad(-30 + 60 * kk / max(k - 1, 1))
        cpos = center + np.array([radius * np.sin(ang), 0.0, -radius * np.cos(ang)]) * 1.0
        pts = base + rng.normal(0, deform, base.shape) + np.array([0, deform * kk, 0])
        R = look_at(cpos, center)
        Tcw = SE3f(R.T, -(R.T @ cpos.astype(np.float32)))
        pc = Tcw * pts.astype(np.float32)
        uv = kb8_project(kb8, pc)
        uv = (np.round((uv.astype(np.float64) + rng.normal(0, rep_error, uv.shape)) * 10 ** decimals)
              / 10 ** decimals).astype(np.float32)
        dep = (pc[:, 2] + rng.normal(0, depth_error / 1000.0, n)).astype(np.float32)
        kf = KeyFrame(kk, Tcw, kb8, n, inv_s2, uv, np.zeros(n, np.int32), dep)
        m.insert_keyframe(kf)
        init = (pts + rng.normal(0, noise3d, pts.shape)).astype(np.float32)
        for i in range(n):
            mp = MapPoint(init[i], next_id); next_id += 1
            m.insert_map_point(mp)
            m.add_observation(kk, mp.id, i)
            kf.map_points[i] = mp
    return m, {"base": base}


class ArrayMap:
    """A Map held as per-keyframe arrays (slot i of every keyframe = correspondence i, MapPoint id
    k * n + i), for scenes too large for one Python object per MapPoint (C3-C5 sizes).  Exposes the
    same C view as Map.to_c (keyframes in the libstdc++ unordered_map order: reverse insertion)."""

    def __init__(self, kfs, kb8, inv_sigma2):
        self.kfs = kfs                 # list of dicts: id, pose (SE3f), uv [n,2], depth [n], pos [n,3] f32
        self.kb8 = np.asarray(kb8, np.float32)
        self.inv_sigma2 = np.asarray(inv_sigma2, np.float32)

    @property
    def n_points(self):
        return sum(len(k["pos"]) for k in self.kfs)

    def to_c(self):
        from . import _abi
        order = list(reversed(range(len(self.kfs))))
        kfs = (_abi.KeyFrameC * len(order))()
        keep = {"kfs": kfs, "arrays": []}
        for n, k in enumerate(order):
            kf, c = self.kfs[k], kfs[n]
            ns = len(kf["pos"])
            c.id = kf["id"]
            c.pose[:] = list(kf["pose"].as7())
            c.kb8[:] = [float(v) for v in self.kb8]
            c.n_scales = len(self.inv_sigma2)
            c.inv_sigma2 = _abi.ptr(self.inv_sigma2, _abi.f32)
            c.depth_scale = 1.0
            c.n_slots = ns
            pid = np.arange(ns, dtype=np.int64) + np.int64(kf["id"]) * ns
            pos = np.ascontiguousarray(kf["pos"], np.float32)
            obs = np.arange(ns, dtype=np.int32)
            uv = np.ascontiguousarray(kf["uv"], np.float32)
            octv = np.zeros(ns, np.int32)
            dep = np.ascontiguousarray(kf["depth"], np.float32)
            c.point_id, c.point_pos, c.obs_index = _abi.ptr(pid, _abi.i64), _abi.ptr(pos, _abi.f32), _abi.ptr(obs, _abi.i32)
            c.kp_uv, c.kp_octave, c.depth = _abi.ptr(uv, _abi.f32), _abi.ptr(octv, _abi.i32), _abi.ptr(dep, _abi.f32)
            c.n_obs = ns
            keep["arrays"].append((k, pid, pos, obs, uv, octv, dep))
        m = _abi.MapC()
        m.n_keyframes = len(order)
        m.keyframes = C_cast(kfs)
        m.global_t[:] = [0, 0, 0, 1, 0, 0, 0]
        m.n_global = 0
        return m, keep


def C_cast(kfs):
    import ctypes
    from . import _abi
    return ctypes.cast(kfs, ctypes.POINTER(_abi.KeyFrameC))


def multi_view_arrays(n=1000, k=8, seed=0, kb8=DRUNKARD_KB8, radius=0.12, rep_error=1.0, decimals=1,
                      depth_error=3.0, deform=0.0025, noise3d=0.004, scale_scene=True):
    """simulate_multi_view's recipe (K cameras on an arc, each keyframe its own deformed copy of the
    cloud, initial MapPoints = truth + N(0, noise3d)) as an ArrayMap.  scale_scene: the camera arc
    radius grows with the cloud's sqrt(n/120) extents (as two_view_problem's scale_scene), keeping
    the reference's 120-point viewing geometry at C3-C5 sizes."""
    rng = np.random.default_rng(seed + 7)
    base, _ = generate_points(n, rigid=0.0, gaussian=0.0, seed=seed)
    sc = np.sqrt(n / 120.0) if scale_scene else 1.0
    center = base.mean(0)
    kfs = []
    for kk in range(k):
        ang = np.deg2rad(-30 + 60 * kk / max(k - 1, 1))
        cpos = center + np.array([radius * sc * np.sin(ang), 0.0, -radius * sc * np.cos(ang)])
        pts = base + rng.normal(0, deform, base.shape) + np.array([0, deform * kk, 0])
        R = look_at(cpos, center)
        Tcw = SE3f(R.T, -(R.T @ cpos.astype(np.float32)))
        pc = Tcw * pts.astype(np.float32)
        uv = kb8_project(kb8, pc)
        uv = (np.round((uv.astype(np.float64) + rng.normal(0, rep_error, uv.shape)) * 10 ** decimals)
              / 10 ** decimals).astype(np.float32)
        dep = (pc[:, 2] + rng.normal(0, depth_error / 1000.0, n)).astype(np.float32)
        init = (pts + rng.normal(0, noise3d, pts.shape)).astype(np.float32)
        kfs.append({"id": kk, "pose": Tcw, "uv": uv, "depth": dep, "pos": init})
    return ArrayMap(kfs, kb8, inv_sigma2_table(8, 1.2))


def multi_view_problem(n, k, seed=1, kb8=DRUNKARD_KB8, rep_weight=1.0, arap_weight=1e7, depth_sigma=np.float32(0.3),
                       pair_window=0):
    """The C3 / C4 / C5 benchmark graphs: multi_view_arrays + the product's host graph builder
    (deftri_arap_build_graph; pair_window > 0: only keyframe pairs at most that far apart in map
    order — the documented sliding-window deviation of C5)."""
    from . import capi
    m = multi_view_arrays(n=n, k=k, seed=seed, kb8=kb8)
    host = capi.Context(-1)
    if pair_window:
        host.set_pair_window(pair_window)
    p = host.build_graph(m, rep_weight, arap_weight, depth_sigma)
    host.close()
    return p


def two_view_problem(n, seed=1, rep_weight=1.0, arap_weight=2e5, depth_sigma=np.float32(0.003), return_map=False,
                     kb8=None):
    """The benchmark scene (BASELINE C1/C2 shapes): simulate_two_view with the extents scaled to n
    correspondences and failed triangulations dropped, then the arapOptimization graph built by the
    product's host builder (deftri_arap_build_graph).  kb8: the camera (default Simulation.yaml's)."""
    from . import capi
    kw = {} if kb8 is None else {"kb8": kb8}
    m, _ = simulate_two_view(n=n, seed=seed, scale_scene=True, compact=True, **kw)
    host = capi.Context(-1)
    p = host.build_graph(m, rep_weight, arap_weight, depth_sigma)
    host.close()
    return (p, m) if return_map else p
