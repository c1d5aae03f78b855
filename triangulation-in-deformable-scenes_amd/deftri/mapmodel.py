"""Minimal mirror of the reference's Map / KeyFrame / MapPoint (Modules/Map/*) — only what the
solver reads and writes (SURVEY §8b "Ownership"):

  MapPoint  : id, fp32 world position            (MapPoint.cc:22-49)
  KeyFrame  : id, pose T_cw (SE3f), KB8 calibration, keypoints + octaves, per-index simulated
              depth, invSigma2 table, estimatedDepthScale_, MapPoint slots (KeyFrame.cc:93-210)
  Map       : keyframes (unordered_map<ID,KF>), map points, observations
              (Map::addObservation / isMapPointInKeyFrame, Map.cc:100-132, 257-264),
              global KF-pair transformations (Map.cc:323-330)

Iteration order of the reference's `std::unordered_map<ID, KeyFrame_>` (libstdc++, integer
hash): `Map.kf_order()` asks the native library for it (deftri_keyframe_order: the same container
filled in this map's insertion order, not a restatement).  Up to 13 keyframes it is the reverse
insertion order, which is what makes pKF1 = KF 0 and pKF2 = KF 1 for the two-view case (SURVEY
Appendix B.1); from 14 on the rehash to 29 buckets interleaves it.  It is what the C-ABI receives.

`Map.clone()` is Map::clone (Map.cc:30-58) as the weight search sees it: new MapPoints and
KeyFrames, the keyframes re-inserted in this map's iteration order (so the clone iterates them in
the order that insertion sequence gives), and NO global-transformation table (the reference does not
copy mGTransformation_).  `copy.deepcopy` stays a plain deep copy (tests use it for isolation).
"""
import ctypes as C
import numpy as np

from . import _abi


def quat_from_mat(R):
    """Eigen Quaternion(Matrix3) (quaternionbase_assign_impl) — returns x, y, z, w (f64)."""
    m = np.asarray(R, dtype=np.float64)
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0:
        t = np.sqrt(t + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        return np.array([(m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t, w])
    i = 0
    if m[1, 1] > m[0, 0]:
        i = 1
    if m[2, 2] > m[i, i]:
        i = 2
    j, k = (i + 1) % 3, (i + 2) % 3
    c = np.zeros(3)
    t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
    c[i] = 0.5 * t
    t = 0.5 / t
    w = (m[k, j] - m[j, k]) * t
    c[j] = (m[j, i] + m[i, j]) * t
    c[k] = (m[k, i] + m[i, k]) * t
    return np.array([c[0], c[1], c[2], w])


def mat_from_quat(q):
    x, y, z, w = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]])


class SE3f:
    """Sophus::SE3f stand-in: rotation (fp32 3x3) + translation (fp32)."""
    def __init__(self, R=None, t=None, q=None):
        self.R = np.eye(3, dtype=np.float32) if R is None else np.asarray(R, dtype=np.float32)
        self.t = np.zeros(3, dtype=np.float32) if t is None else np.asarray(t, dtype=np.float32)
        # Sophus stores the rotation as an fp32 unit quaternion (x y z w); when the pose was built
        # the reference's way (deftri_sim_two_view) that exact quaternion is kept for as7()
        self.q = None if q is None else np.asarray(q, dtype=np.float32)

    def __mul__(self, o):
        if isinstance(o, SE3f):
            return SE3f(self.R @ o.R, self.R @ o.t + self.t)
        return (np.asarray(o, dtype=np.float32) @ self.R.T + self.t).astype(np.float32)

    def inverse(self):
        return SE3f(self.R.T, -(self.R.T @ self.t))

    def unit_quaternion(self):
        q = quat_from_mat(self.R.astype(np.float64))
        return q / np.linalg.norm(q)

    def as7(self):
        """g2o::SE3Quat(unit_quaternion().cast<double>(), translation().cast<double>())."""
        if getattr(self, "_as7", None) is not None:        # an entry deftri_global_insert formed
            return np.array(self._as7, dtype=np.float64)
        q = (self.q if self.q is not None else self.unit_quaternion().astype(np.float32)).astype(np.float64)
        if q[3] < 0:
            q = -q
        # SE3Quat::normalizeRotation in one fixed order of additions (the native se3f_as7 / the C++
        # adapter's se3quat7 use the same)
        q = q / np.sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3])
        return np.concatenate([q, self.t.astype(np.float64)])

    @staticmethod
    def from7(a):
        a = np.asarray(a, dtype=np.float64)
        q = a[:4] / np.linalg.norm(a[:4])
        return SE3f(mat_from_quat(q).astype(np.float32), a[4:7].astype(np.float32))


class MapPoint:
    _next_id = 0

    def __init__(self, position, pid=None):
        self.position = np.asarray(position, dtype=np.float32).copy()
        if pid is None:
            pid = MapPoint._next_id
            MapPoint._next_id += 1
        self.id = int(pid)


class KeyFrame:
    def __init__(self, kid, pose, kb8, n_slots, inv_sigma2, keypoints=None, octaves=None, depth=None):
        self.id = int(kid)
        self.pose = pose                              # SE3f, T_cw
        self.kb8 = np.asarray(kb8, dtype=np.float32)
        self.inv_sigma2 = np.asarray(inv_sigma2, dtype=np.float32)
        self.keypoints = np.zeros((n_slots, 2), np.float32) if keypoints is None else np.asarray(keypoints, np.float32)
        self.octaves = np.zeros(n_slots, np.int32) if octaves is None else np.asarray(octaves, np.int32)
        self.depth = np.zeros(n_slots, np.float32) if depth is None else np.asarray(depth, np.float32)
        self.map_points = [None] * n_slots
        self.estimated_depth_scale = 1.0               # KeyFrame.h:198 default

    @property
    def n_slots(self):
        return len(self.map_points)


class Map:
    def __init__(self, min_common_obs=15):
        self.keyframes = {}           # insertion-ordered
        self.map_points = {}
        self.kf_obs = {}              # kf id -> {mp id -> idx}        (Map::mKeyFrameObs_)
        self.mp_obs = {}              # mp id -> {kf id -> idx}        (Map::mMapPointObs_)
        self.covis = {}               # kf id -> {kf id -> count}      (Map::mCovisibilityGraph_)
        self.min_common_obs = min_common_obs   # Map.minObs (Simulation.yaml:42)
        self.global_T = {}            # (kf1, kf2) -> SE3f

    def insert_keyframe(self, kf):
        self.keyframes[kf.id] = kf
        self.kf_obs.setdefault(kf.id, {})

    def insert_map_point(self, mp):
        self.map_points[mp.id] = mp

    def add_observation(self, kf_id, mp_id, idx):
        """Map::addObservation (Map.cc:100-132): observation tables + covisibility counts."""
        assert mp_id not in self.kf_obs[kf_id]
        self.kf_obs[kf_id][mp_id] = int(idx)
        obs = self.mp_obs.setdefault(mp_id, {})
        obs[kf_id] = int(idx)
        for cov in obs:
            if cov == kf_id:
                continue
            a = self.covis.setdefault(kf_id, {})
            a[cov] = a.get(cov, 0) + 1
            b = self.covis.setdefault(cov, {})
            b[kf_id] = b.get(kf_id, 0) + 1

    def remove_observation(self, kf_id, mp_id):
        """Map::removeObservation (Map.cc:134-149)."""
        del self.kf_obs[kf_id][mp_id]
        del self.mp_obs[mp_id][kf_id]
        for cov in self.mp_obs[mp_id]:
            self.covis[kf_id][cov] -= 1
            self.covis[cov][kf_id] -= 1

    def get_local_map_of_keyframe(self, kf_id):
        """Map::getLocalMapOfKeyFrame (Map.cc:178-209): (local map point ids, local KF ids, fixed KF
        ids), each sorted ascending like the reference's std::set<ID>."""
        local_kfs = {kf_id}
        local_mps = set(self.kf_obs.get(kf_id, {}).keys())
        for cov, n in self.covis.get(kf_id, {}).items():
            if n > self.min_common_obs:
                local_kfs.add(cov)
                local_mps.update(self.kf_obs.get(cov, {}).keys())
        all_kfs = set()
        for mp in local_mps:
            all_kfs.update(self.mp_obs.get(mp, {}).keys())
        return sorted(local_mps), sorted(local_kfs), sorted(all_kfs - local_kfs)

    def is_map_point_in_keyframe(self, mp_id, kf_id):
        return self.kf_obs.get(kf_id, {}).get(mp_id, -1)

    def kf_order(self):
        """libstdc++ unordered_map<ID,KF> iteration order of this map's insertion sequence."""
        from .capi import keyframe_order
        return keyframe_order(list(self.keyframes.keys()))

    def clone(self):
        """Map::clone (Map.cc:30-58): an independent copy whose keyframes were inserted in this map's
        iteration order and whose global-transformation table is empty."""
        import copy
        new = copy.deepcopy(self)
        new.keyframes = {kid: new.keyframes[kid] for kid in self.kf_order()}
        new.global_T = {}
        return new

    def insert_global_T(self, kf1, kf2, T):
        self.global_T[(kf1, kf2)] = T
        self.global_T[(kf2, kf1)] = T.inverse()

    def insert_global_from7(self, kf1, kf2, t7):
        """Map::insertGlobalKeyFramesTransformation(kf1, kf2, T) of a solved T_g (7-vector): the two
        entries exactly as the native loop stores them (deftri_global_insert)."""
        from .capi import global_insert
        fwd, inv = global_insert(t7)
        a, b = SE3f.from7(fwd), SE3f.from7(inv)
        a._as7, b._as7 = fwd, inv
        self.global_T[(kf1, kf2)] = a
        self.global_T[(kf2, kf1)] = b

    def get_global_T(self, kf1, kf2):
        return self.global_T.get((kf1, kf2), SE3f())

    def __deepcopy__(self, memo):
        """Map::clone (the weight search clones the map for every evaluation, nloptOptimization.cc:
        the same independent copy as the generic copy.deepcopy — every MapPoint, KeyFrame and table
        new, numpy arrays copied, the KeyFrames' slots pointing at the new MapPoints — built
        directly instead of by the generic object walk (C2: 3.6 s -> 0.5 s on this container)."""
        import copy
        new = Map.__new__(Map)
        memo[id(self)] = new
        mps = {}
        new_mp = MapPoint.__new__
        for pid, mp in self.map_points.items():
            c = new_mp(MapPoint)
            d = mp.__dict__
            if len(d) == 2 and "position" in d and "id" in d:        # the usual MapPoint
                c.__dict__ = {"position": d["position"].copy(), "id": d["id"]}
            else:
                c.__dict__ = {k: (v.copy() if isinstance(v, np.ndarray) else v if isinstance(v, (int, float, str))
                                  else copy.deepcopy(v, memo)) for k, v in d.items()}
            memo[id(mp)] = c
            mps[pid] = c
        kfs = {}
        for kid, kf in self.keyframes.items():
            c = KeyFrame.__new__(KeyFrame)
            d = {}
            for k, v in kf.__dict__.items():
                if k == "map_points":
                    get = memo.get
                    d[k] = [None if m is None else (get(id(m)) or copy.deepcopy(m, memo)) for m in v]
                elif isinstance(v, np.ndarray):
                    d[k] = v.copy()
                elif isinstance(v, (int, float, str)):
                    d[k] = v
                else:
                    d[k] = copy.deepcopy(v, memo)
            c.__dict__ = d
            memo[id(kf)] = c
            kfs[kid] = c
        for k, v in self.__dict__.items():
            if k == "map_points":
                new.map_points = mps
            elif k == "keyframes":
                new.keyframes = kfs
            elif k in ("kf_obs", "mp_obs", "covis"):
                setattr(new, k, {a: dict(b) for a, b in v.items()})
            else:
                setattr(new, k, copy.deepcopy(v, memo))
        return new

    # ---- C-ABI view -------------------------------------------------------------------------
    def to_c(self):
        """Build a deftri_map view.  Returns (MapC, keep) — keep owns the arrays; positions and
        depth scales are written back through `from_c`."""
        order = self.kf_order()
        kfs = (_abi.KeyFrameC * len(order))()
        keep = {"kfs": kfs, "arrays": []}
        for n, kid in enumerate(order):
            kf = self.keyframes[kid]
            c = kfs[n]
            c.id = kf.id
            c.pose[:] = list(kf.pose.as7())
            c.kb8[:] = [float(v) for v in kf.kb8]
            c.n_scales = len(kf.inv_sigma2)
            inv = np.ascontiguousarray(kf.inv_sigma2, np.float32)
            c.inv_sigma2 = _abi.ptr(inv, _abi.f32)
            c.depth_scale = kf.estimated_depth_scale
            ns = kf.n_slots
            c.n_slots = ns
            pid = np.array([mp.id if mp is not None else -1 for mp in kf.map_points], np.int64)
            pos = np.zeros((ns, 3), np.float32)
            obs = np.full(ns, -1, np.int32)
            for i, mp in enumerate(kf.map_points):
                if mp is not None:
                    pos[i] = mp.position
                    obs[i] = self.is_map_point_in_keyframe(mp.id, kf.id)
            uv = np.ascontiguousarray(kf.keypoints, np.float32)
            octv = np.ascontiguousarray(kf.octaves, np.int32)
            dep = np.ascontiguousarray(kf.depth, np.float32)
            c.point_id, c.point_pos, c.obs_index = _abi.ptr(pid, _abi.i64), _abi.ptr(pos, _abi.f32), _abi.ptr(obs, _abi.i32)
            c.kp_uv, c.kp_octave, c.depth = _abi.ptr(uv, _abi.f32), _abi.ptr(octv, _abi.i32), _abi.ptr(dep, _abi.f32)
            c.n_obs = len(kf.keypoints)
            keep["arrays"].append((kid, pid, pos, obs, uv, octv, dep, inv))
        m = _abi.MapC()
        m.n_keyframes = len(order)
        m.keyframes = C.cast(kfs, C.POINTER(_abi.KeyFrameC))
        m.global_t[:] = [0, 0, 0, 1, 0, 0, 0]
        # Map::mGTransformation_ (both directions, as insertGlobalKeyFramesTransformation stores
        # them): every pair looks up (k2->first, k1->first), g2oBundleAdjustment.cc:664
        entries = sorted(self.global_T.items())
        glob = (_abi.GlobalEntryC * max(1, len(entries)))()
        for n, ((k1, k2), T) in enumerate(entries):
            glob[n].kf1, glob[n].kf2 = int(k1), int(k2)
            glob[n].t[:] = list(T.as7())
        m.n_global = len(entries)
        m.globals = C.cast(glob, C.POINTER(_abi.GlobalEntryC))
        keep["globals"] = glob
        return m, keep

    def from_c(self, m, keep):
        """Write back positions (fp32), depth scales and the global T (reference :967-1007)."""
        for n, (kid, pid, pos, *_rest) in enumerate(keep["arrays"]):
            kf = self.keyframes[kid]
            kf.estimated_depth_scale = float(m.keyframes[n].depth_scale)
            for i, mp in enumerate(kf.map_points):
                if mp is not None:
                    mp.position = pos[i].copy()
        if m.n_keyframes >= 2:
            # the reference hard-codes insertGlobalKeyFramesTransformation(0, 1, T) (:1007): KF ids 0
            # and 1, whatever the map's keyframe ids are
            self.insert_global_from7(0, 1, list(m.global_t[:]))
