"""Flattened LM problem (the graph `arapOptimization` builds), as numpy arrays.

Field meanings follow include/deftri.h (deftri_problem_desc).  A Problem can be saved to /
loaded from an .npz (the golden fixtures under tests/golden/ use this format) and turned into
the ctypes descriptor passed across the C-ABI.
"""
from dataclasses import dataclass, field, fields
import numpy as np

from . import _abi

_I32 = ("rep_point", "rep_cam", "dep_point", "dep_scale", "dep_cam", "arap_pts", "arap_pair",
        "arap_rot")
_F64 = ("points", "tg", "scales", "cam_pose", "rep_obs", "rep_info", "dep_meas", "dep_info",
        "arap_w", "rot", "pair_area", "pair_info", "order_xy")


@dataclass
class Problem:
    points: np.ndarray                 # [P,3] f64
    tg: np.ndarray                     # [Q,7] f64 (qx qy qz qw tx ty tz)
    scales: np.ndarray                 # [S] f64
    cam_kb8: np.ndarray                # [C,8] f32
    cam_pose: np.ndarray               # [C,7] f64
    rep_point: np.ndarray              # [R] i32
    rep_cam: np.ndarray                # [R] i32
    rep_obs: np.ndarray                # [R,2] f64
    rep_info: np.ndarray               # [R] f64
    dep_point: np.ndarray              # [D] i32
    dep_scale: np.ndarray              # [D] i32
    dep_cam: np.ndarray                # [D] i32
    dep_meas: np.ndarray               # [D] f64
    dep_info: np.ndarray               # [D] f64
    arap_pts: np.ndarray               # [E,4] i32
    arap_pair: np.ndarray              # [E] i32
    arap_rot: np.ndarray               # [E,2] i32
    arap_w: np.ndarray                 # [E] f64
    rot: np.ndarray                    # [nR,3,3] f64
    pair_area: np.ndarray              # [Q] f64
    pair_info: np.ndarray              # [Q] f64
    huber_delta: float = float(np.float32(np.sqrt(100.991)))
    order_xy: np.ndarray = None        # [P,2] f64 or None
    _keep: list = field(default_factory=list, repr=False, compare=False)

    def __post_init__(self):
        for k in _I32:
            setattr(self, k, np.ascontiguousarray(getattr(self, k), dtype=np.int32))
        for k in _F64:
            v = getattr(self, k)
            if v is not None:
                setattr(self, k, np.ascontiguousarray(v, dtype=np.float64))
        self.cam_kb8 = np.ascontiguousarray(self.cam_kb8, dtype=np.float32)
        self.points = self.points.reshape(-1, 3)
        self.tg = self.tg.reshape(-1, 7)
        self.cam_kb8 = self.cam_kb8.reshape(-1, 8)
        self.cam_pose = self.cam_pose.reshape(-1, 7)
        self.rep_obs = self.rep_obs.reshape(-1, 2)
        self.arap_pts = self.arap_pts.reshape(-1, 4)
        self.arap_rot = self.arap_rot.reshape(-1, 2)
        self.rot = self.rot.reshape(-1, 3, 3)

    # sizes -------------------------------------------------------------------------------
    @property
    def n_points(self): return int(self.points.shape[0])
    @property
    def n_pairs(self): return int(self.tg.shape[0])
    @property
    def n_scales(self): return int(self.scales.shape[0])
    @property
    def n_unknowns(self): return 6 * self.n_pairs + self.n_scales + 3 * self.n_points

    def summary(self):
        return dict(P=self.n_points, Q=self.n_pairs, S=self.n_scales, C=len(self.cam_pose),
                    R=len(self.rep_point), D=len(self.dep_point), E=len(self.arap_pair),
                    unknowns=self.n_unknowns)

    def validate(self):
        P_, Q, S, C = self.n_points, self.n_pairs, self.n_scales, len(self.cam_pose)
        def rng(a, hi, name):
            if a.size and (a.min() < 0 or a.max() >= hi):
                raise ValueError(f"{name} index out of range [0,{hi})")
        rng(self.rep_point, P_, "rep_point"); rng(self.rep_cam, C, "rep_cam")
        rng(self.dep_point, P_, "dep_point"); rng(self.dep_scale, S, "dep_scale")
        rng(self.dep_cam, C, "dep_cam"); rng(self.arap_pts, P_, "arap_pts")
        rng(self.arap_pair, Q, "arap_pair"); rng(self.arap_rot, len(self.rot), "arap_rot")
        return True

    # C-ABI --------------------------------------------------------------------------------
    def to_desc(self):
        d = _abi.ProblemDesc()
        d.n_points, d.n_pairs, d.n_scales = self.n_points, self.n_pairs, self.n_scales
        d.n_cams = len(self.cam_pose)
        d.n_rep, d.n_depth, d.n_arap = len(self.rep_point), len(self.dep_point), len(self.arap_pair)
        d.n_rot = len(self.rot)
        keep = []
        def f64(name):
            a = getattr(self, name)
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=np.float64); keep.append(a)
            return _abi.ptr(a, _abi.f64)
        def i32(name):
            a = np.ascontiguousarray(getattr(self, name), dtype=np.int32); keep.append(a)
            return _abi.ptr(a, _abi.i32)
        d.points, d.tg, d.scales = f64("points"), f64("tg"), f64("scales")
        kb = np.ascontiguousarray(self.cam_kb8, dtype=np.float32); keep.append(kb)
        d.cam_kb8 = _abi.ptr(kb, _abi.f32)
        d.cam_pose = f64("cam_pose")
        d.rep_point, d.rep_cam, d.rep_obs, d.rep_info = i32("rep_point"), i32("rep_cam"), f64("rep_obs"), f64("rep_info")
        d.huber_delta = float(self.huber_delta)
        d.dep_point, d.dep_scale, d.dep_cam = i32("dep_point"), i32("dep_scale"), i32("dep_cam")
        d.dep_meas, d.dep_info = f64("dep_meas"), f64("dep_info")
        d.arap_pts, d.arap_pair, d.arap_rot, d.arap_w = i32("arap_pts"), i32("arap_pair"), i32("arap_rot"), f64("arap_w")
        d.rot, d.pair_area, d.pair_info = f64("rot"), f64("pair_area"), f64("pair_info")
        d.order_xy = f64("order_xy")
        self._keep = keep
        return d

    def digest(self):
        """sha256 (hex, 16 chars) over every array of the graph in field order: a golden records the
        graph it was computed on, so a graph-builder change that moves any value shows as a stale
        golden instead of a silently looser pin."""
        import hashlib
        h = hashlib.sha256()
        for f in fields(self):
            if f.name.startswith("_"):
                continue
            v = getattr(self, f.name)
            if v is None:
                continue
            h.update(f.name.encode())
            h.update(np.ascontiguousarray(v).tobytes() if isinstance(v, np.ndarray) else repr(v).encode())
        return h.hexdigest()[:16]

    # persistence ----------------------------------------------------------------------------
    def save(self, path):
        arrs = {f.name: getattr(self, f.name) for f in fields(self)
                if not f.name.startswith("_") and getattr(self, f.name) is not None}
        arrs["huber_delta"] = np.array(self.huber_delta)
        np.savez_compressed(path, **arrs)

    @classmethod
    def load(cls, path):
        z = np.load(path, allow_pickle=False)
        kw = {k: z[k] for k in z.files}
        kw["huber_delta"] = float(kw["huber_delta"])
        return cls(**kw)

    @classmethod
    def from_desc(cls, d):
        """Copy a C descriptor (e.g. the one deftri_arap_build_graph returns) into numpy."""
        def arr(p, n, dt):
            if not p or n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)
        P_, Q, S, C = d.n_points, d.n_pairs, d.n_scales, d.n_cams
        R, D, E, NR = d.n_rep, d.n_depth, d.n_arap, d.n_rot
        return cls(points=arr(d.points, 3 * P_, np.float64), tg=arr(d.tg, 7 * Q, np.float64),
                   scales=arr(d.scales, S, np.float64), cam_kb8=arr(d.cam_kb8, 8 * C, np.float32),
                   cam_pose=arr(d.cam_pose, 7 * C, np.float64),
                   rep_point=arr(d.rep_point, R, np.int32), rep_cam=arr(d.rep_cam, R, np.int32),
                   rep_obs=arr(d.rep_obs, 2 * R, np.float64), rep_info=arr(d.rep_info, R, np.float64),
                   dep_point=arr(d.dep_point, D, np.int32), dep_scale=arr(d.dep_scale, D, np.int32),
                   dep_cam=arr(d.dep_cam, D, np.int32), dep_meas=arr(d.dep_meas, D, np.float64),
                   dep_info=arr(d.dep_info, D, np.float64),
                   arap_pts=arr(d.arap_pts, 4 * E, np.int32), arap_pair=arr(d.arap_pair, E, np.int32),
                   arap_rot=arr(d.arap_rot, 2 * E, np.int32), arap_w=arr(d.arap_w, E, np.float64),
                   rot=arr(d.rot, 9 * NR, np.float64), pair_area=arr(d.pair_area, Q, np.float64),
                   pair_info=arr(d.pair_info, Q, np.float64), huber_delta=d.huber_delta,
                   order_xy=(arr(d.order_xy, 2 * P_, np.float64).reshape(-1, 2) if d.order_xy else None))
