"""Reprojection metric of the reference: calculatePixelsStandDev (Modules/Utils/Geometry.cc:370-498).

This is the parity metric of the north star ("final reprojection RMSE"): per camera the RMS of
|obs - KB8(T p)| in u and v, averaged: desvc = (RMS_u + RMS_v) / 2 and desv = (desvc1 + desvc2) / 2.
The "variance" is the mean of squares (no mean subtraction, :449-480).  Projection is fp32 with the
homogeneous T.matrix() product, as in the reference.  Like the reference, nMatches accumulates over
all pairs and the per-camera values of the last pair are reported.
"""
import numpy as np

from .sim import kb8_project


def _pose_matrix_f32(kf):
    """Sophus::SE3f::matrix(): Eigen toRotationMatrix of the fp32 unit quaternion, in fp32."""
    a = kf.pose.as7()
    x, y, z, w = (np.float32(v) for v in a[:4])
    two = np.float32(2)
    tx, ty, tz = two * x, two * y, two * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    one = np.float32(1)
    R = np.array([[one - (tyy + tzz), txy - twz, txz + twy],
                  [txy + twz, one - (txx + tzz), tyz - twx],
                  [txz - twy, tyz + twx, one - (txx + tyy)]], np.float32)
    return R, np.asarray(a[4:7], np.float64).astype(np.float32)


def _project_h(kf, p3w):
    """T1w.matrix() * [p;1] in fp32, column by column as Eigen's lazy product (no FMA), then KB8
    project (Geometry.cc:423-431)."""
    R, t = _pose_matrix_f32(kf)
    p = np.asarray(p3w, np.float32)
    pc = np.stack([((R[r, 0] * p[:, 0] + R[r, 1] * p[:, 1]) + R[r, 2] * p[:, 2]) + t[r] for r in range(3)], 1)
    return kb8_project(kf.kb8, pc.astype(np.float32))


def pixels_stand_dev(m):
    """Host restatement (tests, oracle side).  Like the reference, nMatches and the mean
    accumulators carry over pairs (:454-456 divide the running sums in place), the squared sums do
    not, and the values of the last pair are returned (0 when the map has fewer than two KFs)."""
    order = m.kf_order()
    n_matches = 0
    mean1 = np.zeros(2); mean2 = np.zeros(2)
    out = {"avgc1": 0.0, "avgc2": 0.0, "desvc1": 0.0, "desvc2": 0.0}
    for a in range(len(order)):
        for b in range(a + 1, len(order)):
            kf1, kf2 = m.keyframes[order[b]], m.keyframes[order[a]]
            p1s, p2s, o1s, o2s = [], [], [], []
            for i in range(min(kf1.n_slots, kf2.n_slots)):
                mp1, mp2 = kf1.map_points[i], kf2.map_points[i]
                if mp1 is None or mp2 is None:
                    continue
                i1 = m.is_map_point_in_keyframe(mp1.id, kf1.id)
                i2 = m.is_map_point_in_keyframe(mp2.id, kf2.id)
                if i1 < 0 or i2 < 0:
                    continue
                p1s.append(mp1.position); p2s.append(mp2.position)
                o1s.append(kf1.keypoints[i1]); o2s.append(kf2.keypoints[i2])
            err1 = np.zeros((0, 2)); err2 = np.zeros((0, 2))
            if p1s:
                uv1 = _project_h(kf1, np.array(p1s)).astype(np.float64)
                uv2 = _project_h(kf2, np.array(p2s)).astype(np.float64)
                err1 = np.abs(np.array(o1s, np.float64) - uv1)
                err2 = np.abs(np.array(o2s, np.float64) - uv2)
            n_matches += len(p1s)
            with np.errstate(invalid="ignore", divide="ignore"):
                mean1 = (mean1 + err1.sum(0)) / n_matches
                mean2 = (mean2 + err2.sum(0)) / n_matches
                sd1 = np.sqrt((err1 ** 2).sum(0) / n_matches)
                sd2 = np.sqrt((err2 ** 2).sum(0) / n_matches)
            out = {
                "avgc1": (mean1[0] + mean1[1]) / 2.0, "avgc2": (mean2[0] + mean2[1]) / 2.0,
                "desvc1": (sd1[0] + sd1[1]) / 2.0, "desvc2": (sd2[0] + sd2[1]) / 2.0,
            }
    out["avg"] = (out["avgc1"] + out["avgc2"]) / 2.0
    out["desv"] = (out["desvc1"] + out["desvc2"]) / 2.0
    return out


def apply_solution(m, prob_graph_ids, points):
    """Write solver output points (f64, graph point order) back into a Map as fp32 positions.
    prob_graph_ids: MapPoint id of each graph point (GraphResult order)."""
    for pid, p in zip(prob_graph_ids, points):
        m.map_points[int(pid)].position = np.asarray(p, np.float32)


def measureSimAbsoluteMapErrors(pMap, originalPoints, movedPoints, device=0):
    """Modules/Utils/Measurements.cc:8-98 on the device: {"average_movement", "average_error",
    "rmse", ...} in mm (the Experiment.txt figures)."""
    from . import capi
    return capi.measure_sim_absolute(pMap, originalPoints, movedPoints, device)


def measureRelativeMapErrors(pMap, device=0):
    """Modules/Utils/Measurements.cc:350-518 on the device: per keyframe pair (map order) the
    accumulated "Rel. error", "depthError" and "gloablTError" after that pair."""
    from . import capi
    return capi.measure_relative(pMap, device)
