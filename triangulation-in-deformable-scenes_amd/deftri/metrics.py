"""Reprojection metric of the reference: calculatePixelsStandDev (Modules/Utils/Geometry.cc:370-498).

This is the parity metric of the north star ("final reprojection RMSE"): per camera the RMS of
|obs - KB8(T p)| in u and v, averaged: desvc = (RMS_u + RMS_v) / 2 and desv = (desvc1 + desvc2) / 2.
The "variance" is the mean of squares (no mean subtraction, :449-480).  Projection is fp32 with the
homogeneous T.matrix() product, as in the reference.  Like the reference, nMatches accumulates over
all pairs and the per-camera values of the last pair are reported.
"""
import numpy as np

from .sim import kb8_project


def _project_h(kf, p3w):
    """T1w.matrix() * [p;1] in fp32, then KB8 project (Geometry.cc:423-431)."""
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = kf.pose.R
    T[:3, 3] = kf.pose.t
    ph = np.concatenate([p3w.astype(np.float32), np.ones((len(p3w), 1), np.float32)], 1)
    pc = (ph @ T.T)[:, :3].astype(np.float32)
    return kb8_project(kf.kb8, pc)


def pixels_stand_dev(m):
    order = m.kf_order()
    n_matches = 0
    out = None
    for a in range(len(order)):
        for b in range(a + 1, len(order)):
            kf1, kf2 = m.keyframes[order[b]], m.keyframes[order[a]]
            e1, e2 = [], []
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
            if not p1s:
                continue
            uv1 = _project_h(kf1, np.array(p1s)).astype(np.float64)
            uv2 = _project_h(kf2, np.array(p2s)).astype(np.float64)
            err1 = np.abs(np.array(o1s, np.float64) - uv1)
            err2 = np.abs(np.array(o2s, np.float64) - uv2)
            n_matches += len(p1s)
            mean1 = err1.sum(0) / n_matches
            mean2 = err2.sum(0) / n_matches
            var1 = (err1 ** 2).sum(0) / n_matches
            var2 = (err2 ** 2).sum(0) / n_matches
            sd1, sd2 = np.sqrt(var1), np.sqrt(var2)
            out = {
                "avgc1": (mean1[0] + mean1[1]) / 2.0, "avgc2": (mean2[0] + mean2[1]) / 2.0,
                "desvc1": (sd1[0] + sd1[1]) / 2.0, "desvc2": (sd2[0] + sd2[1]) / 2.0,
            }
    if out is None:
        return {"avgc1": 0.0, "avgc2": 0.0, "avg": 0.0, "desvc1": 0.0, "desvc2": 0.0, "desv": 0.0}
    out["avg"] = (out["avgc1"] + out["avgc2"]) / 2.0
    out["desv"] = (out["desvc1"] + out["desvc2"]) / 2.0
    return out


def apply_solution(m, prob_graph_ids, points):
    """Write solver output points (f64, graph point order) back into a Map as fp32 positions.
    prob_graph_ids: MapPoint id of each graph point (GraphResult order)."""
    for pid, p in zip(prob_graph_ids, points):
        m.map_points[int(pid)].position = np.asarray(p, np.float32)
