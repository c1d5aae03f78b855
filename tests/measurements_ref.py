"""TEST INFRASTRUCTURE ONLY: host restatement of Modules/Utils/Measurements.cc —
measureSimAbsoluteMapErrors (:8-98; float accumulation in the reference's order) and
measureRelativeMapErrors (:350-518; the oracle's qhull mesh, double accumulation, the reference's
slot / position index quirks; depth from the per-index simulated measurement)."""
import numpy as np

from oracle import graph_ref

f32 = np.float32


def sim_absolute(m, original, moved):
    mps = sorted(m.map_points)
    point_count = len(mps)
    tm = te1 = te2 = te = tsq1 = tsq2 = tsq = f32(0)
    for j in range(point_count // 2):
        p1 = m.map_points[2 * j].position.astype(f32); p2 = m.map_points[2 * j + 1].position.astype(f32)
        o = np.asarray(original[j], f32); mv = np.asarray(moved[j], f32)
        mov = o - mv; e1 = p1 - o; e2 = p2 - mv
        sq = lambda v: f32(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2]))
        n_m, n1, n2 = np.sqrt(sq(mov)), np.sqrt(sq(e1)), np.sqrt(sq(e2))
        tm = f32(tm + n_m); te1 = f32(te1 + n1); te2 = f32(te2 + n2); te = f32(te + f32(n2 + n1))
        tsq1 = f32(tsq1 + sq(e1)); tsq2 = f32(tsq2 + sq(e2)); tsq = f32(tsq + f32(sq(e1) + sq(e2)))
    in_kf = int(point_count / 2.0)
    return {"average_movement": float(f32(tm / f32(in_kf))) * 1000, "average_error_original": float(f32(te1 / f32(in_kf))) * 1000,
            "average_error_moved": float(f32(te2 / f32(in_kf))) * 1000, "average_error": float(f32(te / f32(point_count))) * 1000,
            "rmse": float(np.sqrt(f32(tsq / f32(point_count)))) * 1000, "point_count": point_count}


def _R_f32(T):
    """Sophus so3().matrix() of an SE3f: from its fp32 unit quaternion."""
    q = (T.q if T.q is not None else T.unit_quaternion()).astype(f32)
    x, y, z, w = q
    tx, ty, tz = f32(2) * x, f32(2) * y, f32(2) * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz, tyy, tyz, tzz = tx * x, ty * x, tz * x, ty * y, tz * y, tz * z
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy], [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]], f32)


def relative(m):
    order = m.kf_order()
    depth = glob = meansq = 0.0
    valid = matches = 0
    out = []
    for a in range(len(order)):
        for b in range(a + 1, len(order)):
            kf1, kf2 = m.keyframes[order[b]], m.keyframes[order[a]]
            T = m.get_global_T(kf1.id, kf2.id)
            Rg = _R_f32(T).astype(np.float64); Ts = T.t.astype(f32).astype(np.float64)
            s1, s2 = kf1.estimated_depth_scale, kf2.estimated_depth_scale
            v1 = np.array([mp.position.astype(np.float64) for mp in kf1.map_points if mp is not None])
            v2 = np.array([mp.position.astype(np.float64) for mp in kf2.map_points if mp is not None])
            tri, _ = graph_ref.delaunay_mesh(v1)
            adj, _, area = graph_ref.mesh_structures(v1, tri)
            pos_idx = graph_ref.create_vector_map(v1)
            inv = {int(pos_idx[v]): v for v in range(len(v1))}
            cams = []
            for kf in (kf1, kf2):
                q = kf.pose.as7()[:4]; q = q / np.linalg.norm(q)
                R = graph_ref._mat_from_quat(q)
                cams.append((R, kf.pose.as7()[4:]))
            for i in range(min(kf1.n_slots, kf2.n_slots)):
                mp1, mp2 = kf1.map_points[i], kf2.map_points[i]
                if mp1 is None or mp2 is None:
                    continue
                i1 = m.is_map_point_in_keyframe(mp1.id, kf1.id); i2 = m.is_map_point_in_keyframe(mp2.id, kf2.id)
                if i1 < 0 or i2 < 0:
                    continue
                for (R, t), mp, d, s in ((cams[0], mp1, kf1.depth[i1], s1), (cams[1], mp2, kf2.depth[i2], s2)):
                    zc = (R @ mp.position.astype(np.float64) + t)[2]
                    depth += (float(d) - zc * s) ** 2
                if i >= len(v1) or i not in inv or not adj[inv[i]]:
                    continue
                for j in sorted(adj[inv[i]]):
                    pj = int(pos_idx[j])
                    if i >= len(v2) or pj >= len(v2):
                        continue
                    d1 = v1[i] - v1[pj]; d2 = v2[i] - v2[pj]
                    meansq += float(((d2 - d1) ** 2).sum())
                    valid += 1
                    g = ((Rg @ v2[i] - Ts) - v1[i]) + ((Rg @ v2[pj] - Ts) - v1[pj])
                    glob += float((g * g).sum())
                matches += 1
            out.append({"kf1": kf1.id, "kf2": kf2.id, "reported": int(valid > 1), "rel_error": meansq / area,
                        "depth_error": depth, "global_t_error": glob / area, "area": area, "valid_pairs": valid,
                        "n_matches": matches})
    return out
