"""graph_ref.py — TEST INFRASTRUCTURE ONLY (parity checker).

Python restatement of the graph construction inside the reference's `arapOptimization`
(Modules/Optimization/g2oBundleAdjustment.cc:608-957), producing the flattened problem that the
product's C++ builder (csrc/graph_builder.cpp) must reproduce index-for-index.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.

Followed, line by line:
  pair loop (pKF1 = k2->second, pKF2 = k1->second)              g2oBundleAdjustment.cc:640-651
  extractPositions (drops null slots -> compaction)              Modules/Utils/Geometry.cc:258-270
  ComputeDelaunayTriangulation3D: qhull "d Qbb Qt" on (x, y)      Geometry.cc:317-368
     -> here scipy.spatial.Delaunay (the same qhull library); lower-Delaunay facets only
        (upper-Delaunay facets fail qhull's default Delaunay threshold, i.e. isGood() is false;
        their triangles_ slots stay default-constructed in the reference — treated as absent,
        DESIGN.md §4); T = facets.count() = lower + upper facet count
  Open3D ComputeAdjacencyList / GetEdgeToVerticesMap / GetSurfaceArea (restated)
  ComputeEdgeWeightsCot(mesh, 0)                                  Geometry.cc:272-298
  createVectorMap (first isApprox(1e-6) match)                    Geometry.cc:300-315
  computeR (per-vertex SVD Procrustes, det fix)                   Geometry.cc:549-604
  vertex / edge insertion and the slot/position index quirk       g2oBundleAdjustment.cc:701-953
Simulation fix: depth = per-index simulated depth (KeyFrame.cc:123-125).
"""
import numpy as np
from scipy.spatial import ConvexHull, Delaunay, cKDTree


def _quat_from_mat(m):
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0:
        t = np.sqrt(t + 1.0); w = 0.5 * t; t = 0.5 / t
        return np.array([(m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t, w])
    i = 0
    if m[1, 1] > m[0, 0]:
        i = 1
    if m[2, 2] > m[i, i]:
        i = 2
    j, k = (i + 1) % 3, (i + 2) % 3
    c = np.zeros(3)
    t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
    c[i] = 0.5 * t; t = 0.5 / t
    w = (m[k, j] - m[j, k]) * t
    c[j] = (m[j, i] + m[i, j]) * t; c[k] = (m[k, i] + m[i, k]) * t
    return np.array([c[0], c[1], c[2], w])


def _mat_from_quat(q):
    x, y, z, w = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]])


def delaunay_mesh(pos):
    """Lower-Delaunay triangles of pos[:, :2] (qhull) and the reference's facet count T."""
    n = len(pos)
    if n < 3:
        raise ValueError("Not enough points to create a triangular mesh.")   # Geometry.cc:321-324
    xy = pos[:, :2]
    tri = Delaunay(xy).simplices.astype(np.int64)
    lifted = np.c_[xy, (xy * xy).sum(1)]
    T = len(ConvexHull(lifted).simplices)          # facets.count(): lower + upper
    return tri, T


def create_vector_map(pos, precision=1e-6):
    """createVectorMap(vertices = pos, positions = pos): vertex k -> first isApprox match."""
    n = len(pos)
    out = np.arange(n)
    tree = cKDTree(pos)
    nrm2 = (pos * pos).sum(1)
    for k in range(n):
        r = precision * np.sqrt(nrm2[k]) * 1.0000001 + 1e-300
        cand = sorted(tree.query_ball_point(pos[k], r))
        for p in cand:
            if p > k:
                break
            d2 = ((pos[k] - pos[p]) ** 2).sum()
            if d2 <= precision * precision * min(nrm2[k], nrm2[p]):
                out[k] = p
                break
    return out


def mesh_structures(pos, tri):
    n = len(pos)
    adj = [set() for _ in range(n)]
    e2v = {}
    for t in tri:
        a, b, c = int(t[0]), int(t[1]), int(t[2])
        for (u, v) in ((a, b), (a, c), (b, a), (b, c), (c, a), (c, b)):
            adj[u].add(v)
        for (u, v, o) in ((a, b, c), (b, c, a), (c, a, b)):
            e2v.setdefault((min(u, v), max(u, v)), []).append(o)
    w = {}
    for e, opp in e2v.items():
        s = 0.0
        for o in opp:
            a = pos[e[0]] - pos[o]; b = pos[e[1]] - pos[o]
            s += a.dot(b) / np.linalg.norm(np.cross(a, b))
        wt = s / len(opp) if opp else 0.0
        w[e] = wt if wt >= 0.0 else 0.0
    area = 0.0
    for t in tri:
        x = pos[t[0]] - pos[t[1]]; y = pos[t[0]] - pos[t[2]]
        area += 0.5 * np.linalg.norm(np.cross(x, y))
    return adj, w, area


def eigen_jacobi_svd3(M):
    """Eigen::JacobiSVD<Matrix3d>(M, ComputeFullU|ComputeFullV) — two-sided Jacobi sweep
    (real_2x2_jacobi_svd, JacobiRotation::makeJacobi), precision 2*eps, sign fix, descending
    selection sort.  Returns U, s, V with M = U diag(s) V^T."""
    eps = np.finfo(np.float64).eps
    tiny = np.finfo(np.float64).tiny
    precision = 2.0 * eps
    scale = float(np.abs(M).max())
    if scale == 0.0:
        scale = 1.0
    W = [[float(M[i][j]) / scale for j in range(3)] for i in range(3)]
    U = [[1.0 if i == j else 0.0 for j in range(3)] for i in range(3)]
    V = [[1.0 if i == j else 0.0 for j in range(3)] for i in range(3)]

    def left(A, p, q, c, s):
        for i in range(3):
            x, y = A[p][i], A[q][i]
            A[p][i] = c * x + s * y
            A[q][i] = -s * x + c * y

    def right(A, p, q, c, s):            # applyOnTheRight(p, q, (c, s)) uses the transpose (c, -s)
        tc, ts = c, -s
        for i in range(3):
            x, y = A[i][p], A[i][q]
            A[i][p] = tc * x + ts * y
            A[i][q] = -ts * x + tc * y

    maxd = max(abs(W[0][0]), abs(W[1][1]), abs(W[2][2]))
    finished = False
    guard = 0
    while not finished and guard < 1000:
        guard += 1
        finished = True
        for p in (1, 2):
            for q in range(p):
                thr = max(tiny, precision * maxd)
                if abs(W[p][q]) > thr or abs(W[q][p]) > thr:
                    finished = False
                    m00, m01, m10, m11 = W[p][p], W[p][q], W[q][p], W[q][q]
                    t = m00 + m11
                    d = m10 - m01
                    if abs(d) < tiny:
                        r1s, r1c = 0.0, 1.0
                    else:
                        u = t / d
                        tmp = np.sqrt(1.0 + u * u)
                        r1s, r1c = 1.0 / tmp, u / tmp
                    a0, a1 = r1c * m00 + r1s * m10, r1c * m01 + r1s * m11
                    b0, b1 = -r1s * m00 + r1c * m10, -r1s * m01 + r1c * m11
                    m00, m01, m10, m11 = a0, a1, b0, b1
                    deno = 2.0 * abs(m01)
                    if deno < tiny:
                        jc, js = 1.0, 0.0
                    else:
                        tau = (m00 - m11) / deno
                        ww = np.sqrt(tau * tau + 1.0)
                        tt = 1.0 / (tau + ww) if tau > 0 else 1.0 / (tau - ww)
                        sign_t = 1.0 if tt > 0 else -1.0
                        n = 1.0 / np.sqrt(tt * tt + 1.0)
                        js = -sign_t * (m01 / abs(m01)) * abs(tt) * n
                        jc = n
                    ltc, lts = jc, -js                       # j_right.transpose()
                    lc = r1c * ltc - r1s * lts               # rot1 * j_right^T
                    ls = r1c * lts + r1s * ltc
                    left(W, p, q, lc, ls)
                    right(U, p, q, lc, -ls)
                    right(W, p, q, jc, js)
                    right(V, p, q, jc, js)
                    maxd = max(maxd, abs(W[p][p]), abs(W[q][q]))
    s = [0.0, 0.0, 0.0]
    for i in range(3):
        a = W[i][i]
        s[i] = abs(a)
        if a < 0:
            for r in range(3):
                U[r][i] = -U[r][i]
    s = [v * scale for v in s]
    for i in range(3):
        pos, mx = i, s[i]
        for k in range(i + 1, 3):
            if s[k] > mx:
                mx, pos = s[k], k
        if mx == 0.0:
            break
        if pos != i:
            s[i], s[pos] = s[pos], s[i]
            for r in range(3):
                U[r][i], U[r][pos] = U[r][pos], U[r][i]
                V[r][i], V[r][pos] = V[r][pos], V[r][i]
    return np.array(U), np.array(s), np.array(V)


def _det3(M):
    h = lambda a, b, c: M[0][a] * (M[1][b] * M[2][c] - M[1][c] * M[2][b])
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1)


def procrustes(S):
    U, s, V = eigen_jacobi_svd3(S)
    R = np.array([[sum(V[i][k] * U[j][k] for k in range(3)) for j in range(3)] for i in range(3)])
    if _det3(R) < 0:
        U = U.copy(); U[:, 2] *= -1
        R = np.array([[sum(V[i][k] * U[j][k] for k in range(3)) for j in range(3)] for i in range(3)])
    return _mat_from_quat(_quat_from_mat(R))            # Sophus::SO3d keeps a quaternion


def compute_R(pos1, pos2, adj, w, posIdx):
    n = len(pos1)
    inv = {}
    for v in range(n):
        inv[int(posIdx[v])] = v
    Rs = np.tile(np.eye(3), (n, 1, 1))
    for p in range(n):
        if p not in inv:
            continue
        i = inv[p]
        S = np.zeros((3, 3))
        for j in sorted(adj[i]):
            wt = w[(min(i, j), max(i, j))]
            e1 = pos1[posIdx[i]] - pos1[posIdx[j]]
            e2 = pos2[posIdx[i]] - pos2[posIdx[j]]
            for r in range(3):
                for c in range(3):
                    S[r, c] += wt * e1[r] * e2[c]
        Rs[i] = procrustes(S)
    return Rs


def build_arap_graph(m, rep_weight, arap_weight, depth_error, mesh_override=None):
    """Returns (Problem-kwargs dict, info dict).  `m` is a deftri.mapmodel.Map."""
    order = m.kf_order()
    kfs = [m.keyframes[k] for k in order]
    cams, cam_index = [], {}
    def cam_of(kf):
        if kf.id not in cam_index:
            cam_index[kf.id] = len(cams)
            cams.append(kf)
        return cam_index[kf.id]
    point_vid = {}               # MapPoint id -> point index (first-encounter order)
    point_pos = []
    def add_point(mp):
        if mp.id not in point_vid:
            point_vid[mp.id] = len(point_pos)
            point_pos.append(mp.position.astype(np.float64))
        return point_vid[mp.id]
    tg, scales, scale_kf = [], [], []
    rep_point, rep_cam, rep_obs, rep_info = [], [], [], []
    dep_point, dep_scale, dep_cam, dep_meas, dep_info = [], [], [], [], []
    arap_pts, arap_pair, arap_rot, arap_w = [], [], [], []
    rot_tables, pair_area, pair_info = [], [], []
    rot_base = 0
    info_dep = 1.0 / (float(np.float32(depth_error)) * float(np.float32(depth_error)))
    order_xy = []
    vertex_ids = []             # reference currId order: ('T',q) ('s',k) ('p', point index)
    for a in range(len(kfs)):
        for b in range(a + 1, len(kfs)):
            kf1, kf2 = kfs[b], kfs[a]                 # pKF1 = k2->second, pKF2 = k1->second
            q = len(tg)
            v1 = kf1.map_points; v2 = kf2.map_points
            pos1 = np.array([mp.position.astype(np.float64) for mp in v1 if mp is not None])
            pos2 = np.array([mp.position.astype(np.float64) for mp in v2 if mp is not None])
            if mesh_override is not None:
                tri, T = mesh_override(pos1)
            else:
                tri, T = delaunay_mesh(pos1)
            adj, w, area = mesh_structures(pos1, tri)
            Tg = m.get_global_T(kf1.id, kf2.id)
            Tg7 = Tg.as7()
            if np.linalg.norm(Tg.t.astype(np.float32)) == 0 and np.allclose(Tg.R, np.eye(3), atol=1e-5):
                Tg7 = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
            posIdx = create_vector_map(pos1)
            inv = {}
            for vtx in range(len(pos1)):
                inv[int(posIdx[vtx])] = vtx
            Rs = compute_R(pos1, pos2, adj, w, posIdx)
            rot_tables.append(Rs)
            tg.append(Tg7); vertex_ids.append(("T", q))
            s1 = len(scales); scales.append(kf1.estimated_depth_scale); scale_kf.append(kf1.id)
            vertex_ids.append(("s", s1))
            s2 = len(scales); scales.append(kf2.estimated_depth_scale); scale_kf.append(kf2.id)
            vertex_ids.append(("s", s2))
            c1, c2 = cam_of(kf1), cam_of(kf2)
            pair_area.append(area)
            pair_info.append(arap_weight * float(T) ** 2)
            for mpIndex in range(len(v1)):
                mp1, mp2 = v1[mpIndex], v2[mpIndex]
                if mp1 is None or mp2 is None:
                    continue
                for mp in (mp1, mp2):
                    if mp.id not in point_vid:
                        add_point(mp); vertex_ids.append(("p", point_vid[mp.id]))
                        order_xy.append(None)
                i1 = m.is_map_point_in_keyframe(mp1.id, kf1.id)
                i2 = m.is_map_point_in_keyframe(mp2.id, kf2.id)
                if i1 < 0 or i2 < 0:
                    continue
                p1, p2 = point_vid[mp1.id], point_vid[mp2.id]
                for (pp, kf, idx, cam, sc) in ((p1, kf1, i1, c1, s1), (p2, kf2, i2, c2, s2)):
                    rep_point.append(pp); rep_cam.append(cam)
                    rep_obs.append(kf.keypoints[idx].astype(np.float64))
                    rep_info.append(float(kf.inv_sigma2[kf.octaves[idx]]) * rep_weight)
                for (pp, kf, idx, cam, sc) in ((p1, kf1, i1, c1, s1), (p2, kf2, i2, c2, s2)):
                    dep_point.append(pp); dep_scale.append(sc); dep_cam.append(cam)
                    dep_meas.append(float(kf.depth[idx])); dep_info.append(info_dep)
                if mpIndex not in inv:                 # slot index used as a position index
                    continue
                i = inv[mpIndex]
                if not adj[i]:
                    continue
                for j in sorted(adj[i]):
                    slot = int(posIdx[j])              # position index used as a slot index
                    mpj1, mpj2 = v1[slot], v2[slot]
                    if mpj1 is None or mpj2 is None:
                        continue
                    for mp in (mpj1, mpj2):
                        if mp.id not in point_vid:
                            add_point(mp); vertex_ids.append(("p", point_vid[mp.id]))
                            order_xy.append(None)
                    arap_pts.append((p1, p2, point_vid[mpj1.id], point_vid[mpj2.id]))
                    arap_pair.append(q)
                    arap_rot.append((rot_base + i, rot_base + j))
                    arap_w.append(w[(min(i, j), max(i, j))])
            rot_base += len(pos1)
    P = len(point_pos)
    cam_kb8 = np.array([c.kb8 for c in cams], np.float32)
    cam_pose = np.array([c.pose.as7() for c in cams])
    prob = dict(
        points=np.array(point_pos).reshape(-1, 3), tg=np.array(tg).reshape(-1, 7),
        scales=np.array(scales, np.float64), cam_kb8=cam_kb8, cam_pose=cam_pose,
        rep_point=np.array(rep_point, np.int32), rep_cam=np.array(rep_cam, np.int32),
        rep_obs=np.array(rep_obs).reshape(-1, 2), rep_info=np.array(rep_info),
        dep_point=np.array(dep_point, np.int32), dep_scale=np.array(dep_scale, np.int32),
        dep_cam=np.array(dep_cam, np.int32), dep_meas=np.array(dep_meas), dep_info=np.array(dep_info),
        arap_pts=np.array(arap_pts, np.int32).reshape(-1, 4), arap_pair=np.array(arap_pair, np.int32),
        arap_rot=np.array(arap_rot, np.int32).reshape(-1, 2), arap_w=np.array(arap_w),
        rot=np.concatenate(rot_tables).reshape(-1, 3, 3) if rot_tables else np.zeros((0, 3, 3)),
        pair_area=np.array(pair_area), pair_info=np.array(pair_info),
        huber_delta=float(np.float32(np.sqrt(100.991))),
    )
    info = {"vertex_ids": vertex_ids, "point_ids": {v: k for k, v in point_vid.items()},
            "scale_kf": scale_kf, "kf_order": order}
    return prob, info
