"""TEST INFRASTRUCTURE ONLY: arapOptimization(pMap, rep, global, arap, alpha, beta, depthError,
nIt) driven by the oracle (oracle/graph_ref.py graph build + oracle/deftri_oracle.c LM) with the
reference's write-back (g2oBundleAdjustment.cc:967-1007: fp32 positions, last scale per KF, T_g to
pair (0, 1), returns sum ||p_old - p_new||).  Lets tests run the outer weight search of
deformationOptimization once on the device and once on the oracle."""
import numpy as np

from deftri.mapmodel import SE3f
from deftri.problem import Problem
from oracle import graph_ref, oracle


def oracle_arap(m, rep, glob, arap, alpha, beta, depth_sigma, n_it):
    kw, info = graph_ref.build_arap_graph(m, rep, arap, depth_sigma)
    prob = Problem(**kw)
    ref = oracle.solve_lm(prob, int(n_it), analytic=False)   # the reference: numeric J
    upd = 0.0
    for k in range(prob.n_points):
        mp = m.map_points[info["point_ids"][k]]
        new = ref["points"][k].astype(np.float32)
        d = (mp.position - new).astype(np.float32)
        upd += float(np.sqrt(np.float32(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])))
        mp.position = new
    for s, kid in enumerate(info["scale_kf"]):
        m.keyframes[kid].estimated_depth_scale = float(ref["scales"][s])
    if prob.n_pairs:
        m.insert_global_from7(0, 1, list(ref["tg"][-1]))      # reference :1007 (KF ids 0, 1)
    return upd
