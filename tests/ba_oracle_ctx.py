"""TEST INFRASTRUCTURE ONLY: an object with the BAContext interface whose methods run the CPU
oracle (oracle/ba_oracle.c).  Lets the parity tests drive the reference control flow of
deftri/ba.py (bundleAdjustment / localBundleAdjustment / poseOnlyOptimization) once on the device
and once on the oracle, then compare."""
import numpy as np

from oracle import oracle


class OracleBA:
    def upload(self, prob):
        self.prob = prob
        self.poses = prob.poses.copy()
        self.points = prob.points.copy()
        self.err = np.zeros((prob.n_edges, 2))
        self.level = prob.edge_level.copy()
        self.robust = prob.edge_robust.copy()

    def set_state(self, poses=None, points=None):
        if poses is not None:
            self.poses = np.array(poses, np.float64).reshape(-1, 7).copy()
        if points is not None:
            self.points = np.array(points, np.float64).reshape(-1, 3).copy()

    def set_edge_flags(self, level=None, robust=None):
        if level is not None:
            self.level = np.array(level, np.uint8)
        if robust is not None:
            self.robust = np.array(robust, np.uint8)

    def solve_lm(self, n_iterations=10, level=0, **kw):
        r = oracle.ba_solve(self.prob, n_iterations, level=level, edge_level=self.level, edge_robust=self.robust,
                            poses=self.poses, points=self.points, err=self.err, **kw)
        self.poses, self.points, self.err = r["poses"], r["points"], r["err"]
        return r["report"]

    def compute_errors(self, mask=None):
        fresh = oracle.ba_compute_errors(self.prob, self.poses, self.points)
        if mask is None:
            self.err = fresh
        else:
            m = np.asarray(mask, bool)
            self.err = np.where(m[:, None], fresh, self.err)

    def edge_chi2(self):
        return oracle.ba_edge_chi2(self.prob, self.poses, self.points, self.err)

    def download(self):
        return self.poses.copy(), self.points.copy()
