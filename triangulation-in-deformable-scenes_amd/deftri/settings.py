"""Settings — the solver-relevant subset of the reference's cv::FileStorage YAML reader
(Modules/System/Settings.cc:27-190).  Missing numeric keys read as 0 (as cv::FileNode does),
missing strings as "".  `validate_for_solver()` rejects the one value that makes the reference's
depth information infinite (Measurements.DepthWeight absent -> sigma_d = 0).
"""
import re

NUMERIC = {
    "Camera.fx": "fx", "Camera.fy": "fy", "Camera.cx": "cx", "Camera.cy": "cy",
    "Camera.d0": "k0", "Camera.d1": "k1", "Camera.d2": "k2", "Camera.d3": "k3",
    "Camera.cols": "cols", "Camera.rows": "rows",
    "FeatureExtractor.nScales": "n_scales", "FeatureExtractor.fScaleFactor": "scale_factor",
    "Camera.FirstPose.x": "c1x", "Camera.FirstPose.y": "c1y", "Camera.FirstPose.z": "c1z",
    "Camera.SecondPose.x": "c2x", "Camera.SecondPose.y": "c2y", "Camera.SecondPose.z": "c2z",
    "Keypoints.RepError": "rep_error", "Keypoints.decimalsApproximation": "decimals",
    "Measurements.DepthError": "depth_error", "Measurements.DepthWeight": "depth_weight",
    "Measurements.DepthScale.C1": "depth_scale_c1", "Measurements.DepthScale.C2": "depth_scale_c2",
    "Optimization.rep": "rep", "Optimization.arap": "arap", "Optimization.global": "global_",
    "Optimization.alpha": "alpha", "Optimization.beta": "beta",
    "Optimization.numberOfOptimizations": "n_optimizations",
    "Optimization.numberOfIterations": "n_iterations",
    "Optimization.nlopt.numberOfIterations": "nlopt_iterations",
    "Optimization.nlopt.relTolerance": "nlopt_rel_tol", "Optimization.nlopt.absTolerance": "nlopt_abs_tol",
    "Optimization.nlopt.rep.lowerBound": "nlopt_rep_lb", "Optimization.nlopt.rep.upperBound": "nlopt_rep_ub",
    "Optimization.nlopt.global.lowerBound": "nlopt_global_lb", "Optimization.nlopt.global.upperBound": "nlopt_global_ub",
    "Optimization.nlopt.arap.lowerBound": "nlopt_arap_lb", "Optimization.nlopt.arap.upperBound": "nlopt_arap_ub",
    "Triangulation.minCos": "min_cos",
}
STRINGS = {
    "Optimization.selection": "selection", "Optimization.weightsSelection": "weights_selection",
    "Triangulation.method": "trian_method", "Triangulation.seed.location": "trian_location",
    "Experiment.Filepath": "exp_file",
}


def parse_yaml_subset(text):
    out = {}
    for line in text.splitlines():
        line = line.split("#", 1)[0].strip()
        if not line or line.startswith("%") or ":" not in line:
            continue
        k, v = line.split(":", 1)
        v = v.strip()
        if v.startswith('"') and v.endswith('"'):
            v = v[1:-1]
        out[k.strip()] = v
    return out


class Settings:
    def __init__(self, text=None, path=None):
        if path is not None:
            with open(path) as f:
                text = f.read()
        kv = parse_yaml_subset(text or "")
        for key, attr in NUMERIC.items():
            v = kv.get(key)
            try:
                setattr(self, attr, float(v) if v is not None and re.match(r"^[-+0-9.eE]+$", v) else 0.0)
            except ValueError:
                setattr(self, attr, 0.0)
        for key, attr in STRINGS.items():
            setattr(self, attr, kv.get(key, ""))
        self.n_scales = int(self.n_scales)
        self.n_optimizations = int(self.n_optimizations)
        self.n_iterations = int(self.n_iterations)

    @property
    def depth_sigma(self):
        """SimulatedDepthErrorStanDesv = DepthWeight / 1000 (float), g2oBundleAdjustment.cc:449."""
        import numpy as np
        return np.float32(np.float32(self.depth_weight) / np.float32(1000.0))

    def validate_for_solver(self):
        if self.depth_weight == 0.0:
            raise ValueError("Measurements.DepthWeight is missing/0: depth information 1/sigma^2 would be "
                             "infinite (reference Settings.cc:124, g2oBundleAdjustment.cc:823-824)")
        return True
