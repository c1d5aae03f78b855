"""Which step of tests/test_gpu_parity.py::test_degenerate_maps leaves a pending HIP launch error."""
import ctypes, sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "triangulation-in-deformable-scenes_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np
import torch  # noqa
from deftri import capi, optimization
hip = ctypes.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = ctypes.c_char_p
def probe(tag):
    e = hip.hipGetLastError()
    print(tag, e, hip.hipGetErrorString(e).decode(), flush=True)
import test_gpu_parity as T
probe("start")
m1 = T._single_kf_map()
upd = [1.0]
optimization.arapOptimization(m1, 1.0, 50.0, 2e5, 0.0, 0.0, np.float32(0.003), 5, upd)
probe("arapOptimization")
ctx = capi.Context(0)
probe("context")
pe = ctx.pixels_stand_dev(m1)
probe("pixels")
kf = m1.keyframes[0]
x1, x2, v = ctx.triangulate_nrslam(np.zeros((0, 2)), np.zeros((0, 2)), kf.kb8, kf.kb8, kf.pose, kf.pose)
probe("triangulate")
