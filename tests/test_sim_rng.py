"""The simulation's noise streams are the reference's (SLAM.cc:281-338): libstdc++
std::default_random_engine (minstd_rand0: x <- 16807 x mod 2^31-1, seed 1) driving
std::normal_distribution<float> (Marsaglia polar method on generate_canonical<float, 24> draws,
second value cached).  deftri_sim_normal_stream (the C++ <random> the reference links) against a
pure-Python restatement of libstdc++'s bits/random.tcc, with glibc's logf / sqrtf; and the
create_data.py draw order of the point clouds."""
import ctypes as C
import ctypes.util

import numpy as np

from deftri import capi, sim

_libm = C.CDLL(ctypes.util.find_library("m"))
_libm.logf.restype = C.c_float; _libm.logf.argtypes = [C.c_float]
_libm.sqrtf.restype = C.c_float; _libm.sqrtf.argtypes = [C.c_float]
f32 = np.float32


def libstdcxx_normal_float(n, mean, stddev):
    x = 1                                           # minstd_rand0 default seed
    saved, have = None, False
    out = []

    def canonical():                               # generate_canonical<float, 24>: one engine call
        nonlocal x
        x = (16807 * x) % 2147483647
        s = f32(x - 1)                              # (urng() - min()) as float
        tmp = f32(2147483646.0)                     # float(1) * (max - min + 1): 2^31 - 2 -> 2^31 in float
        r = f32(s / tmp)
        return r if r < f32(1) else np.nextafter(f32(1), f32(0))
    for _ in range(n):
        if have:
            have = False
            v = saved
        else:
            while True:
                u = f32(float(f32(2.0) * canonical()) - 1.0)    # float * float, then - 1.0 in double
                w = f32(float(f32(2.0) * canonical()) - 1.0)
                r2 = f32(f32(u * u) + f32(w * w))
                if not (r2 > 1.0 or r2 == 0.0):
                    break
            mult = f32(_libm.sqrtf(f32(f32(f32(-2) * f32(_libm.logf(r2))) / r2)))
            saved, have = f32(u * mult), True
            v = f32(w * mult)
        out.append(f32(f32(v * f32(stddev)) + f32(mean)))
    return np.array(out, np.float32)


def test_normal_stream_is_libstdcxx():
    lib = capi.load()
    for mean, sd, n in ((0.0, 1.0, 2000), (0.0, 0.003, 500), (0.25, 2.5, 300)):
        got = np.zeros(n, np.float32)
        assert lib.deftri_sim_normal_stream(n, mean, sd, got.ctypes.data_as(C.POINTER(C.c_float))) == 0
        ref = libstdcxx_normal_float(n, mean, sd)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert abs(got.mean() - 0.25) < 0.5 and 1.5 < got.std() < 3.5


def test_two_view_streams_follow_slam_cc():
    """createKeyPoints draws 4 per correspondence (x1, y1, x2, y2), getSimulatedDepthMeasurements 2
    (d1, d2), each from its own fresh engine: the keypoint noise is recovered to the 0.1 px rounding
    and the depth noise to fp32 rounding."""
    orig, moved = sim.generate_points(50, seed=3)
    kb8 = sim.SIM_KB8
    uv1, uv2, d1, d2, q1, q2 = capi.sim_two_view(orig, moved, (-0.1, 0.02, 0.12), (0.14, 0.01, 0.06), kb8, kb8,
                                                 1.0, 1, 3.0, (0.4, 1.7))
    kn = libstdcxx_normal_float(4 * 50, 0.0, 1.0).reshape(50, 4)
    dn = libstdcxx_normal_float(2 * 50, 0.0, 0.003).reshape(50, 2)
    pc1 = orig.astype(np.float32) + np.float32([-0.1, 0.02, 0.12])     # T1w = (I, c1)
    p1 = sim.kb8_project(kb8, pc1)
    assert np.abs(uv1 - (p1 + kn[:, :2])).max() <= 0.05 + 1e-3
    assert np.abs(d1 - (pc1[:, 2] * np.float32(0.4) + dn[:, 0])).max() <= 1e-7
    assert q1.tolist()[:4] == [0.0, 0.0, 0.0, 1.0]
    assert abs(np.linalg.norm(q2[:4]) - 1) < 1e-6


def test_create_data_draw_order():
    """np.random.seed(s) + create_data.generate_points' calls == sim.generate_points(seed=s)."""
    n, g, rig = 40, 0.0025, 0.0025
    rs = np.random.RandomState(7)
    o = np.zeros((n, 3))
    o[:, 0] = rs.normal(0.0, 0.03, n); o[:, 1] = rs.normal(0.0, 0.001, n); o[:, 2] = rs.normal(0.0, 0.01, n)
    mv = o.copy()
    for i in range(n):
        mv[i, 1] += rig
        mv[i, 0] += rs.normal(scale=g); mv[i, 1] += rs.normal(scale=g); mv[i, 2] += rs.normal(scale=g)
    ro = sim.rotate_points(o, -45, 0, 45) + [0, 0, 0.2]
    rm = sim.rotate_points(mv, -45, 0, 45) + [0, 0, 0.2]
    a, b = sim.generate_points(n, rigid=rig, gaussian=g, seed=7, scale_density=False)
    assert np.array_equal(a, ro) and np.array_equal(b, rm)
