"""Test helper for the C++ adapter (adapter/): writes a deftri.mapmodel.Map in the binary layout
adapter/test/map_io.h reads, and reads adapter_driver's output back.  Test infrastructure only."""
import struct

import numpy as np

from deftri import mapmodel


def _pose_q(T):
    """The fp32 quaternion (x, y, z, w) the Python model's pose carries (as7's source), or the one a
    test chose to dump for it (q_dump: the C++ model normalizes it into T.q)."""
    if getattr(T, "q_dump", None) is not None:
        return np.asarray(T.q_dump, np.float32)
    if T.q is not None:
        return np.asarray(T.q, np.float32)
    return mapmodel.quat_from_mat(T.R.astype(np.float64)).astype(np.float32)


def write_map(path, m, original=None, moved=None, scale_factor=1.2):
    kids = list(m.keyframes)
    assert kids == list(range(len(kids))), "the model numbers keyframes 0.. in insertion order"
    pids = list(m.map_points)
    assert pids == list(range(len(pids))), "the model numbers map points 0.. in insertion order"
    out = [b"DTMAP001", struct.pack("<i", len(kids))]
    for kid in kids:
        kf = m.keyframes[kid]
        out.append(struct.pack("<q", kf.id))
        out.append(_pose_q(kf.pose).tobytes())
        out.append(np.asarray(kf.pose.t, np.float32).tobytes())
        out.append(np.asarray(kf.kb8, np.float32).tobytes())
        isig = np.asarray(kf.inv_sigma2, np.float32)
        out.append(struct.pack("<if", len(isig), scale_factor))
        out.append(isig.tobytes())
        out.append(struct.pack("<d", float(kf.estimated_depth_scale)))
        n = kf.n_slots
        assert len(kf.keypoints) == n
        out.append(struct.pack("<i", n))
        out.append(np.ascontiguousarray(kf.keypoints, np.float32).tobytes())
        out.append(np.ascontiguousarray(kf.octaves, np.int32).tobytes())
        out.append(np.ascontiguousarray(kf.depth, np.float32).tobytes())
        out.append(np.array([mp.id if mp is not None else -1 for mp in kf.map_points], np.int64).tobytes())
    out.append(struct.pack("<i", len(pids)))
    for pid in pids:
        out.append(struct.pack("<q", pid))
        out.append(np.asarray(m.map_points[pid].position, np.float32).tobytes())
    obs = [(k, mp, idx) for k in kids for mp, idx in m.kf_obs.get(k, {}).items()]
    out.append(struct.pack("<i", len(obs)))
    for o in obs:
        out.append(struct.pack("<qqq", *o))
    gts = [(a, b, T) for (a, b), T in sorted(m.global_T.items()) if a < b]
    out.append(struct.pack("<i", len(gts)))
    for a, b, T in gts:
        out.append(struct.pack("<qq", a, b))
        out.append(_pose_q(T).tobytes())
        out.append(np.asarray(T.t, np.float32).tobytes())
    o = np.zeros((0, 3), np.float32) if original is None else np.asarray(original, np.float32)
    mv = np.zeros((0, 3), np.float32) if moved is None else np.asarray(moved, np.float32)
    out.append(struct.pack("<i", len(o)))
    out.append(o.tobytes())
    out.append(mv.tobytes())
    with open(path, "wb") as f:
        f.write(b"".join(out))


def read_state(path):
    b = open(path, "rb").read()
    assert b[:8] == b"DTOUT001"
    off = 8

    def take(fmt):
        nonlocal off
        v = struct.unpack_from("<" + fmt, b, off)
        off += struct.calcsize("<" + fmt)
        return v

    (nkf,) = take("i")
    kfs = {}
    for _ in range(nkf):
        (kid,) = take("q")
        (scale,) = take("d")
        pose = np.array(take("7d"))
        kfs[kid] = {"depth_scale": scale, "pose": pose}
    (nmp,) = take("i")
    pts, present = {}, {}
    for _ in range(nmp):
        (pid,) = take("q")
        pts[pid] = np.array(take("3f"), np.float32)
        (present[pid],) = take("B")
    g = np.array(take("14d"))
    (nx,) = take("i")
    extra = list(take(f"{nx}d")) if nx else []
    return {"keyframes": kfs, "points": pts, "present": present, "global01": g[:7], "global10": g[7:],
            "extra": extra}
