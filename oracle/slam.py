"""ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of the landmark-map
step (``LSLAM_UKF_MAP``, lidar_slam_amd/slam.py).

Per robot and revolution, in the order the device runs it:

1. UKF predict with u (oracle/ukf.py: filterpy 1.4.5 + UKFMethods.py intent);
2. per chunk: ``landmark_extraction``'s ransac and line (oracle/cpu.py, C
   restatement of skimage 0.18.3 + ransac_functions.py:23-31, chained
   numpy-legacy stream), the line moved into the world frame of the predicted
   pose (p_w = R(th) p + t, direction rotated, a = u_y/u_x, b = p_y - a p_x as
   ransac_functions.py:26-27), the association walk of ransac_functions.py:34-54
   on the robot's map (``or_associate``);
3. UKF update with the matched chunks only: z = range/bearing of the foot of
   the matched landmark's pos (seen from the predicted pose) on the chunk's
   fitted line, against ``hx`` (UKFMethods.py:26-34) of that pos, R = the
   slots' diagonal; dense filterpy update
   (np.linalg.inv of S) — the device uses the rank-7 Woodbury form, so this
   is an independent check of the masking.

The map glue is this build's own (the reference never wrote it), so beyond the
pieces above it is parity-unpinned; with the pose held at 0 and no filter
steps it reduces exactly to the reference's check_ransac over the revolution,
which tests/test_map_oracle.py pins against the golden live run.
"""
from __future__ import annotations

import math

import numpy as np

from . import cpu
from . import ukf as oukf


def to_world(m, x):
    c, s = math.cos(x[2]), math.sin(x[2])
    px = (c * m["ox"] - s * m["oy"]) + x[0]
    py = (s * m["ox"] + c * m["oy"]) + x[1]
    ex = (c * m["tip_x"] - s * m["tip_y"]) + x[0]
    ey = (s * m["tip_x"] + c * m["tip_y"]) + x[1]
    ux = c * m["ux"] - s * m["uy"]
    uy = s * m["ux"] + c * m["uy"]
    with np.errstate(divide="ignore", invalid="ignore"):
        a = float(np.float64(uy) / np.float64(ux))
    b = py - a * px
    return {"a": a, "b": b, "pos": (px, py), "end": (ex, ey)}


def observe_point(m, pw, x):
    """Range/bearing (robot frame) of the foot of map point pw, seen from pose x,
    on the chunk's fitted line o + t u (the measurement of a matched chunk)."""
    c, s = math.cos(x[2]), math.sin(x[2])
    dx, dy = pw[0] - x[0], pw[1] - x[1]
    qx = c * dx + s * dy
    qy = c * dy - s * dx
    t = (qx - m["ox"]) * m["ux"] + (qy - m["oy"]) * m["uy"]
    fx = m["ox"] + t * m["ux"]
    fy = m["oy"] + t * m["uy"]
    return math.sqrt(fx * fx + fy * fy), math.atan2(fy, fx)


class RobotState:
    def __init__(self, seed, x0=None, P0=None, cap=256):
        self.st = cpu.MTState(seed=int(seed))
        self.lst = []
        self.x = np.zeros(3) if x0 is None else np.array(x0, np.float64)
        self.P = np.diag([.1, .1, .05]) if P0 is None else np.array(P0, np.float64).reshape(3, 3)
        self.cap = cap
        self.id_next = 0


def map_step(rs: RobotState, xy, cpo, u, R_diag, predict=True, update=True, thr=20.0, trials=100, dt=oukf.DT):
    """One revolution (chunks cpo[k]:cpo[k+1] of xy) for one robot.
    Returns (mask, models list)."""
    x, P = rs.x.copy(), rs.P.copy()
    f = oukf.UKF(1, dt=dt)
    f.x, f.P = x, P
    if predict:
        f.predict(np.asarray(u, np.float64))
    else:
        f.sigmas_f = f.points.sigma_points(f.x, f.P)
    xp = f.x.copy()
    masks, models, meas = [], [], []
    for k in range(len(cpo) - 1):
        p0, p1 = cpo[k], cpo[k + 1]
        m, mod, _ = cpu.ransac(xy[p0:p1], thr, trials, state=rs.st)
        mod["landmark_id"] = rs.id_next + k
        mod["match_index"] = -1
        if mod["flags"] & cpu.FLAG_VALID:
            w = to_world(mod, xp)
            F = dict(w, id=rs.id_next + k)
            mi, matched, rs.lst = cpu.associate(rs.lst, F, rs.cap)
            mod["match_index"] = mi
            mod["flags"] |= cpu.FLAG_MATCHED if mi >= 0 else cpu.FLAG_NEW_LANDMARK
            if mi >= 0:
                meas.append((k, observe_point(mod, matched["pos"], xp), matched["pos"]))
        masks.append(m)
        models.append(mod)
    rs.id_next += len(cpo) - 1
    if update and meas:
        slots = [k for k, _, _ in meas]
        Rd = np.concatenate([[R_diag[2 * k], R_diag[2 * k + 1]] for k in slots])
        f.R = np.diag(Rd)
        z = np.concatenate([np.array(zz) for _, zz, _ in meas])
        f.update(z, [tuple(p) for _, _, p in meas])
    rs.x, rs.P = f.x, f.P
    return (np.concatenate(masks) if masks else np.zeros(0, np.uint8)), models
