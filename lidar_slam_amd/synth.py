"""Synthetic 2-D LiDAR room scans (SURVEY.md §8d generator).

The reference has no recorded data (its only data file, ``./data/scan_prop.txt``
read by ``line_detection.py:29``, is not shipped), so every benchmark and test
scan is synthetic.  One scan = one RPLidar revolution seen from a robot pose
inside a 4000 x 3000 mm rectangular room:

* pose: x, y uniform with an 800 mm margin, heading uniform on (-pi, pi];
* ``n_beams`` beams at ``theta_k = k * 360 / n_beams`` degrees, RPLidar
  convention (clockwise, 0 = forward), i.e. the angle that
  ``functions.py:59-60`` feeds into ``d*cos(-theta*pi/180 + pi/2)``;
* range = ray-to-wall distance + N(0, 5 mm), 3 % outliers uniform in
  [150, 5000] mm, optional zero-range dropouts.

Everything is seeded by ``np.random.default_rng(1_000_003 * scan_id + cfg)``
so any shard of a batch can be regenerated independently on any rank.
Pure NumPy; works under numpy 1.26 (fixture container) and 2.x.
"""
from __future__ import annotations

import numpy as np

ROOM_W = 4000.0
ROOM_H = 3000.0
MARGIN = 800.0
NOISE_MM = 5.0
OUTLIER_FRAC = 0.03
CHUNK = 100  # functions.py:14 MIN_NEIGHBOORS


def _ray_room(px, py, ang):
    """Distance from (px, py) along direction ``ang`` (rad, CCW from +x) to the
    walls of [0, W] x [0, H]."""
    c = np.cos(ang)
    s = np.sin(ang)
    big = np.full_like(ang, np.inf)
    with np.errstate(divide="ignore", invalid="ignore"):
        tx = np.where(c > 1e-12, (ROOM_W - px) / c, np.where(c < -1e-12, (0.0 - px) / c, big))
        ty = np.where(s > 1e-12, (ROOM_H - py) / s, np.where(s < -1e-12, (0.0 - py) / s, big))
    return np.minimum(tx, ty)


def scan_polar(scan_id: int, n_beams: int = 720, cfg: int = 0, dropout: float = 0.0):
    """Return (theta_deg, dist_mm, pose) for one synthetic revolution."""
    rng = np.random.default_rng(1_000_003 * int(scan_id) + int(cfg))
    px = rng.uniform(MARGIN, ROOM_W - MARGIN)
    py = rng.uniform(MARGIN, ROOM_H - MARGIN)
    heading = -rng.uniform(-np.pi, np.pi)  # uniform on (-pi, pi]
    theta = np.arange(n_beams, dtype=np.float64) * (360.0 / n_beams)
    # beam direction in the world frame: robot heading + (pi/2 - theta_rad)
    world = heading + (np.pi / 2 - np.deg2rad(theta))
    dist = _ray_room(px, py, world) + rng.normal(0.0, NOISE_MM, n_beams)
    out = rng.random(n_beams) < OUTLIER_FRAC
    dist = np.where(out, rng.uniform(150.0, 5000.0, n_beams), dist)
    if dropout > 0.0:
        dist = np.where(rng.random(n_beams) < dropout, 0.0, dist)
    return theta, dist, np.array([px, py, heading])


def scan_polar_at(pose, scan_id: int, n_beams: int = 720, cfg: int = 0):
    """(theta_deg, dist_mm) of one revolution seen from a GIVEN pose (x, y,
    heading): the landmark-map trajectories (``trajectory``).  Same beam model
    and noise as ``scan_polar``, its own seed stream."""
    rng = np.random.default_rng(1_000_003 * int(scan_id) + int(cfg) + 0x5A17)
    px, py, heading = (float(v) for v in pose)
    theta = np.arange(n_beams, dtype=np.float64) * (360.0 / n_beams)
    world = heading + (np.pi / 2 - np.deg2rad(theta))
    dist = _ray_room(px, py, world) + rng.normal(0.0, NOISE_MM, n_beams)
    out = rng.random(n_beams) < OUTLIER_FRAC
    dist = np.where(out, rng.uniform(150.0, 5000.0, n_beams), dist)
    return theta, dist


def trajectory(robot_ids, n_steps: int, u=(2.0, 2.5), dt: float = 0.005, wheel_radius: float = 50.0,
               wheel_base: float = 200.0):
    """True poses [n_steps + 1, R, 3] of R robots driven by wheel speeds u with
    the motion model of UKFMethods.py:17-24 (intended form); start poses as
    ``scan_polar``'s (uniform in the room, 800 mm margin, heading on (-pi, pi])."""
    R = len(robot_ids)
    poses = np.zeros((n_steps + 1, R, 3))
    for i, r in enumerate(robot_ids):
        rng = np.random.default_rng(1_000_003 * int(r) + 77)
        poses[0, i] = (rng.uniform(MARGIN, ROOM_W - MARGIN), rng.uniform(MARGIN, ROOM_H - MARGIN),
                       -rng.uniform(-np.pi, np.pi))
    vl, vr = u
    for k in range(n_steps):
        th = poses[k, :, 2]
        v = wheel_radius / 2.0 * (vl + vr)
        poses[k + 1, :, 0] = poses[k, :, 0] + dt * v * np.cos(th)
        poses[k + 1, :, 1] = poses[k, :, 1] + dt * v * np.sin(th)
        poses[k + 1, :, 2] = th + dt * (wheel_radius / wheel_base) * (vr - vl)
    return poses


def revolutions_at(poses, step: int, robot_ids, n_beams: int = 720):
    """One revolution per robot from its true pose at ``step`` (``trajectory``),
    in the chunked CSR layout of ``make_batch`` (robot r = scan r)."""
    xs, sco, cpo = [], [0], [0]
    sizes = chunk_sizes(n_beams)
    used = int(sum(sizes))
    for i, r in enumerate(robot_ids):
        th, d = scan_polar_at(poses[i], 1_000 * int(r) + int(step), n_beams)
        xs.append(polar_to_xy_ref(th, d)[:used])
        for n in sizes:
            cpo.append(cpo[-1] + n)
        sco.append(sco[-1] + len(sizes))
    return {"xy": np.ascontiguousarray(np.concatenate(xs, axis=0)),
            "scan_chunk_off": np.asarray(sco, dtype=np.int32), "chunk_pt_off": np.asarray(cpo, dtype=np.int32)}


def polar_to_xy_ref(theta_deg, dist):
    """NumPy form of ``functions.py:59-60`` (x = d*cos(-theta*A + pi/2))."""
    a = -np.asarray(theta_deg, dtype=np.float64) * (np.pi / 180) + np.pi / 2
    d = np.asarray(dist, dtype=np.float64)
    return np.stack([d * np.cos(a), d * np.sin(a)], axis=-1)


def chunk_sizes(n_points: int, chunk: int = CHUNK):
    """Chunk sizes ``functions.py:61-76`` emits for one revolution of
    ``n_points`` measures: full chunks of ``chunk`` points, then the remainder
    only if it holds more than 2 points (a remainder of 1-2 points is
    dropped, ``functions.py:71-74``)."""
    sizes = [chunk] * (n_points // chunk)
    rem = n_points % chunk
    if rem > 2:
        sizes.append(rem)
    return sizes


def make_batch(scan_ids, n_beams: int = 720, cfg: int = 0):
    """Cartesian batch in the drop-in layout.

    Returns dict with ``xy`` (P,2) f64 (AoS, points of dropped remainders
    excluded), the raw measures ``theta_deg`` / ``dist_mm`` (P,),
    ``scan_chunk_off`` (S+1) i32, ``chunk_pt_off`` (C+1) i32,
    ``poses`` (S,3).
    """
    xs, ths, ds, poses, sco, cpo = [], [], [], [], [0], [0]
    for s in scan_ids:
        th, d, pose = scan_polar(s, n_beams, cfg)
        xy = polar_to_xy_ref(th, d)
        sizes = chunk_sizes(n_beams)
        used = int(sum(sizes))
        xs.append(xy[:used])
        ths.append(th[:used])
        ds.append(d[:used])
        for n in sizes:
            cpo.append(cpo[-1] + n)
        sco.append(sco[-1] + len(sizes))
        poses.append(pose)
    return {
        "xy": np.ascontiguousarray(np.concatenate(xs, axis=0)),
        "theta_deg": np.concatenate(ths),
        "dist_mm": np.concatenate(ds),
        "scan_chunk_off": np.asarray(sco, dtype=np.int32),
        "chunk_pt_off": np.asarray(cpo, dtype=np.int32),
        "poses": np.asarray(poses),
    }


def express_packets(n_packets: int, per_rev: float = 22.5, seed: int = 0, corrupt: float = 0.0,
                    scan_id: int | None = None):
    """A synthetic RPLidar express stream (lidar.py:59-91 layout), uint8 [M, 84].

    Start angles advance 360/per_rev degrees per packet (jittered) and wrap once
    per revolution, so a revolution holds ~32*per_rev measures (720 at the
    default 22.5).  Cabin bytes are random unless ``scan_id`` is given, in which
    case the 10-bit-shifted distances follow ``scan_polar(scan_id)``'s ranges.
    A fraction ``corrupt`` of the packets gets a broken checksum or sync nibble.
    """
    rng = np.random.default_rng(7_000_003 * seed + 11)
    M = int(n_packets)
    pk = rng.integers(0, 256, (M, 84), dtype=np.uint8)
    step = 360.0 / per_rev
    jit = 0.1 * min(step, 360.0 - step)
    ang = (rng.uniform(0, step) + step * np.arange(M) + rng.uniform(-jit, jit, M)) % 360.0
    q6 = (np.floor(ang * 64).astype(np.int64)) % (360 * 64)
    pk[:, 2] = q6 & 0xFF
    pk[:, 3] = ((q6 >> 8) & 0x7F) | np.where(rng.random(M) < 0.02, 0x80, 0)
    if scan_id is not None:
        _, d, _ = scan_polar(scan_id, n_beams=max(M * 32, 1))
        dq = np.clip(np.round(d[:M * 32]), 0, (1 << 14) - 1).astype(np.int64).reshape(M, 16, 2)
        i = 5 * np.arange(16)
        for h, (lo, hi) in enumerate(((4, 5), (6, 7))):
            keep = pk[:, i + lo] & 3  # the angle-offset bits share the low byte
            pk[:, i + lo] = ((dq[:, :, h] & 0x3F) << 2).astype(np.uint8) | keep
            pk[:, i + hi] = (dq[:, :, h] >> 6).astype(np.uint8)
    cs = np.bitwise_xor.reduce(pk[:, 2:], axis=1)
    pk[:, 0] = 0xA0 | (cs & 0x0F)
    pk[:, 1] = 0x50 | (cs >> 4)
    if corrupt > 0:
        bad = np.nonzero(rng.random(M) < corrupt)[0]
        kind = rng.integers(0, 3, bad.size)
        pk[bad[kind == 0], 0] ^= 0x40          # sync nibble
        pk[bad[kind == 1], 1] ^= 0x01          # checksum nibble
        pk[bad[kind == 2], 40] ^= 0x08         # payload byte
    return pk
