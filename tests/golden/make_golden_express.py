"""Golden vectors for the RPLidar express-scan codec FROM THE REFERENCE.

Run ONLY in the build container with the interpreter that imports the
reference:

    /opt/conda/bin/python3.9 tests/golden/make_golden_express.py

It imports ``/root/reference/lidar.py`` unmodified.  pyserial is absent here and
only the serial-port methods use it, so ``serial`` is stubbed by an empty
module.  Recorded, for a synthetic stream of 84-byte express packets:
  * ``ExpressPacket.decode`` (lidar.py:59-91) per packet: 32 distances, 32
    angle corrections, new_scan, start_angle, or the ValueError it raises
    (bad sync nibbles / bad checksum);
  * the measure stream ``Lidar.scan('express')`` yields (lidar.py:327-338,
    179-187): for each packet p with a successor, 32 (new_scan, angle,
    distance) computed by ``Lidar._process_express_scan`` from p and the next
    packet's start_angle.
  * the capture loop ``functions.scanning(rawPoints)`` (functions.py:47-81,
    unmodified; ``mainWindow`` stubbed as in make_golden.py) run over a
    stand-in ``Lidar`` whose ``scan('express')`` yields exactly the measure
    stream above, with ``time.time`` faked so that the first ``drop``
    measures fall inside the 1-second warm-up: every ``rawPoints.put`` (a
    chunk of [dX, dY] or the revolution delimiter 0) is recorded.
Output: tests/golden/express.npz (plain arrays, no pickles).
"""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import blaspin  # noqa: E402  (pins OPENBLAS_CORETYPE; must precede numpy)
import numpy as np  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("LSLAM_GOLDEN_OUT", HERE)  # the dispatch census writes elsewhere
sys.path.insert(0, REF)
sys.modules["serial"] = types.ModuleType("serial")  # only the port methods use it

import lidar  # noqa: E402  (reference, unmodified)

_stub = types.ModuleType("mainWindow")  # mainWindow.py needs the absent PyQt5.QtChart
_stub.time = __import__("time")
_stub.ploting = lambda *a, **k: None
sys.modules["mainWindow"] = _stub
import functions  # noqa: E402  (reference, unmodified)


def make_packets(n_rev=3, per_rev=24, seed=7):
    """A plausible express stream: start angles advance ~360/per_rev per
    packet with jitter and wrap once per revolution; payload bytes random."""
    rng = np.random.default_rng(seed)
    pk = []
    ang = rng.uniform(0, 10)
    for p in range(n_rev * per_rev + 1):
        b = bytearray(rng.integers(0, 256, 84, dtype=np.uint8).tobytes())
        q6 = int(round(ang * 64)) % (360 * 64)
        b[2] = q6 & 0xFF
        b[3] = ((q6 >> 8) & 0x7F) | (0x80 if rng.random() < 0.05 else 0)
        cs = 0
        for x in b[2:]:
            cs ^= x
        b[0] = 0xA0 | (cs & 0x0F)
        b[1] = 0x50 | (cs >> 4)
        pk.append(bytes(b))
        ang = (ang + 360.0 / per_rev + rng.uniform(-0.3, 0.3)) % 360.0
    # edge angles: exactly 0 and the largest start angle, and a wrap to 0
    return pk


def make_revolutions(rev_packets, seed):
    """Clean packets whose start angles wrap after exactly rev_packets[r]
    packets per revolution (the first and last revolutions are open)."""
    rng = np.random.default_rng(seed)
    pk = []
    for k in rev_packets:
        for i in range(k):
            b = bytearray(rng.integers(0, 256, 84, dtype=np.uint8).tobytes())
            q6 = int((i + rng.uniform(0.05, 0.6)) * 360 * 64 / k) % (360 * 64)
            b[2] = q6 & 0xFF
            b[3] = ((q6 >> 8) & 0x7F) | (0x80 if rng.random() < 0.05 else 0)
            cs = 0
            for x in b[2:]:
                cs ^= x
            b[0] = 0xA0 | (cs & 0x0F)
            b[1] = 0x50 | (cs >> 4)
            pk.append(bytes(b))
    return pk


class _Queue:
    def __init__(self):
        self.items = []

    def put(self, x):
        self.items.append(x)


def capture(stream, drop):
    """functions.scanning over a stand-in Lidar yielding the reference's
    measure stream of `stream`; the first `drop` measures are warm-up."""
    dec = [lidar.ExpressPacket.decode(raw) for raw in stream]
    L = object.__new__(lidar.Lidar)

    class FakeLidar:
        def __init__(self, port):
            pass

        def scan(self, scan_type, max_buf_meas=False, speed=0):
            for p in range(len(dec) - 1):
                for t in range(1, 33):
                    yield L._process_express_scan(dec[p], dec[p + 1].start_angle, t), 0.0

    clock = {"n": -1}

    def fake_time():  # call 0 = start_time; call i >= 1 = measure i-1
        clock["n"] += 1
        return 0.0 if clock["n"] <= drop else 2.0

    q = _Queue()
    saved = functions.Lidar, functions.time
    functions.Lidar = FakeLidar
    functions.time = types.SimpleNamespace(time=fake_time)
    try:
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            functions.scanning(q)
    finally:
        functions.Lidar, functions.time = saved
    # flatten: xy of every chunk, chunk sizes, and after how many chunks each 0 came
    xy, sizes, delim = [], [], []
    for it in q.items:
        if isinstance(it, int) and it == 0:
            delim.append(len(sizes))
        else:
            a = np.asarray(it, np.float64).reshape(-1, 2)
            xy.append(a)
            sizes.append(len(a))
    xy = np.concatenate(xy) if xy else np.zeros((0, 2))
    return dict(packets=np.frombuffer(b"".join(stream), np.uint8).reshape(len(stream), 84),
                drop=np.int32(drop), xy=xy, chunk_sizes=np.array(sizes, np.int32), delim=np.array(delim, np.int32))


def corrupt(pk, rng):
    out = list(pk)
    bad = {}
    for idx, kind in ((5, "sync1"), (11, "sync2"), (17, "checksum"), (23, "checksum_hi")):
        b = bytearray(out[idx])
        if kind == "sync1":
            b[0] = (b[0] & 0x0F) | 0xB0
        elif kind == "sync2":
            b[1] = (b[1] & 0x0F) | 0x40
        elif kind == "checksum":
            b[40] ^= 0x10
        else:
            b[1] ^= 0x01
        out[idx] = bytes(b)
        bad[idx] = kind
    return out, bad


def main():
    rng = np.random.default_rng(11)
    clean = make_packets()
    dirty, bad = corrupt(clean, rng)
    recs = {}
    for name, stream in (("clean", clean), ("dirty", dirty)):
        M = len(stream)
        valid = np.zeros(M, np.uint8)
        dist = np.zeros((M, 32), np.int64)
        corr = np.zeros((M, 32), np.float64)
        nsf = np.zeros(M, np.uint8)
        start = np.zeros(M, np.float64)
        decoded = []
        for p, raw in enumerate(stream):
            try:
                e = lidar.ExpressPacket.decode(raw)
            except ValueError:
                decoded.append(None)
                continue
            valid[p] = 1
            dist[p] = e.distance
            corr[p] = e.angle
            nsf[p] = e.new_scan
            start[p] = e.start_angle
            decoded.append(e)
        # the measure stream: packet p's 32 measures need packets p and p+1 decoded
        L = object.__new__(lidar.Lidar)
        m_ok = np.zeros((M - 1, 32), np.uint8)
        m_new = np.zeros((M - 1, 32), np.uint8)
        m_ang = np.zeros((M - 1, 32), np.float64)
        m_dist = np.zeros((M - 1, 32), np.int64)
        for p in range(M - 1):
            if decoded[p] is None or decoded[p + 1] is None:
                continue
            for t in range(1, 33):
                ns, q, a, d = L._process_express_scan(decoded[p], decoded[p + 1].start_angle, t)
                m_ok[p, t - 1] = 1
                m_new[p, t - 1] = ns
                m_ang[p, t - 1] = a
                m_dist[p, t - 1] = d
        recs[name] = dict(packets=np.frombuffer(b"".join(stream), np.uint8).reshape(M, 84), valid=valid,
                          dist=dist, corr=corr, new_scan_bit=nsf, start=start, m_ok=m_ok, m_new=m_new,
                          m_ang=m_ang, m_dist=m_dist)
    flat = {}
    for name, r in recs.items():
        for k, v in r.items():
            flat["%s_%s" % (name, k)] = v
    flat["bad_index"] = np.array(sorted(bad), np.int32)
    # capture loop: (A) first revolution of 289 - 88 = 201 points (remainder 1
    # dropped), a 1-packet revolution, an 800-point one; (B) 161 - 59 = 102
    # (remainder 2 dropped), a 2-packet revolution, a 3-packet one
    caps = {"capA": capture(make_revolutions([10, 23, 1, 25, 22, 7], 5), 88),
            "capB": capture(make_revolutions([6, 2, 3, 24, 21, 4], 6), 59)}
    for name, r in caps.items():
        for k, v in r.items():
            flat["%s_%s" % (name, k)] = v
    blaspin.save_npz(os.path.join(OUT, "express.npz"), **flat)
    print("express.npz:", {k: v.shape for k, v in flat.items()})


if __name__ == "__main__":
    main()
