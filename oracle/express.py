"""ORACLE - TEST INFRASTRUCTURE ONLY (never imported by lidar_slam_amd/).

NumPy restatement of the RPLidar express-scan codec the reference uses
(SURVEY §8f rank 2), vectorised over packets:

  * lidar.py:55-59   twos_comp(val, bits): val - 2^bits if bit (bits-1) is set
                     (no masking: values with higher bits set pass through)
  * lidar.py:59-91   ExpressPacket.decode: sync nibbles 0xA / 0x5, XOR checksum
                     of bytes 2..83 == (b0 & 0xF) + ((b1 & 0xF) << 4),
                     new_scan = b3 >> 7, start_angle = (b2 + ((b3 & 0x7F) << 8)) / 64,
                     per cabin pair k (i = 5k): d1 = (b[i+4] >> 2) + (b[i+5] << 6),
                     a1 = twos_comp((b[i+8] & 0xF) + ((b[i+4] & 3) << 4), 5) / 8,
                     d2 = (b[i+6] >> 2) + (b[i+7] << 6),
                     a2 = twos_comp(((b[i+8] >> 4) & 0xF) + ((b[i+6] & 3) << 4), 5) / 8
  * lidar.py:179-187 Lidar._process_express_scan(data, new_angle, trame):
                     new_scan = new_angle < start and trame == 1,
                     angle = (start + (((new_angle - start) % 360) / 32) * trame
                              - angle[trame - 1]) % 360    (Python float %, floor mod)
  * lidar.py:327-338 the measure stream: packet p's 32 measures use packet
                     p+1's start angle; a packet that fails to decode raises in
                     the reference, so measures touching it are invalid here.

Pinned by tests/golden/express.npz (tests/golden/make_golden_express.py, which
imports the reference's lidar.py).
"""
import numpy as np


def twos_comp(val, bits):
    val = np.asarray(val, np.int64)
    return np.where((val & (1 << (bits - 1))) != 0, val - (1 << bits), val)


def decode_packets(packets):
    """packets: uint8 [M, 84] -> dict(valid, dist [M,32] int, corr [M,32] f64,
    new_scan_bit [M], start [M] f64).  Invalid packets have zeros."""
    b = np.asarray(packets, np.int64).reshape(-1, 84)
    sync = ((b[:, 0] >> 4) == 0xA) & ((b[:, 1] >> 4) == 0x5)
    cs = np.bitwise_xor.reduce(b[:, 2:], axis=1)
    ok = sync & (cs == (b[:, 0] & 0xF) + ((b[:, 1] & 0xF) << 4))
    new_scan = b[:, 3] >> 7
    start = (b[:, 2] + ((b[:, 3] & 0x7F) << 8)) / 64.0
    i = np.arange(0, 80, 5)
    d1 = (b[:, i + 4] >> 2) + (b[:, i + 5] << 6)
    a1 = twos_comp((b[:, i + 8] & 0xF) + ((b[:, i + 4] & 3) << 4), 5) / 8.0
    d2 = (b[:, i + 6] >> 2) + (b[:, i + 7] << 6)
    a2 = twos_comp(((b[:, i + 8] >> 4) & 0xF) + ((b[:, i + 6] & 3) << 4), 5) / 8.0
    dist = np.stack([d1, d2], 2).reshape(-1, 32)
    corr = np.stack([a1, a2], 2).reshape(-1, 32)
    z = ~ok
    dist[z] = 0
    corr[z] = 0.0
    new_scan = np.where(ok, new_scan, 0)
    start = np.where(ok, start, 0.0)
    return dict(valid=ok.astype(np.uint8), dist=dist, corr=corr, new_scan_bit=new_scan.astype(np.uint8), start=start)


def measures(dec):
    """The measure stream of Lidar.scan('express') over a decoded packet array:
    [M-1, 32] ok / new_scan / angle (deg) / distance (int)."""
    v = dec["valid"].astype(bool)
    ok = v[:-1] & v[1:]
    s = dec["start"][:-1, None]
    na = dec["start"][1:, None]
    t = np.arange(1, 33, dtype=np.float64)[None, :]
    ang = np.remainder(s + (np.remainder(na - s, 360.0) / 32.0) * t - dec["corr"][:-1], 360.0)
    new = (na < s) & (t == 1)
    ok2 = np.repeat(ok[:, None], 32, 1)
    return dict(m_ok=ok2.astype(np.uint8), m_new=(new & ok2).astype(np.uint8), m_ang=np.where(ok2, ang, 0.0),
                m_dist=np.where(ok2, dec["dist"][:-1], 0))


def capture(packets, drop=0, chunk=100, min_rem=2):
    """functions.py:47-81 over the measure stream of `packets` (the capture
    loop; the first `drop` measures are the 1-second warm-up of :58).

    Restated as the reference's per-measure state machine: append (dX, dY)
    (:59-63); every `chunk` points put the list (:64-67); on the
    new-revolution flag put the remainder if it has more than `min_rem` points,
    then the delimiter 0 (:68-76).  Measures of packets that fail to decode
    are skipped (the reference raises instead).  Returns dict(xy [P, 2],
    chunk_sizes, delim) in the format of tests/golden/express.npz's cap* keys:
    delim[r] = number of chunks put before revolution r's 0.
    """
    m = measures(decode_packets(packets))
    ok, new, ang, dist = (m[k].ravel() for k in ("m_ok", "m_new", "m_ang", "m_dist"))
    pts, xy, sizes, delim = [], [], [], []
    for i in range(drop, ok.size):
        if not ok[i]:
            continue
        d, a = float(dist[i]), float(ang[i])
        pts.append((d * np.cos(-a * (np.pi / 180) + np.pi / 2), d * np.sin(-a * (np.pi / 180) + np.pi / 2)))
        if len(pts) == chunk:
            xy += pts
            sizes.append(len(pts))
            pts = []
        if new[i]:
            if len(pts) > min_rem:
                xy += pts
                sizes.append(len(pts))
            delim.append(len(sizes))
            pts = []
    return dict(xy=np.array(xy, np.float64).reshape(-1, 2), chunk_sizes=np.array(sizes, np.int32),
                delim=np.array(delim, np.int32))


def revolutions(packets, skip=0):
    """The completed revolutions of `packets` as CSR (what lslam_express_scans
    returns): xy [P, 2], scan_chunk_off [S+1], chunk_pt_off [C+1], and the
    packet holding the last new-revolution flag (-1 if none).  Chunks of the
    open revolution after the last flag are not included."""
    cap = capture(packets, drop=skip)
    S = len(cap["delim"])
    C = int(cap["delim"][-1]) if S else 0
    sizes = cap["chunk_sizes"][:C]
    cpo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    sco = np.concatenate([[0], cap["delim"]]).astype(np.int32)
    m = measures(decode_packets(packets))["m_new"]
    flagged = np.nonzero(m[:, 0])[0]
    flagged = flagged[flagged > 0] if skip else flagged
    resume = int(flagged[-1]) if flagged.size else -1
    return dict(xy=cap["xy"][:cpo[-1]], scan_chunk_off=sco, chunk_pt_off=cpo, resume=resume)
