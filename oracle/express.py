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
