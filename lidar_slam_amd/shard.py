"""One batch of scans split across the GPUs of a node, and the per-scan results
gathered back (65,536 scans over 8 MI355X).

This replaces the reference's hand-off of scan chunks between its capture and
RANSAC processes through one ``multiprocessing.Queue`` (SLAM.py:13,18-23).  The
scans are independent (per-scan seeds and landmark lists), so the split is a
partition and the only communication is moving inputs in and results out:

* ``shard_range``: rank r owns the contiguous scans [lo, hi) (sizes differ by at
  most one).  Its chunks and points follow from the CSR offsets, which every
  rank holds (they are small), so every rank knows every shard's byte counts.
* ``Shard.inputs``: the rank's slice of a host batch with the CSR rebased to 0.
* ``gather``: each result field of the shards (mask per point, chunk records,
  UKF x / P, landmark counts and lists per scan) goes to the root in rank order,
  which IS batch order: the gathered arrays equal a single-GPU run's bit for bit.
  The transport is a ``gatherv(send, recv, counts, root)`` callable: RCCL over
  xGMI on the GPUs (lidar_slam_amd.collective), or gloo on CPU for the tests.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .pipeline import LANDMARK_DTYPE, MODEL_DTYPE


def shard_range(n_scans: int, world: int, rank: int):
    """Contiguous, balanced: the first n_scans % world ranks hold one more scan."""
    base, extra = divmod(int(n_scans), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


# per-scan inputs (first axis = scans); the names ScanPipeline / bench.py's C4 leg use
PER_SCAN = frozenset(("seeds", "poses", "mt_state", "id_base", "landmarks", "lmk_count",
                      "ukf_x", "ukf_P", "ukf_u", "ukf_z", "ukf_lmk", "x", "P", "u", "z", "lmk"))


@dataclass
class Shard:
    rank: int
    lo: int      # scans [lo, hi)
    hi: int
    c0: int      # chunks [c0, c1)
    c1: int
    p0: int      # points [p0, p1)
    p1: int

    @property
    def n_scans(self):
        return self.hi - self.lo

    def inputs(self, batch):
        """The shard's slice of a host batch: xy / theta / dist by points, CSR rebased,
        the per-scan arrays named in ``PER_SCAN`` (seeds, poses, MT states, UKF inputs, landmark
        lists) by scans; every other entry (e.g. ``ukf_R_diag``, whose length 2L may equal the
        scan count) unchanged."""
        sco, cpo = batch["scan_chunk_off"], batch["chunk_pt_off"]
        out = {}
        for k, v in batch.items():
            if k == "scan_chunk_off":
                out[k] = (sco[self.lo:self.hi + 1] - self.c0).astype(np.int32)
            elif k == "chunk_pt_off":
                out[k] = (cpo[self.c0:self.c1 + 1] - self.p0).astype(np.int32)
            elif k in ("xy", "theta_deg", "dist_mm"):
                out[k] = v[self.p0:self.p1]
            elif k in PER_SCAN:
                if v.shape[0] != len(sco) - 1:
                    raise ValueError("per-scan input %r has %d rows for %d scans" % (k, v.shape[0], len(sco) - 1))
                out[k] = v[self.lo:self.hi]
            else:
                out[k] = v
        return out

    def field_bytes(self, lmk_capacity=0):
        """Bytes of each gathered result field for this shard."""
        S = self.n_scans
        f = {"mask": self.p1 - self.p0, "models": (self.c1 - self.c0) * MODEL_DTYPE.itemsize,
             "ukf_x": S * 24, "ukf_P": S * 72}
        if lmk_capacity:
            f["lmk_count"] = S * 4
            f["landmarks"] = S * lmk_capacity * LANDMARK_DTYPE.itemsize
        return f


def plan(scan_chunk_off, chunk_pt_off, world):
    """Every rank's Shard (the same list on every rank)."""
    sco = np.asarray(scan_chunk_off)
    cpo = np.asarray(chunk_pt_off)
    out = []
    for r in range(world):
        lo, hi = shard_range(len(sco) - 1, world, r)
        c0, c1 = int(sco[lo]), int(sco[hi])
        out.append(Shard(r, lo, hi, c0, c1, int(cpo[c0]), int(cpo[c1])))
    return out


FIELDS = ("mask", "models", "ukf_x", "ukf_P", "lmk_count", "landmarks")
DTYPES = {"mask": np.uint8, "models": MODEL_DTYPE, "ukf_x": np.float64, "ukf_P": np.float64, "lmk_count": np.int32,
          "landmarks": LANDMARK_DTYPE}


def gather(shards, rank, local, gatherv, alloc, root=0, lmk_capacity=0):
    """Gather the fields present in ``local`` (name -> this rank's buffer) to ``root``.

    gatherv(send, recv, counts_bytes, root) moves each rank's ``counts_bytes[r]`` bytes of
    ``send`` into ``recv`` at offset sum(counts_bytes[:r]) on the root (recv is None
    elsewhere); alloc(field, nbytes) makes the root's receive buffer.  Returns
    {field: recv buffer} on the root, {} elsewhere."""
    out = {}
    for name in FIELDS:
        if name not in local:
            continue
        counts = [s.field_bytes(lmk_capacity)[name] for s in shards]
        recv = alloc(name, sum(counts)) if rank == root else None
        gatherv(local[name], recv, counts, root)
        if rank == root:
            out[name] = recv
    return out


def host_view(name, raw, n_scans, lmk_capacity=0):
    """A gathered field's bytes as the single-GPU result array."""
    a = np.frombuffer(raw, DTYPES[name]) if not isinstance(raw, np.ndarray) else raw.view(DTYPES[name]).ravel()
    if name == "ukf_x":
        return a.reshape(n_scans, 3)
    if name == "ukf_P":
        return a.reshape(n_scans, 3, 3)
    if name == "landmarks":
        return a.reshape(n_scans, lmk_capacity)
    return a
