"""Drop-in for ``landmarking.py``: the Landmark value object callers hold.

The hot path never calls these methods (the association walk of
ransac_functions.py:34-54 runs on the GPU, lslam_landmarks / the scan kernel's
post pass); the class is here so that code holding the reference's Landmark
objects (check_ransac's list, mainWindow's plots) keeps its attribute and method
surface: a, b, id, life, pos, end, timesObserved, spec and the accessors of
landmarking.py:12-64, with the association semantics of landmarking.py:48-77
(life floored at 0, ``is_equal`` with the three tolerances).  The reference's
``landmarks_track`` (landmarking.py:79-82) is not provided: it is never called
and, comparing a bound method with 0, never removes anything.
"""
from __future__ import annotations

import numpy as np

LIFE = 40          # landmarking.py:3
TOLERANCE_A = 0.1  # landmarking.py:4
TOLERANCE_B = 10   # landmarking.py:5
TOLERANCE = 100    # landmarking.py:6


def _gap(p, q):
    """Euclidean distance as numpy's norm computes it for 2-vectors (the reference uses np.linalg.norm)."""
    return np.linalg.norm(np.asarray(p, np.float64) - np.asarray(q, np.float64))


class Landmark():
    spec = "line"

    def __init__(self, a, b, ID, x, y, tipX, tipY):
        self.a, self.b, self.id = a, b, ID
        self.pos = np.array([x, y])        # the fitted origin (inlier centroid)
        self.end = np.array([tipX, tipY])  # the last inlier's x on the fitted line
        self.life = LIFE
        self.timesObserved = 0

    def __str__(self):
        x, y = self.pos
        return "Landmark ID: {}\n(x, y): ({}, {})\nequation: {} * x + {}\n".format(self.id, x, y, self.a, self.b)

    # accessors the reference's callers use
    def get_id(self):
        return self.id

    def get_a(self):
        return self.a

    def get_b(self):
        return self.b

    def get_pos(self):
        return self.pos

    def get_end(self):
        return self.end

    def get_life(self):
        return self.life

    def observed(self):
        self.timesObserved += 1

    def reset_life(self):
        self.life = LIFE

    def decrease_life(self):
        """One unmatched association pass: life floors at 0; True once it is 0, else None
        (the caller removes the landmark on True, ransac_functions.py:39-41)."""
        if self.life > 0:
            self.life -= 1
        return True if self.life == 0 else None

    def distance_end_origin(self, other):
        return _gap(self.end, other.get_pos())

    def distance_origin_end(self, other):
        return _gap(self.pos, other.get_end())

    def is_equal(self, other):
        """Same line (slope within TOLERANCE_A, intercept within TOLERANCE_B) and the two
        segments continue each other (one's end within TOLERANCE of the other's origin)."""
        same_line = abs(self.a - other.get_a()) <= TOLERANCE_A and abs(self.b - other.get_b()) <= TOLERANCE_B
        if not same_line:  # (NaN slopes of vertical fits never match)
            return False
        return bool(self.distance_end_origin(other) <= TOLERANCE or self.distance_origin_end(other) <= TOLERANCE)
