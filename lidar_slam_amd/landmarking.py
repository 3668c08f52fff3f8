"""Drop-in for ``landmarking.py`` (the reference's Landmark value object).

Same class, constants, method names and semantics as landmarking.py:1-82.  The
association walk of the hot path runs on the GPU (lslam_landmarks / the fused
scan kernel); these methods remain for callers that use a Landmark directly.
"""
from __future__ import annotations

import numpy as np

LIFE = 40          # landmarking.py:3
TOLERANCE_A = 0.1  # landmarking.py:4
TOLERANCE_B = 10   # landmarking.py:5
TOLERANCE = 100    # landmarking.py:6


class Landmark():
    spec = "line"

    def __init__(self, a, b, ID, x, y, tipX, tipY):
        self.a = a
        self.b = b
        self.id = ID
        self.life = LIFE
        self.pos = np.array([x, y])
        self.end = np.array([tipX, tipY])
        self.timesObserved = 0

    def __str__(self):
        return ("Landmark ID: {}\n".format(self.id)
                + "(x, y): ({}, {})\n".format(self.pos[0], self.pos[1])
                + "equation: {} * x + {}\n".format(self.a, self.b))

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

    def decrease_life(self):
        """landmarking.py:48-52: floor at 0; True once it reaches 0, else None."""
        if self.life > 0:
            self.life -= 1
        if self.life == 0:
            return True

    def reset_life(self):
        self.life = LIFE

    def distance_end_origin(self, landmark):
        return np.linalg.norm(self.end - landmark.get_pos())

    def distance_origin_end(self, landmark):
        return np.linalg.norm(self.pos - landmark.get_end())

    def is_equal(self, landmark):
        """landmarking.py:66-77."""
        distA = abs(self.a - landmark.get_a())
        distB = abs(self.b - landmark.get_b())
        dEO = self.distance_end_origin(landmark)
        dOE = self.distance_origin_end(landmark)
        if distA <= TOLERANCE_A and distB <= TOLERANCE_B:
            return bool(dEO <= TOLERANCE or dOE <= TOLERANCE)
        return False


def landmarks_track(landmarks):
    """landmarking.py:79-82, kept with the reference's behaviour: it compares
    the bound method ``get_life`` (not its value) with 0, so it never removes
    anything."""
    for landmark in landmarks:
        if landmark.get_life == 0:  # noqa: reference bug reproduced on purpose
            landmarks.remove(landmark)
