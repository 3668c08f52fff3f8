"""ORACLE — TEST INFRASTRUCTURE ONLY.  NumPy twin of the reference CPU path.

Restates, with the reference's per-trial NumPy structure (and therefore its
CPU cost profile), what ``ransac_functions.landmark_extraction``
(ransac_functions.py:15-59) does through scikit-image 0.18.3:
``ransac`` (fit.py:581-881) with ``LineModelND.estimate/residuals``
(fit.py:66-132) on numpy's global legacy RandomState, then the association
walk (ransac_functions.py:34-54, landmarking.py:48-77).  The reference's
Python cannot travel to the GPU box, so bench.py times THIS twin there as the
``cpu_baseline`` ("port"), on a bounded sample of the benchmark's scans.
The twin is checked against the golden vectors in tests/test_numpy_twin.py.
"""
from __future__ import annotations

import numpy as np

THRESHOLD, MAX_TRIALS, MIN_SAMPLES = 20, 100, 2   # ransac_functions.py:9-11
LIFE, TOL_A, TOL_B, TOL = 40, 0.1, 10, 100         # landmarking.py:3-6


class LineModelND:
    def __init__(self):
        self.params = None

    def estimate(self, data):
        origin = data.mean(axis=0)
        data = data - origin
        if data.shape[0] == 2:
            direction = data[1] - data[0]
            norm = np.linalg.norm(direction)
            if norm != 0:
                direction /= norm
        elif data.shape[0] > 2:
            _, _, v = np.linalg.svd(data, full_matrices=False)
            direction = v[0]
        else:
            raise ValueError("At least 2 input points needed.")
        self.params = (origin, direction)
        return True

    def residuals(self, data):
        origin, direction = self.params
        res = (data - origin) - ((data - origin) @ direction)[..., np.newaxis] * direction
        return np.sqrt(np.einsum("ij,ij->i", res, res))


def ransac(data, min_samples=2, residual_threshold=20, max_trials=100, random_state=None):
    rs = random_state if random_state is not None else np.random.mtrand._rand
    best_model, best_num, best_sum, best_inliers = None, 0, np.inf, None
    n = len(data)
    if not (0 < min_samples < n):
        raise ValueError("`min_samples` must be in range (0, <number-of-samples>)")
    idx = rs.choice(n, min_samples, replace=False)
    for t in range(max_trials):
        samples = data[idx]
        idx = rs.choice(n, min_samples, replace=False)
        m = LineModelND()
        m.estimate(samples)
        r = np.abs(m.residuals(data))
        inl = r < residual_threshold
        s = np.sum(r ** 2)
        c = np.sum(inl)
        if c > best_num or (c == best_num and s < best_sum):
            best_model, best_num, best_sum, best_inliers = m, c, s, inl
            if best_sum <= 0:
                break
    if best_inliers is not None and any(best_inliers):
        best_model.estimate(data[best_inliers])
    else:
        best_model, best_inliers = None, None
    return best_model, best_inliers


class Landmark:
    def __init__(self, a, b, ID, x, y, tipX, tipY):
        self.a, self.b, self.id, self.life = a, b, ID, LIFE
        self.pos = np.array([x, y])
        self.end = np.array([tipX, tipY])

    def decrease_life(self):
        if self.life > 0:
            self.life -= 1
        if self.life == 0:
            return True

    def is_equal(self, o):
        distA = abs(self.a - o.a)
        distB = abs(self.b - o.b)
        dEO = np.linalg.norm(self.end - o.pos)
        dOE = np.linalg.norm(self.pos - o.end)
        if distA <= TOL_A and distB <= TOL_B:
            return dEO <= TOL or dOE <= TOL
        return False


def landmark_extraction(data, landmark_number, landmarks, random_state=None):
    model, inliers = ransac(data, MIN_SAMPLES, THRESHOLD, MAX_TRIALS, random_state)
    params = model.params
    a = params[1][1] / params[1][0]
    b = params[0][1] - a * params[0][0]
    x_base = np.array(data[inliers, 0])
    tip_x = x_base[-1]
    fitted = Landmark(a, b, landmark_number, params[0][0], params[0][1], tip_x, tip_x * a + b)
    i, equal = 0, False
    if len(landmarks) > 0:
        while i < len(landmarks) and not equal:
            equal = landmarks[i].is_equal(fitted)
            if not equal:
                if landmarks[i].decrease_life():
                    landmarks.remove(landmarks[i])
            i += 1
        if equal:
            landmarks[i - 1].life = LIFE
            y_base = landmarks[i - 1].a * x_base + landmarks[i - 1].b
            new = False
        else:
            y_base = a * x_base + b
            new = True
    else:
        y_base = a * x_base + b
        new = True
    return (x_base, y_base), fitted, new, inliers


def process_scan(xy, chunk_pt_off, seed):
    """check_ransac over one scan's chunks (per-scan seed, fresh landmark list)."""
    rs = np.random.RandomState(int(seed))
    landmarks = []
    masks = []
    for k in range(len(chunk_pt_off) - 1):
        data = xy[chunk_pt_off[k]:chunk_pt_off[k + 1]]
        _, fitted, new, inl = landmark_extraction(data, k, landmarks, rs)
        if new:
            landmarks.append(fitted)
        masks.append(inl)
    return masks, landmarks
