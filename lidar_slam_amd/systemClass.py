"""Drop-in for ``systemClass.py`` (which does not parse in the reference, F3):
the System it was written to build, with the UKF step on the GPU.

Constants and configuration are systemClass.py:7-29's: LANDMARK_NUMBER = 8,
VAR_DIST = 0.5**2, VAR_ANGLE = 0.3**2, DT = 0.005,
MerweScaledSigmaPoints(n=3, alpha=1e-4, beta=2, kappa=0), x = the robot's pose,
P = diag(.1, .1, .05), R = diag([VAR_DIST, VAR_ANGLE] * LANDMARK_NUMBER),
Q = 1e-3 * I.  The pose holder the reference imports from robot.py (robot.py:5-14:
a zero [x, y, theta] vector and its length) is ``PoseHolder`` below.
"""
import numpy as np

from .ukf import UnscentedKalmanFilter

LANDMARK_NUMBER = 8   # systemClass.py:7
VAR_DIST = 0.5 ** 2   # systemClass.py:8
VAR_ANGLE = 0.3 ** 2  # systemClass.py:9
DT = 0.005            # systemClass.py:10
POSE_DIM = 3          # [x, y, theta] (robot.py:6-7)


class PoseHolder:
    """The planar pose the filter starts from.  ``get_dim_x`` / ``get_pos`` are the two
    calls systemClass.py:21,34 makes on the reference's robot object."""

    def __init__(self, pose=None):
        self.pose = np.zeros(POSE_DIM) if pose is None else np.asarray(pose, np.float64).reshape(POSE_DIM)

    def get_dim_x(self):
        return self.pose.size

    def get_pos(self):
        return self.pose


class System():

    def __init__(self, landmarks, device=0):
        self.robot = PoseHolder()
        self.dt = DT
        self.varDist = VAR_DIST
        self.varAngle = VAR_ANGLE
        self.landmarks = landmarks
        self.ukf = UnscentedKalmanFilter(dim_x=self.robot.get_dim_x(), dim_z=2 * LANDMARK_NUMBER, dt=DT,
                                         alpha=0.0001, beta=2, kappa=0, device=device)
        self.config_ukf()

    def config_ukf(self):
        self.ukf.x = self.robot.get_pos()
        self.ukf.P = np.diag([.1, .1, 0.05])
        self.ukf.R = np.diag([self.varDist, self.varAngle] * LANDMARK_NUMBER)
        self.ukf.Q = np.eye(3) * 0.001
