"""lidar_slam_amd — MI355X-native per-scan hot path of Farofeiro231/LiDAR_SLAM.

RANSAC line/landmark extraction (ransac_functions.py / landmarking.py, with
scikit-image 0.18.3 ``ransac``/``LineModelND`` semantics and numpy's legacy
MT19937 stream) and the intended UKF predict/update (UKFMethods.py /
systemClass.py with filterpy semantics), as hand-written HIP kernels for
gfx950 behind a C ABI (include/lidarslam.h) loaded with ctypes.

Drop-in modules mirror the reference's call surface:
  lidar_slam_amd.ransac_functions  landmark_extraction / check_ransac
  lidar_slam_amd.landmarking       Landmark
  lidar_slam_amd.systemClass       System (.ukf.predict / .ukf.update)
  lidar_slam_amd.functions         polar->Cartesian + chunking of a revolution
Batched API: lidar_slam_amd.pipeline.ScanPipeline.
"""
__version__ = "0.1.0"
