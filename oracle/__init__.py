"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's hot path, used exclusively as the checker
by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg.  The product package ``lidar_slam_amd`` never imports anything from here;
its HIP path fails loudly if its extension is missing.

* ``oracle.cpu``       ctypes binding of ``ransac_oracle.c`` (plain-C, bit-exact
                       restatement of skimage 0.18.3 ``ransac``/``LineModelND``
                       + numpy legacy MT19937 + ``ransac_functions.py`` /
                       ``landmarking.py``).  Pinned against ``tests/golden``.
* ``oracle.numpy_twin`` NumPy restatement with skimage's per-trial structure
                       (the reference's actual CPU cost; cpu_baseline "port").
* ``oracle.ukf``       NumPy restatement of the intended UKF (UKFMethods.py /
                       systemClass.py + filterpy 1.4.5 semantics).
                       PARITY UNPINNED: the reference UKF does not parse and
                       filterpy is absent; self-pinned by known-answer tests.
"""
