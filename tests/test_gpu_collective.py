"""The RCCL binding (lidar_slam_amd/collective.py) on one GPU: a one-rank communicator,
a broadcast and the C4 gather of a pipeline call's results (shard.gather over
Comm.gatherv, on the lslam context stream) equal the results read directly.  The
multi-rank exchange runs in bench.py's C4 leg on the driver's 8-GPU node; its
bookkeeping is tested on CPU (tests/test_shard.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


def test_one_rank_comm_broadcast(ctx):
    from lidar_slam_amd import collective
    comm = collective.Comm.from_process_group(ctx, None)
    a = ctx.to_device(np.arange(1000, dtype=np.uint8))
    comm.broadcast(a, 1000, 0)
    ctx.sync()
    assert np.array_equal(a.download(), np.arange(1000, dtype=np.uint8))
    comm.close()


def test_gather_of_pipeline_results_on_the_stream(ctx):
    import bench
    from lidar_slam_amd import collective, shard
    from lidar_slam_amd.device import DeviceArray
    from lidar_slam_amd.pipeline import ScanPipeline
    ids = list(range(512))
    b, wk = bench.make_workload(ids, 720, 20)
    p = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                     lmk_capacity=64, ukf=wk)
    comm = collective.Comm.from_process_group(ctx, None)
    plan = shard.plan(b["scan_chunk_off"], b["chunk_pt_off"], 1)
    local = {"mask": p.mask, "models": p.models, "ukf_x": p.ukf_x, "ukf_P": p.ukf_P, "lmk_count": p.lmk_count}
    recv = {}

    def alloc(k, n):
        recv[k] = DeviceArray(ctx, (n,), np.uint8)
        return recv[k]

    p.run(sync=False)                     # no sync: the gather is ordered after the call on the stream
    shard.gather(plan, 0, local, comm.gatherv, alloc, lmk_capacity=64)
    ctx.sync()
    r = p.results()
    for k in local:
        got = shard.host_view(k, recv[k].download(), len(ids), 64)
        assert got.tobytes() == np.ascontiguousarray(r[k]).tobytes(), k
    comm.close()
