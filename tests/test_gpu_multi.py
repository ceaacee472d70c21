"""Multi-GPU fan-out behind the C ABI (SURVEY.md §8(b) Threading row, §8(e)).

The reference forks 8 std::threads inside renderScene (src/Scene.cpp:294-363); librtg forks one
host thread per GPU inside rtg_render (rtg_render_opts.num_devices) and gathers the row-block
shards over RCCL, or, one process per GPU, through rtg_comm_* + rtg_render_ranked.  On a 1-GPU
box the RCCL path runs with one rank (ncclCommInitAll / ncclCommInitRank over one device, the
rank's rows sent to itself), and the N-shard path runs with the device listed N times (shards
copied instead of sent).  Every frame must equal the single-device frame bit for bit."""
import numpy as np
import pytest

import rtg
from rtg import scenegen

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a).view(np.int32)


@pytest.fixture(scope="module")
def cornell():
    sc = scenegen.cornell(96, 61, spp=6, level=1)
    r = rtg.Renderer(sc, device=0)
    ref = r.render(0)
    st = r.stats()
    yield r, ref, st
    r.close()


def test_one_device_list_renders_without_rccl(gpu, cornell):
    """num_devices = 1 with a device list is the plain single-device render (no communicator, so
    no RCCL library is needed for it)."""
    r, ref, st = cornell
    for _ in range(2):                      # the second call reuses the communicator
        img = r.render(0, num_devices=1, devices=[0])
        assert np.array_equal(_bits(img), _bits(ref))
        s = r.stats()
        assert s["devices"] == 1
        assert s["total_rays"] == st["total_rays"]


@pytest.mark.parametrize("n,block", [(2, 4), (3, 4), (4, 1), (5, 8)])
def test_shards_on_a_repeated_device_are_bit_identical(gpu, cornell, n, block):
    r, ref, st = cornell
    img = r.render(0, num_devices=n, devices=[0] * n, row_block=block)
    assert np.array_equal(_bits(img), _bits(ref))
    s = r.stats()
    assert s["devices"] == n
    assert s["primary_rays"] == st["primary_rays"]
    assert s["total_rays"] == st["total_rays"]


def test_multi_device_render_into_device_memory(gpu, cornell):
    import torch
    r, ref, _ = cornell
    out = torch.full((ref.shape[0], ref.shape[1], 3), float("nan"), dtype=torch.float32, device="cuda:0")
    r.render_device(0, out.data_ptr(), torch.cuda.current_stream().cuda_stream, num_devices=2, devices=[0, 0])
    torch.cuda.synchronize()
    assert np.array_equal(_bits(out.cpu().numpy()), _bits(ref))


def test_num_devices_beyond_the_visible_devices_is_an_error(gpu, lib, cornell):
    r, _, _ = cornell
    n = lib.rtg_device_count()
    with pytest.raises(rtg.RtgError, match="NO_DEVICE|visible"):
        r.render(0, num_devices=n + 1)
    with pytest.raises(rtg.RtgError):
        r.render(0, num_devices=2, devices=[0, n])          # device index out of range
    with pytest.raises(rtg.RtgError):
        r.render(0, num_devices=2, devices=[0, 0], row_stride=2)   # shards are the library's


def test_ranked_single_rank_gathers_through_rccl(gpu, cornell):
    import torch
    r, ref, _ = cornell
    comm = rtg.Comm(rtg.Comm.unique_id(), 1, 0, 0)
    try:
        out = torch.zeros((ref.shape[0], ref.shape[1], 3), dtype=torch.float32, device="cuda:0")
        for _ in range(2):
            r.render_ranked(0, comm, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert np.array_equal(_bits(out.cpu().numpy()), _bits(ref))
        assert r.stats()["devices"] == 1
    finally:
        comm.close()


def test_ranked_rank_failure_is_agreed_not_hung(gpu, cornell):
    """A rank whose shard fails (here: a bad camera) still joins the ranks' failure agreement
    (an allreduce of a failure flag before the gather), so no rank waits in the gather for it;
    the communicator stays usable for the next frame."""
    import copy
    import torch
    r, ref, _ = cornell
    comm = rtg.Comm(rtg.Comm.unique_id(), 1, 0, 0)
    try:
        out = torch.zeros((ref.shape[0], ref.shape[1], 3), dtype=torch.float32, device="cuda:0")
        bad = copy.deepcopy(r.scene.cameras[0])
        bad.num_samples = 0
        with pytest.raises(rtg.RtgError, match="bad camera"):
            r.render_ranked(bad, comm, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        r.render_ranked(0, comm, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(_bits(out.cpu().numpy()), _bits(ref))
    finally:
        comm.close()


def test_ranked_peer_that_never_joins_times_out(gpu):
    """a two-rank communicator whose second rank never calls ncclCommInitRank.  The
    first rank's set-up is non-blocking with a deadline (rtg_comm_init_rank_timeout): it aborts the
    communicator and returns an error within the timeout instead of waiting forever."""
    import time
    t0 = time.monotonic()
    with pytest.raises(rtg.RtgError, match="did not respond|timed out|aborted"):
        rtg.Comm(rtg.Comm.unique_id(), 2, 0, 0, timeout_ms=2000)
    assert time.monotonic() - t0 < 30.0


def test_dragon_full_frame_two_shards(gpu):
    """The bench scene at 1080p (1 spp): the shard + gather path at full size."""
    sc = scenegen.dragon1m(1920, 1080, spp=1)
    with rtg.Renderer(sc, device=0) as r:
        ref = r.render(0)
        img = r.render(0, num_devices=2, devices=[0, 0])
        assert np.array_equal(_bits(img), _bits(ref))
        img1 = r.render(0, num_devices=1, devices=[0])
        assert np.array_equal(_bits(img1), _bits(ref))


def test_cli_devices_flag(gpu, tmp_path):
    """rtg_cli --devices: the native host's renderScene on the multi-GPU path writes the same file."""
    import subprocess
    from rtg import native
    from rtg.scene import write_xml
    sc = scenegen.multilight(40, 30, spp=2)
    sc.cameras[0].image_name = "m.png"
    xml = write_xml(sc, str(tmp_path / "m.xml"))
    cli = native.CLI_PATH
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir(); b.mkdir()
    subprocess.run([cli, xml, "--out-dir", str(a)], check=True, capture_output=True, timeout=120)
    n = rtg.load_library().rtg_device_count()
    out = subprocess.run([cli, xml, "--devices", str(n), "--out-dir", str(b)], check=True, capture_output=True,
                         text=True, timeout=120)
    assert f"{n} GPU" in out.stdout
    assert (a / "m.png").read_bytes() == (b / "m.png").read_bytes()
