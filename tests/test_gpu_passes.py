"""Pass scheduling of rtg_render (rtg_host.cpp render_impl): pass sizes, lanes and the tile order of
a pass's pixels (tile_pixel).  Which pass renders a pixel must never change its value -- every
sample of a pixel is in one pass and summed in sample order (src/Scene.cpp:386-409) -- so every
schedule gives the same frame bit for bit, repeated frames included."""
import numpy as np
import pytest

import rtg
from rtg import scenegen

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a).view(np.int32)


@pytest.mark.parametrize("batch,streams", [(2000, 0), (3000, 3), (700, 1)])
def test_pass_sizes_and_lanes_give_the_same_frame(gpu, batch, streams):
    sc = scenegen.dragon1m(96, 54, spp=4, nu=60, nv=30)      # glass + mirror: very unequal pixel costs
    with rtg.Renderer(sc, device=gpu) as r:
        ref = r.render(0)
        rays = r.stats()["total_rays"]
        for _ in range(2):
            img = r.render(0, max_batch_rays=batch, streams=streams)
            assert np.array_equal(_bits(img), _bits(ref))
            assert r.stats()["total_rays"] == rays


def test_row_shards_with_small_passes_gather_to_the_frame(gpu):
    sc = scenegen.dragon1m(64, 40, spp=3, nu=40, nv=20)
    with rtg.Renderer(sc, device=gpu) as r:
        ref = r.render(0)
        for _ in range(3):
            img = r.render(0, num_devices=3, devices=[0, 0, 0], max_batch_rays=900)
            assert np.array_equal(_bits(img), _bits(ref))


@pytest.mark.parametrize("tile_band", [1, 3, 16, 4096])
def test_tile_order_does_not_change_the_frame(gpu, tile_band):
    sc = scenegen.cornell(70, 45, spp=3, level=1)
    with rtg.Renderer(sc, device=gpu) as r:
        ref = r.render(0)
        img = r.render(0, max_batch_rays=1000, tile_band=tile_band)
        shard = r.render(0, num_devices=2, devices=[0, 0], tile_band=tile_band)
    assert np.array_equal(_bits(img), _bits(ref))
    assert np.array_equal(_bits(shard), _bits(ref))


def test_wide_row_with_a_tall_band_is_not_mis_tiled(gpu):
    """tile_pixel forms tile_h * tile_band * nx in 32-bit ints.  A 2^20-pixel row with
    tile_band = 4096 would be 2^35 pixels per band; the band is clamped so that one band stays below
    2^31, and the frame equals the one-tile-high order bit for bit (pixels are not mis-placed)."""
    sc = scenegen.simple(1 << 20, 1)
    with rtg.Renderer(sc, device=gpu) as r:
        ref = r.render(0, tile_band=1)
        img = r.render(0, tile_band=4096)
        shard = r.render(0, num_devices=2, devices=[0, 0], tile_band=4096)
    assert np.isfinite(ref).all()
    assert np.array_equal(_bits(img), _bits(ref))
    assert np.array_equal(_bits(shard), _bits(ref))


@pytest.mark.parametrize("ny", [1, 5])
def test_more_shards_than_row_blocks(gpu, ny):
    """Shards that own no rows (an image with fewer 4-row blocks than shards, e.g. 8 GPUs and a short
    image) render nothing and the gather still yields the single-device frame (round 6: the pass count of
    an empty shard divided by zero)."""
    sc = scenegen.simple(64, ny)
    with rtg.Renderer(sc, device=gpu) as r:
        ref = r.render(0)
        shard = r.render(0, num_devices=3, devices=[0, 0, 0])
    assert np.array_equal(_bits(shard), _bits(ref))
