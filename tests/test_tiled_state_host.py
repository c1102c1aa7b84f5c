"""flat.TiledState on CPU tensors: every element of every stream sits where
bdl_adam_args' tiling formula (include/bdl_sgmcmc.h, ABI v7) says the kernel
reads it, views round-trip through flat() / load(), and abi() names the
kernel's stream slots.  No GPU."""
import numpy as np
import pytest
import torch

from bayesdll_amd.flat import TILE_LOG2_MAX, TiledState

SLOTS = ("mom", "adam_m", "adam_v", "sgd_buf")


def kernel_index(e, s, log2, streams):
    """Block index of element e of stream slot s (the header's formula, with
    the stream base at s * 4 * 2^log2 floats)."""
    g = e // 4
    return s * (4 << log2) + (((g >> log2) * streams << log2) + (g & ((1 << log2) - 1))) * 4 + e % 4


@pytest.mark.parametrize("n,log2", [(1, None), (7, None), (4096, None), (4097, 2), (1000, 3),
                                    (12345, 4), (70001, 5)])
@pytest.mark.parametrize("names", [("adam_m", "adam_v"), ("adam_m", "adam_v", "sgd_buf"), SLOTS])
def test_every_element_sits_where_the_kernel_reads_it(n, log2, names):
    ts = TiledState(n, names, "cpu", log2=log2)
    rng = np.random.default_rng(n)
    want = {nm: torch.from_numpy(rng.standard_normal(n).astype(np.float32)) for nm in names}
    for nm in names:
        ts.load(nm, want[nm])
    blk = ts.block.numpy()
    e = np.arange(n)
    for s, nm in enumerate(names):
        idx = np.array([kernel_index(int(k), s, ts.log2, len(names)) for k in e])
        assert np.array_equal(blk[idx], want[nm].numpy())
        assert torch.equal(ts.flat(nm), want[nm])
    # padding and other streams untouched: the block holds exactly the loaded values
    assert np.count_nonzero(blk) == sum(int(torch.count_nonzero(v)) for v in want.values())


def test_one_tile_streams_are_contiguous_views():
    ts = TiledState(1000, ("adam_m", "adam_v"), "cpu")
    assert ts.ntiles == 1
    v = ts.stream("adam_v")
    assert v.dim() == 1 and v.numel() == 1000 and v.is_contiguous()
    v.fill_(2.0)
    assert ts.flat("adam_v").data_ptr() == v.data_ptr()
    assert float(ts.block[:ts.tile].abs().sum()) == 0.0  # adam_m's slot untouched


def test_many_tiles_give_2d_views_and_flat_copies():
    ts = TiledState(70001, ("adam_m", "adam_v", "sgd_buf"), "cpu", log2=5)
    assert ts.ntiles == -(-70001 // 128)
    v = ts.stream("adam_v")
    assert v.shape == (ts.ntiles, 128)
    v.zero_()
    v[0, 0] = 3.0
    assert ts.flat("adam_v")[0] == 3.0 and ts.flat("adam_v").numel() == 70001


def test_abi_mask_follows_slot_order():
    ts = TiledState(64, ("adam_m", "adam_v", "sgd_buf"), "cpu")
    assert ts.abi(SLOTS) == (ts.log2, 3, 0b1110)
    ts4 = TiledState(64, SLOTS, "cpu")
    assert ts4.abi(SLOTS)[1:] == (4, 0b1111)


def test_default_tile_is_at_most_16_mib_per_stream():
    assert TiledState(10, ("adam_m",), "cpu").log2 >= 1
    assert TiledState(4 << 12, ("adam_m",), "cpu").log2 == 12  # one tile, no padding
    assert TILE_LOG2_MAX == 20  # ViT-L/32 (306,535,400): 2^20 float4 groups = 16 MiB per tile
