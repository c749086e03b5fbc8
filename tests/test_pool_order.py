"""The sample pool's item visiting order (blenderraytracer_amd/csrc/pool_order.h), enumerated by the
kernel's own header code on the CPU (tests/hostcheck): it must be a permutation of the items
(chunk * tiles + tile), so that every (tile, chunk) of the frame is traced exactly once and its
partials land where reduce_kernel reads them — the order only decides which items are in flight
together (tile blocks and XCD runs).  The GPU tests check the images themselves."""
import numpy as np
import pytest

from tests import hostcheck_binding as hc

SIZES = [(1920, 1080, 12), (1920, 1080, 1), (13, 7, 3), (8, 8, 1), (1, 1, 2), (100, 100, 3), (4096, 16, 2),
         (9, 4000, 1), (515, 517, 5)]


def _check(order, tiles, chunks):
    n = tiles * chunks
    assert order.shape == (n,)
    assert np.array_equal(np.sort(order), np.arange(n, dtype=np.uint32)), "not a permutation"


@pytest.mark.parametrize("cw,ch,chunks", SIZES)
@pytest.mark.parametrize("one_wave", [True, False])
def test_pool_order_is_a_permutation(cw, ch, chunks, one_wave):
    order, s, k, tiles = hc.pool_order(cw, ch, chunks, one_wave)
    _check(order, tiles, chunks)
    if not one_wave or k == 0:
        # the queue (and a launch without XCD runs) keeps chunk-major order: position p is in chunk p // tiles
        assert np.array_equal(order // tiles, np.arange(tiles * chunks) // tiles)


def test_pool_order_blocks_are_compact():
    """With S x S tile blocks, every run of S*S positions inside a full block covers an S x S square."""
    order, s, k, tiles = hc.pool_order(1920, 1080, 1, False)
    if s <= 1:
        pytest.skip("raster tile order in this build")
    tx = (1920 + 7) // 8
    xs, ys = order % tx, order // tx
    blk = order[: s * s]
    assert xs[: s * s].max() - xs[: s * s].min() == s - 1 and ys[: s * s].max() - ys[: s * s].min() == s - 1, blk


@pytest.mark.parametrize("cw,ch,chunks", [(1920, 1080, 12), (13, 7, 3), (515, 517, 5), (8, 8, 1)])
def test_pool_order_odd_parameters(cw, ch, chunks):
    """A build with odd block and run sizes (3 x 3 tiles, runs of 5) is still a permutation, and its XCD
    runs are contiguous: workgroups b, b + 8, ... of a full group take consecutive positions."""
    L = hc.lib(("RT_TILE_BLOCK=3", "RT_XCD_RUN=5"))
    import ctypes as C
    L.ptc_pool_order.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_int)]
    L.ptc_pool_order.restype = C.c_longlong
    tiles = ((cw + 7) // 8) * ((ch + 7) // 8)
    for one_wave in (1, 0):
        out = np.zeros(tiles * chunks, dtype=np.uint32)
        par = (C.c_int * 3)()
        assert L.ptc_pool_order(cw, ch, chunks, one_wave, out.ctypes.data_as(C.POINTER(C.c_uint32)), par) == tiles * chunks
        assert (par[0], par[1], par[2]) == (3, 5, tiles)
        _check(out, tiles, chunks)


def _chunk_range(L, s_begin, s_end, batch, batch_chunks, gci, chunk):
    import ctypes as C
    out = (C.c_int * 4)()
    L.ptc_chunk_range(s_begin, s_end, batch, batch_chunks, gci, chunk, out)
    return tuple(out)


@pytest.mark.parametrize("s0,s1,batch,chunk", [(0, 512, 32, 32), (0, 24, 3, 3), (0, 17, 4, 4), (5, 17, 4, 3),
                                               (0, 8, 2, 2), (0, 100, 7, 3), (3, 64, 16, 5), (0, 1000, 64, 45)])
def test_fused_chunks_are_the_batches_chunks(s0, s1, batch, chunk):
    """A fused launch (launch_trace_batches: every batch of a progressive render in one pool launch)
    gives launch chunk gci the samples that chunk gci % batch_chunks of batch gci // batch_chunks has in
    that batch's own launch, and an empty range to the chunks a short last batch does not have — so
    the items, their partials and the reduces are those of one launch per batch (bit-identical sums;
    the GPU test test_overlapped_batches_equal_serial_batches checks the images)."""
    import ctypes as C
    L = hc.lib()
    L.ptc_chunk_range.argtypes = [C.c_int] * 6 + [C.POINTER(C.c_int)]
    nb = -(-(s1 - s0) // batch)
    chunks_b = -(-batch // chunk)
    seen = []
    for gci in range(nb * chunks_b):
        b, ci, sb, se = _chunk_range(L, s0, s1, batch, chunks_b, gci, chunk)
        assert (b, ci) == (gci // chunks_b, gci % chunks_b)
        bb, be = s0 + b * batch, min(s1, s0 + (b + 1) * batch)      # batch b's own launch
        nchunks = -(-(be - bb) // chunk)
        if ci < nchunks:
            assert (sb, se) == _chunk_range(L, bb, be, 0, 0, ci, chunk)[2:], (gci, b, ci)
            seen.extend(range(sb, se))
        else:
            assert se <= sb, (gci, sb, se)                          # a short last batch's missing chunk
    assert seen == list(range(s0, s1))                               # every sample once, in order


@pytest.mark.parametrize("s0,s1,batch,chunk,ways", [(0, 512, 32, 32, 2), (0, 512, 32, 11, 8), (0, 24, 3, 3, 3),
                                                    (5, 17, 4, 3, 2), (0, 100, 7, 3, 3), (0, 1000, 64, 45, 8)])
def test_multi_device_fused_chunks_are_the_batches_chunks(s0, s1, batch, chunk, ways):
    """The whole-batch multi-device split with fused launches: device d's launch (s_begin = s0 + d batch,
    ImageParams::batch_ways = N) gives its local batch lb the samples and chunks of the render's batch
    k = d + lb N as that batch's own launch has them, so every sample is traced once, by one device, in
    the same chunks as on one device (bit-identical sums after the batch-order reduces)."""
    import ctypes as C
    L = hc.lib()
    L.ptc_chunk_range.argtypes = [C.c_int] * 6 + [C.POINTER(C.c_int)]
    L.ptc_chunk_range_ways.argtypes = [C.c_int] * 7 + [C.POINTER(C.c_int)]
    nb = -(-(s1 - s0) // batch)
    chunks_b = -(-batch // chunk)
    seen = []
    for d in range(ways):
        nbd = -(-(nb - d) // ways) if nb > d else 0
        for gci in range(nbd * chunks_b):
            out = (C.c_int * 4)()
            L.ptc_chunk_range_ways(s0 + d * batch, s1, batch, chunks_b, ways, gci, chunk, out)
            lb, ci, sb, se = tuple(out)
            k = d + lb * ways
            bb, be = s0 + k * batch, min(s1, s0 + (k + 1) * batch)
            if ci < -(-(be - bb) // chunk):
                assert (sb, se) == _chunk_range(L, bb, be, 0, 0, ci, chunk)[2:], (d, gci)
                seen.extend(range(sb, se))
            else:
                assert se <= sb
    assert sorted(seen) == list(range(s0, s1))



@pytest.mark.parametrize("cw,ch,chunks,bands", [(1920, 1080, 4, 8), (1920, 1080, 1, 64), (13, 7, 3, 1), (515, 517, 5, 7),
                                                (64, 72, 2, 9), (8, 8, 1, 1), (100, 33, 3, 5)])
def test_band_order(cw, ch, chunks, bands):
    """rt_trace_device_bands' item order (pool_order.h band_item): a permutation of the items in which every
    band's items — whole tile rows, all chunks — form one contiguous run of positions, in band order, of
    exactly band_items(b) items; the bands tile the crop's rows (the kernel counts each item into
    band_of_tile of its tile, so every band's flag is raised by its own items only)."""
    import ctypes as C
    L = hc.lib()
    L.ptc_band_order.argtypes = [C.c_int] * 4 + [C.POINTER(C.c_uint32), C.POINTER(C.c_int), C.POINTER(C.c_uint32)]
    L.ptc_band_order.restype = C.c_longlong
    tiles_x, tiles_y = (cw + 7) // 8, (ch + 7) // 8
    tiles = tiles_x * tiles_y
    out = np.zeros(tiles * chunks, dtype=np.uint32)
    band = np.zeros(tiles * chunks, dtype=np.int32)
    counts = np.zeros(bands, dtype=np.uint32)
    assert L.ptc_band_order(cw, ch, chunks, bands, out.ctypes.data_as(C.POINTER(C.c_uint32)),
                            band.ctypes.data_as(C.POINTER(C.c_int)), counts.ctypes.data_as(C.POINTER(C.c_uint32))) == out.size
    _check(out, tiles, chunks)
    assert np.all(np.diff(band) >= 0), "bands not contiguous / in order"
    assert int(counts.sum()) == out.size
    assert np.array_equal(np.bincount(band, minlength=bands), counts)
    rows = (out % tiles) // tiles_x
    for b in range(bands):                    # band b: tile rows [b T / B, (b + 1) T / B)
        sel = rows[band == b]
        if sel.size:
            assert sel.min() == b * tiles_y // bands and sel.max() == (b + 1) * tiles_y // bands - 1
