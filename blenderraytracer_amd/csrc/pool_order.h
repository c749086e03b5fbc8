// pool_order.h — the sample pool's 8x8 tiles, the order in which its (tile, chunk) items are visited
// and the samples of each chunk (pt_trace.hip).  Host-and-device code: tests/hostcheck enumerates them
// on the CPU (tests/test_pool_order.py: the order is a permutation; a fused launch's chunks are the
// chunks of the per-batch launches).
#pragma once
#include "pt_path.h"

namespace rt {

// 8x8 tile `tile` of the crop: origin, valid width and valid pixel count (edge tiles are ragged)
struct Tile { int x0, y0, vw, nv; };
RT_HD Tile tile_of(const ImageParams& im, int tile) {
    const int tiles_x = (im.cw + 7) / 8;
    Tile t;
    t.x0 = (tile % tiles_x) * 8;
    t.y0 = (tile / tiles_x) * 8;
    t.vw = min(8, im.cw - t.x0);
    t.nv = t.vw * min(8, im.ch - t.y0);
    return t;
}

// Visiting order of the pool's (tile, chunk) items.  It is a permutation only: each item is traced as
// before and its partials stay at item = chunk * tiles + tile, so the sums are unchanged bit for bit.
// RT_TILE_BLOCK = S: within a chunk the tiles are taken in blocks of S x S tiles (raster order inside
// a block, blocks in raster order), so the items in flight cover compact screen regions rather than
// full-width bands.  RT_XCD_RUN = K (one-wave pool kernel): workgroups b, b + 8, b + 16, ... share an
// XCD (dispatch deals workgroups round-robin over the 8 XCDs); they take K consecutive positions of the
// order, so each XCD's L2 serves its own screen region instead of all eight serving the same band.
#ifndef RT_TILE_BLOCK
#define RT_TILE_BLOCK 1
#endif
#ifndef RT_XCD_RUN
#define RT_XCD_RUN 1024          // mesh50k +2.8 %, tile blocks ±0 on top
#endif
RT_HD int tile_at(const ImageParams& im, int t) {
    constexpr int S = RT_TILE_BLOCK;
    if constexpr (S <= 1) {
        return t;
    } else {
        const int tiles_x = (im.cw + 7) / 8, tiles_y = (im.ch + 7) / 8;
        const int band = t / (S * tiles_x);
        const int rows = min(S, tiles_y - band * S);       // the last band may be shorter
        const int o = t - band * S * tiles_x;
        const int c = o / (S * rows);                      // every block before the last is S wide
        const int oo = o - c * S * rows;
        const int w = min(S, tiles_x - c * S);
        const int r = oo / w;
        return (band * S + r) * tiles_x + c * S + (oo - r * w);
    }
}
// position in the visiting order of one-wave workgroup b of a launch of n workgroups
RT_HD unsigned pool_position(unsigned b, unsigned n) {
    constexpr unsigned K = RT_XCD_RUN;
    if constexpr (K == 0) {
        return b;
    } else {
        const unsigned g = b / (8 * K), r = b - g * 8 * K;
        if ((g + 1) * 8 * K > n) return b;                 // the last, partial group keeps its order
        return g * 8 * K + (r & 7) * K + (r >> 3);
    }
}
// Band-major order (ImageParams::bands = B > 0, rt_trace_device_bands): the crop's tile rows split into B
// horizontal bands (band b: tile rows [b T / B, (b + 1) T / B), T tile rows), all items of band b — its
// tiles x the launch's band_chunks chunks, chunk-major inside the band — before any of band b + 1, so the
// bands' pixels become final one after another and each can be reduced across GPUs while the later bands
// trace.  A permutation only: every item is traced as before, its partials stay at
// chunk * tiles + tile, and the reduce adds each pixel's chunks in chunk order (bit-identical sums).
RT_HD int band_row0(const ImageParams& im, int b) {
    return (int)((long long)b * ((im.ch + 7) / 8) / im.bands);
}
RT_HD unsigned band_item(const ImageParams& im, unsigned p, int tiles) {
    const int tiles_x = (im.cw + 7) / 8;
    const unsigned chunks = (unsigned)im.band_chunks;
    for (int b = 0; b < im.bands; ++b) {
        const int r0 = band_row0(im, b), r1 = band_row0(im, b + 1);
        const unsigned n = (unsigned)((r1 - r0) * tiles_x);
        if (p < n * chunks) {
            const unsigned ci = p / n;
            return ci * (unsigned)tiles + (unsigned)(r0 * tiles_x) + (p - ci * n);
        }
        p -= n * chunks;
    }
    return p;   // positions beyond the items (not taken)
}
// band of tile `tile` and the items that complete it: the largest b with floor(b T / B) <= row, i.e.
// b T < (row + 1) B, so b = floor(((row + 1) B - 1) / T)
RT_HD int band_of_tile(const ImageParams& im, int tile) {
    const int row = tile / ((im.cw + 7) / 8);
    return (int)(((long long)(row + 1) * im.bands - 1) / ((im.ch + 7) / 8));
}
RT_HD uint32_t band_items(const ImageParams& im, int b) {
    return (uint32_t)((band_row0(im, b + 1) - band_row0(im, b)) * ((im.cw + 7) / 8)) * (uint32_t)im.band_chunks;
}

// item (chunk * tiles + tile) at position p of the visiting order.  (A longest-first order of each
// chunk's tiles, from a host estimate of the frame's cost, measured slower in round 5: DESIGN.md §4.)
RT_HD unsigned item_at(const ImageParams& im, unsigned p, int tiles) {
    if (im.bands > 0) return band_item(im, p, tiles);
    if constexpr (RT_TILE_BLOCK <= 1) return p;
    const unsigned ci = p / (unsigned)tiles;
    return ci * (unsigned)tiles + (unsigned)tile_at(im, (int)(p - ci * (unsigned)tiles));
}

// (batch, chunk within it, first sample, end sample) of launch chunk gci (ImageParams::batch_chunks)
struct ChunkRange { int b, ci, sb, se; };
RT_HD ChunkRange chunk_range(const ImageParams& im, int gci, int chunk) {
    ChunkRange r;
    r.b = im.batch_chunks ? gci / im.batch_chunks : 0;
    r.ci = gci - r.b * im.batch_chunks;
    const int bs = im.s_begin + r.b * im.batch_samples * (im.batch_ways > 1 ? im.batch_ways : 1);
    r.sb = bs + r.ci * chunk;
    r.se = min(im.batch_chunks ? min(im.s_end, bs + im.batch_samples) : im.s_end, r.sb + chunk);
    return r;
}

}  // namespace rt
