// Host mirror of the GEMM dispatch's rasters: which workgroup of a launch computes which output tile,
// in which round (persistent grids) and piece (split-K). It runs the very raster functions the kernels
// run (xcd_remap, tile_coords, tile_coords_sq are __host__ __device__, gemm_tile_common.h), so a bad
// output tile found by the ABFT check (gemm_abft.hip) maps back to its workgroup, and through the
// placement record of the checked dispatch (note_placement) to the XCD and CU that computed it.
#pragma once

#include <hip/hip_runtime.h>

#include "gemm_tile_common.h"

struct GemmRaster {
  // GENERIC: 2-D grid, one workgroup per tile (blockIdx.y = tile row); GRID / GRID_SQ: one workgroup per
  // tile through xcd_remap + tile_coords / tile_coords_sq; PERSISTENT / PERSISTENT_SQ: `grid` workgroups
  // walking XCD-contiguous tile runs / the square super-tiles in rounds; SMALL: one workgroup per
  // (tile, K piece) through xcd_remap (gemm_small.h).
  // SPLIT: one workgroup per (tile, K piece) of the asm frame's split-K form, piece-major through
  // xcd_remap, tiles in tile_coords order (gemm_w4ap.h SPLIT).
  enum Kind { GENERIC = 0, GRID = 1, GRID_SQ = 2, PERSISTENT = 3, PERSISTENT_SQ = 4, SMALL = 5, SPLIT = 6 };
  int kind = GENERIC, variant = 0, tile_m = 64, tile_n = 64, grid = 0, splits = 1, pmajor = 0;

  static GemmRaster generic(int v, int tm, int tn) { return {GENERIC, v, tm, tn, 0, 1, 0}; }
  static GemmRaster grid_of(int v, int tm, int tn, int nwg, bool sq) { return {sq ? GRID_SQ : GRID, v, tm, tn, nwg, 1, 0}; }
  static GemmRaster persistent(int v, int tm, int tn, int g, bool sq) {
    return {sq ? PERSISTENT_SQ : PERSISTENT, v, tm, tn, g, 1, 0};
  }
  static GemmRaster small(int v, int tm, int tn, int splits, int pmajor) { return {SMALL, v, tm, tn, 0, splits, pmajor}; }
  static GemmRaster split(int v, int splits, int pmajor) { return {SPLIT, v, 256, 256, 0, splits, pmajor}; }
};

// `info` (8 ints): variant, kind, tile_m, tile_n, tiles_m, tiles_n, launch grid (workgroups), pieces per
// tile. `owners` / `rounds` (optional, `cap` ints each): for tile t = tm * tiles_n + tn and piece p, the
// workgroup (linear block id) at [t * pieces + p] and the round of its tile loop it reached the tile in
// (0 for one-tile-per-workgroup grids). Returns the tile count, -1 when `cap` is too small.
inline int raster_fill(const GemmRaster& r, int M, int N, int* info, int* owners, int* rounds, int cap) {
  const int tiles_m = (M + r.tile_m - 1) / r.tile_m, tiles_n = (N + r.tile_n - 1) / r.tile_n;
  const int nt = tiles_m * tiles_n;
  const int pieces = r.kind == GemmRaster::SMALL || r.kind == GemmRaster::SPLIT ? r.splits : 1;
  int grid = r.grid;
  if (r.kind == GemmRaster::GENERIC) grid = nt;
  if (r.kind == GemmRaster::SMALL || r.kind == GemmRaster::SPLIT) grid = nt * r.splits;
  if (info) {
    const int v[8] = {r.variant, r.kind, r.tile_m, r.tile_n, tiles_m, tiles_n, grid, pieces};
    for (int i = 0; i < 8; ++i) info[i] = v[i];
  }
  if (!owners) return nt;
  if ((long long)nt * pieces > cap) return -1;
  for (int i = 0; i < nt * pieces; ++i) {
    owners[i] = -1;
    if (rounds) rounds[i] = 0;
  }
  auto put = [&](int tm, int tn, int piece, int b, int round) {
    if (tm < 0 || tm >= tiles_m || tn < 0 || tn >= tiles_n) return;
    const int at = (tm * tiles_n + tn) * pieces + piece;
    owners[at] = b;
    if (rounds) rounds[at] = round;
  };
  switch (r.kind) {
    case GemmRaster::GENERIC:
      for (int tm = 0; tm < tiles_m; ++tm)
        for (int tn = 0; tn < tiles_n; ++tn) put(tm, tn, 0, tm * tiles_n + tn, 0);
      break;
    case GemmRaster::GRID:
    case GemmRaster::GRID_SQ:
      for (int b = 0; b < nt; ++b) {
        int tm, tn;
        if (r.kind == GemmRaster::GRID_SQ) tile_coords_sq(b, tiles_n, tm, tn);
        else tile_coords(xcd_remap(b, nt), tiles_m, tiles_n, tm, tn);
        put(tm, tn, 0, b, 0);
      }
      break;
    case GemmRaster::PERSISTENT: {
      const int per = grid / NXCD, q = nt / NXCD, rem = nt % NXCD;
      for (int b = 0; b < grid; ++b) {
        const int xcd = b % NXCD;
        const int t_begin = (xcd < rem) ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
        const int t_end = t_begin + q + (xcd < rem ? 1 : 0);
        int round = 0;
        for (int t = t_begin + b / NXCD; per > 0 && t < t_end; t += per, ++round) {
          int tm, tn;
          tile_coords(t, tiles_m, tiles_n, tm, tn);
          put(tm, tn, 0, b, round);
        }
      }
      break;
    }
    case GemmRaster::PERSISTENT_SQ:
      for (int b = 0; b < grid; ++b) {
        int round = 0;
        for (int t = b; t < nt; t += grid, ++round) {
          int tm, tn;
          tile_coords_sq(t, tiles_n, tm, tn);
          put(tm, tn, 0, b, round);
        }
      }
      break;
    case GemmRaster::SMALL: {
      const int items = nt * r.splits;
      for (int b = 0; b < items; ++b) {
        const int item = xcd_remap(b, items);
        int tile = item, piece = 0;
        if (r.splits > 1) {
          piece = r.pmajor ? item / nt : item % r.splits;
          tile = r.pmajor ? item - piece * nt : item / r.splits;
        }
        put(tile / tiles_n, tile % tiles_n, piece, b, 0);
      }
      break;
    }
    case GemmRaster::SPLIT: {
      const int items = nt * r.splits;
      for (int b = 0; b < items; ++b) {
        const int item = xcd_remap(b, items);
        const int piece = r.pmajor ? item / nt : item % r.splits;
        int tm, tn;
        tile_coords(r.pmajor ? item - piece * nt : item / r.splits, tiles_m, tiles_n, tm, tn);
        put(tm, tn, piece, b, 0);
      }
      break;
    }
  }
  return nt;
}

// Points the placement record of this TU's REC kernels on `stream`'s device at `placement` (device
// memory, 2 x uint32 per workgroup; nullptr turns recording off). Synchronous: the launch that follows
// on any stream sees it.
inline hipError_t set_placement_record(hipStream_t stream, uint32_t* placement) {
  int dev = 0, prev = 0;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) return e;
  dev = prev;
  if (stream != nullptr && stream != hipStreamPerThread && (e = hipStreamGetDevice(stream, &dev)) != hipSuccess)
    return e;
  if (dev != prev && (e = hipSetDevice(dev)) != hipSuccess) return e;
  e = hipMemcpyToSymbol(HIP_SYMBOL(g_wg_placement), &placement, sizeof placement, 0, hipMemcpyHostToDevice);
  if (dev != prev) (void)hipSetDevice(prev);
  return e;
}
