// gol-mi355x: CPU backend — bit-packed stepper, halo helpers, init and I/O on host memory.
//
// This is both the GPU-less plumbing backend (BASELINE config 1: 256^2 x 100 gens on the CPU) and
// the C++ oracle for the HIP kernels.  It implements exactly the same temporal-blocking semantics
// as the GPU kernel: a superstep of k generations reads k ghost rows above and below the tile and
// the ghost words beside it, and the ghost area is evolved redundantly (shrinking by one row per
// generation) so no exchange is needed inside the superstep.
#pragma once

#include "gol/geometry.hpp"
#include "gol/pattern.hpp"

namespace gol {
namespace cpu {

// One generation for rows [r_lo, r_hi) (all words -1 .. nw) of `dst` from `src`.
void step_rows(const u64* src, u64* dst, const Layout& L, i64 r_lo, i64 r_hi);

// k generations (k <= L.R).  Ping-pongs between a and b; returns the buffer with the result.
u64* superstep(u64* a, u64* b, const Layout& L, int k);

// x-periodic ghost words (and tail ghost bits) for rows [r_lo, r_hi).
void fill_ghost_cols_wrap(u64* buf, const Layout& L, i64 r_lo, i64 r_hi);
// y-periodic ghost rows of a tile that is its own vertical neighbour (any h, even h < R).
void fill_ghost_rows_wrap(u64* buf, const Layout& L);

// Initialise the tile from a pattern (ghost area zeroed; caller refreshes halos).
void init_tile(u64* buf, const Layout& L, const Geometry& g, const PatternSpec& p);

// Dense, masked copy of the tile words (h * nw), and the reverse.
void extract_words(const u64* buf, const Layout& L, u64* dense);
void insert_words(u64* buf, const Layout& L, const u64* dense);

// Live-cell count and decomposition-invariant fingerprint of the tile.
u64 population(const u64* buf, const Layout& L);
u64 fingerprint(const u64* buf, const Layout& L, i64 grow0, i64 gword0, i64 gwords);

}  // namespace cpu
}  // namespace gol
