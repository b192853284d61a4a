// gol-mi355x: board geometry, domain decomposition and the bit-packed tile layout.
//
// Reference semantics (gol-main.c:76, gol-main.c:84-87, gol-main.c:124): each of the P ranks owns
// an N x N tile, the tiles are stacked vertically into a (P*N) x N torus, and the vertical wrap
// goes around the ring of ranks.  That is "per-rank" mode and stays the default.  This module
// generalises it:
//   * global mode (GOL_GLOBAL=1): N is the side of the *global* N x N board, split over P ranks;
//   * 1-D row strips (Px = 1) or a 2-D Px x Py block torus with 8 neighbours (N,S,E,W + corners);
//   * uneven splits (rows in units of 1, columns in units of 64-cell words in 2-D).
//
// Tile storage (Layout): 1 bit per cell, 64 cells per u64 word, bit b of word c = column 64c+b.
// Every row carries one ghost word on each side (word -1 and word nw) and the tile carries R ghost
// rows above and below (rows -R..-1 and h..h+R-1).  R is the halo depth: one exchange feeds R
// generations (temporal blocking).  Row r / word c lives at  (r + R) * pitch + (c + 1).
#pragma once

#include <array>
#include <string>
#include <vector>

#include "gol/common.hpp"

namespace gol {

enum Dir : int { DIR_N = 0, DIR_S, DIR_W, DIR_E, DIR_NW, DIR_NE, DIR_SW, DIR_SE, NUM_DIRS };

inline Dir opposite(Dir d) {
    static const Dir o[NUM_DIRS] = {DIR_S, DIR_N, DIR_E, DIR_W, DIR_SE, DIR_SW, DIR_NE, DIR_NW};
    return o[d];
}
inline int dir_dy(Dir d) {
    static const int v[NUM_DIRS] = {-1, 1, 0, 0, -1, -1, 1, 1};
    return v[d];
}
inline int dir_dx(Dir d) {
    static const int v[NUM_DIRS] = {0, 0, -1, 1, -1, 1, -1, 1};
    return v[d];
}
const char* dir_name(Dir d);

// How the global board is laid out across ranks.
struct Decomposition {
    i64 H = 0, W = 0;       // global rows / columns
    int P = 1;              // number of ranks
    int Px = 1, Py = 1;     // process grid (Px columns of ranks, Py rows of ranks); rank = cy*Px + cx
    bool per_rank = true;   // reference semantics: N is the per-rank tile side
    std::vector<i64> row_starts;  // size Py+1
    std::vector<i64> col_starts;  // size Px+1 (multiples of 64 when Px > 1)
    // Logical row strips used by the per-rank dump files and by the reference patterns:
    // strip s covers global rows [strip_starts[s], strip_starts[s+1]).  Always P strips.
    std::vector<i64> strip_starts;

    bool want_2d = false;   // GOL_DECOMP=2d was requested (a 1 x Py grid can still run the 2-D halo
                            // layout through the transport: Engine self-exchange mode)
    bool two_d() const { return Px > 1; }
    int rank_of(int cx, int cy) const { return (int)(pmod(cy, Py) * Px + pmod(cx, Px)); }
    std::string describe() const;
};

// N: CLI worldSize.  grid: "" / "auto" / "PxxPy" (e.g. "4x2").  decomp: "1d" / "2d" / "auto".
// width: board columns (0 = N, the reference's square tiles; the CLI is always square).  Per-rank
// mode: every rank's strip is N rows; global mode: the board is N rows x width columns.
Decomposition make_decomposition(i64 N, int P, bool global_mode, const std::string& decomp,
                                 const std::string& grid, i64 width = 0);

// This rank's view: tile extent, offsets and neighbours.
struct Geometry {
    Decomposition dec;
    int rank = 0;
    int cx = 0, cy = 0;
    i64 row0 = 0, col0 = 0;  // global coordinates of tile cell (0,0)
    i64 h = 0, w = 0;        // tile rows / columns
    std::array<int, NUM_DIRS> nbr{};

    bool is_self(Dir d) const { return nbr[d] == rank; }
    i64 global_words() const { return ceil_div(dec.W, 64); }
    i64 word0() const { return col0 / 64; }  // global word index of tile word 0 (col0 % 64 == 0)
};

Geometry make_geometry(const Decomposition& dec, int rank);

// Bit-packed tile storage with ghost words/rows.
struct Layout {
    i64 h = 0, w = 0;  // tile rows / columns (cells)
    i64 nw = 0;        // words per row
    int R = 1;         // ghost rows above and below (halo depth)
    i64 pitch = 0;     // words per stored row (nw + 2 ghost words, padded)

    Layout() = default;
    Layout(i64 h_, i64 w_, int R_);
    i64 rows_total() const { return h + 2 * (i64)R; }
    i64 words() const { return rows_total() * pitch; }
    i64 bytes() const { return words() * 8; }
    i64 index(i64 r, i64 c) const { return (r + R) * pitch + (c + 1); }
    // Valid-bit mask of word c (c in [0, nw)).
    u64 mask(i64 c) const { return word_mask(c, w); }
    bool aligned() const { return (w % 64) == 0; }
};

// Largest halo depth usable for a decomposition: bounded by the smallest tile height (a halo may
// not reach past the neighbouring tile), by the 64 bits of the ghost word, and by `requested`.
int clamp_halo_depth(const Decomposition& dec, int requested);

}  // namespace gol
