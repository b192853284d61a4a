// gol-mi355x: work plans for the temporal-blocked stencil kernel.
//
// The reference launches one thread per byte-cell over the whole N x N tile every generation
// (gol-with-cuda.cu:189-198, 264-277).  Here a generation sweep is planned once on the host and
// replayed: the output region(s) of a superstep are cut into *segments*, each a block of output
// rows x up to 62 output words, and the segments are packed side by side into 64-lane waves.
//
//   lane layout of a segment of `nwords` output words starting at word c0:
//       [halo c0-1] [c0] [c0+1] ... [c0+nwords-1] [halo c0+nwords]      (nwords + 2 lanes)
//
// Every lane owns one 64-cell word column and streams down the rows; horizontal neighbours come
// from the adjacent lanes through DPP (wave_shr/wave_shl).  The two halo lanes carry the
// neighbouring words: after k <= 64 generations only their outer bits are invalid, so the interior
// lanes stay exact.  Several narrow segments can share one wave (the 2-D edge columns, the
// remainder of a row), so lane utilisation stays high for any width.
#pragma once

#include <string>
#include <map>
#include <vector>

#include "gol/common.hpp"

namespace gol {

// Per-lane descriptor, read once at kernel start (16 bytes, naturally aligned).
struct LaneDesc {
    i32 row0;   // first output row of this lane's segment (tile coordinates)
    i32 col;    // word column this lane streams (-1 .. nw)
    u32 flags;  // LANE_* bits
    i32 nrows;  // output rows of the segment; identical for all 64 lanes of a wave (0: idle wave)
};

enum : u32 {
    LANE_STORE = 1u << 0,  // interior lane whose word is an output word
};

// Output region of a superstep: rows [r0, r1) x words [c0, c1) of the tile.
struct Region {
    i64 r0, r1, c0, c1;
};

static constexpr int kWaveLanes = 64;
static constexpr int kSegWords = kWaveLanes - 2;  // output words of a full-width segment
static constexpr int kWavesPerBlock = 4;  // 256-thread workgroups of independent waves

struct PlanStats {
    i64 waves = 0;        // including padding waves
    i64 active_lanes = 0; // lanes that store an output word (summed over waves, per row)
    i64 lane_rows = 0;    // total lane x input-row slots issued
    i64 out_words = 0;    // output words produced
};

// Build the lane descriptors for `regions` (all within a tile with `nw` words per row).
// `rows_per_chunk` is the segment height S (rows of output per wave); `k` the generations per pass
// (only used to account for the 2k extra input rows per segment in the stats).  With `xwrap` the
// tile is its own E/W neighbour (w % 64 == 0): halo lanes left of word 0 stream word nw-1 and halo
// lanes right of word nw-1 stream word 0, so no ghost words are needed.
// Waves are ordered for L2 locality: row-major, and whole workgroups of `wg_waves` waves
// permuted so each of the `xcds` XCDs (workgroup b runs on XCD b % xcds) gets a contiguous stretch.
// With `fold` (the tile kernel's STEP_TILE_FOLD) segments are packed into 32-lane tiles of <= 30
// output words, and each tile's 64 lanes are its 32 lanes twice: the kernel folds the tile's rows so
// lanes 0-31 stream the top half and lanes 32-63 (bottom up) the bottom half.
// With `age_weights` (C > 1 values; a single region, not folded) the plan's row bands get heights
// proportional to the weight of the dispatch class their full-width segments land in: workgroup b of
// nwg is in class b * C / nwg.  On MI355X the co-resident waves of a SIMD are issued by age, and in a
// one-round plan of 3 workgroups per CU the first-dispatched third of the grid finished a pass in ~half
// the time of the last third (tools/stamp_probe.hip, profiles/stamp_probe.txt): weights (w0 > w1 > w2)
// give the older waves taller segments so that a SIMD's waves finish together.  (Measured: every weight
// set made the pass slower — it is VALU-bound, the SIMD busy until its last wave ends whatever the
// split, profiles/stamp_age_weights.txt — so no engine plan uses it; tools/stamp_probe.hip does.)
std::vector<LaneDesc> build_plan(const std::vector<Region>& regions, i64 nw, i64 h, i64 rows_per_chunk, int k,
                                 bool xwrap, PlanStats* stats = nullptr, int wg_waves = kWavesPerBlock,
                                 int xcds = 8, bool fold = false, const std::vector<double>* age_weights = nullptr);

// Bounds check of a plan before it is uploaded (a bad plan would fault the GPU): every lane's word
// column lies in [-1, nw]; without y-wrap its input rows [row0-k, row0+nrows+k) lie in the
// allocated rows [-R, h+R); store lanes write rows inside [-R, h+R) and columns in [-1, nw]
// (ghost words are outputs of the earlier passes of a 2-D multi-pass superstep).
// Returns an empty string when the plan is safe, else a description of the first violation.
std::string validate_plan(const std::vector<LaneDesc>& lanes, i64 nw, i64 h, int R, int k, bool wrap_y);

// Number of waves (padded to whole workgroups) of the plan, without materialising lanes.
i64 plan_waves(const std::vector<Region>& regions, i64 nw, i64 h, i64 rows_per_chunk, bool fold = false);

// Pick a segment height so that the sweep has enough waves to fill the GPU (about `target_waves`)
// while keeping the 2k-row vertical halo overhead small.
i64 choose_rows_per_chunk(const std::vector<Region>& regions, int k, i64 target_waves, i64 min_rows);

// Occupancy-balanced segment height: the smallest S >= min_rows whose plan fits in ONE round of
// `resident_waves` (every wave resident from the start, equal work, no straggler workgroups).
// Time ~ rounds x (S + k), so one full round with the shortest segments is optimal.
i64 balanced_rows_per_chunk(const std::vector<Region>& regions, i64 nw, i64 h, int k, i64 resident_waves,
                            i64 min_rows, bool xwrap, bool fold = false);

// Segment height for the streaming kernel on BIG regions: one round (balanced_rows_per_chunk) while its
// segments are at most about `round_rows` tall, otherwise the whole number of rounds (at most
// `max_rounds`) that brings them nearest to it.  Waves of one round start together and stream equal
// work, but they do not finish together (the co-resident waves of a SIMD compete for issue), and a
// one-round pass ends on its slowest wave; with several rounds a finished wave's slot takes the next
// segment, at the price of 2k halo rows per extra segment.  Measured, K = 8, one tile, kbench
// (profiles/bigboard_rounds.txt): 131072^2 one round (1425 rows) 163 us/gen, 2 rounds 149.4-150, 4
// rounds (360 rows) 145-145.6, 8 rounds 145.7-147.3; 65536^2 keeps one round (365 rows; 2 rounds of
// 180: 46.7 vs 44.8-45.8).  round_rows <= 0 disables it (one round).
i64 round_balanced_rows(const std::vector<Region>& regions, i64 nw, i64 h, int k, i64 resident_waves, i64 min_rows,
                        bool xwrap, i64 round_rows, i64 max_rounds = 32);

// The cheapest cut of a k-generation superstep into kernel passes, given the measured cost (us) of one
// pass at each available depth: dynamic programming over k (a pass streams the board through HBM once
// whatever its depth, so the costs are far from linear in the depth).  Deepest pass first (12 + 8 measured
// faster than 8 + 12).  Empty when no depth sums to k.
std::vector<int> cheapest_cut(int k, const std::map<int, double>& pass_cost);

// Neighbour tiles of a resident plan (hip_kernels.hpp step_resident: one plan wave = one tile, kept
// by one workgroup for a whole run).  Tile t reads, for each of its lanes, rows [row0-k, row0+nrows+k)
// of the lane's word column (modulo h with wrap_y); its neighbours are the OTHER tiles whose store
// lanes own words there.  CSR: idx[off[t] .. off[t+1]).  Returns an empty string, or a description
// of why the plan cannot run resident (a column not covered exactly once by store lanes, a lane
// outside [0, nw), a read outside the owned rows without wrap_y).
std::string resident_neighbours(const std::vector<LaneDesc>& lanes, i64 nw, i64 h, int k, bool wrap_y,
                                std::vector<u32>& off, std::vector<u32>& idx);

}  // namespace gol
