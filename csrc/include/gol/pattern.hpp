// gol-mi355x: initial board patterns.
//
// Reference patterns (gol-with-cuda.cu:55-171, dispatcher gol-with-cuda.cu:302-327), applied to each
// logical row strip s of height hs and width W (per-rank mode: strip s == rank s's N x N tile):
//   0  all zeros                                   (gol-with-cuda.cu:56-69)
//   1  all ones                                    (gol-with-cuda.cu:72-92)
//   2  flat indices (hs-1)*W + 127 .. +136, clipped to the strip: the LAST row, columns 127..136,
//      on every strip                              (gol-with-cuda.cu:95-120, survey Q4)
//   3  strip 0: cells (0,0),(0,W-1); ELSE IF last strip: (hs-1,0),(hs-1,W-1)  (gol-with-cuda.cu:123-147)
//   4  strip 0: cells (0,0),(0,1),(0,W-1) by flat index (a blinker across the x-wrap)
//                                                  (gol-with-cuda.cu:150-171)
//   5  NEW: seeded counter-based random board (density 1/2), a pure function of (seed, global row,
//      global 64-cell word), hence identical for every decomposition and rank count.
// Any other value is rejected with the reference's message "Pattern %u has not been implemented \n".
#pragma once

#include <utility>
#include <vector>

#include "gol/geometry.hpp"

namespace gol {

enum class Fill { Zero, Ones, Random };

struct PatternSpec {
    unsigned pattern = 0;
    u64 seed = 0;
    Fill fill = Fill::Zero;
    std::vector<std::pair<i64, i64>> cells;  // extra live cells, global (row, col)
};

// Throws ContractError(255) with the reference message for unknown patterns.
PatternSpec make_pattern(unsigned pattern, const Decomposition& dec, u64 seed);

// Reference message for an unknown pattern (gol-with-cuda.cu:325).
std::string unknown_pattern_message(unsigned pattern);

}  // namespace gol
