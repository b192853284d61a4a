// gol-mi355x: pattern placement (see pattern.hpp for the semantics and reference citations).
#include "gol/pattern.hpp"

namespace gol {

std::string unknown_pattern_message(unsigned pattern) {
    return strprintf("Pattern %u has not been implemented \n", pattern);
}

PatternSpec make_pattern(unsigned pattern, const Decomposition& dec, u64 seed) {
    PatternSpec p;
    p.pattern = pattern;
    p.seed = seed;
    const i64 W = dec.W;
    const int S = (int)dec.strip_starts.size() - 1;
    // Flat index inside strip s -> global cell, clipped to the strip like the reference's buffer.
    auto add_flat = [&](int s, i64 flat) {
        i64 hs = dec.strip_starts[s + 1] - dec.strip_starts[s];
        if (flat < 0 || flat >= hs * W) return;
        p.cells.push_back({dec.strip_starts[s] + flat / W, flat % W});
    };
    switch (pattern) {
        case 0:
            p.fill = Fill::Zero;
            break;
        case 1:
            p.fill = Fill::Ones;
            break;
        case 2:
            for (int s = 0; s < S; ++s) {
                i64 hs = dec.strip_starts[s + 1] - dec.strip_starts[s];
                i64 row_offset = (hs - 1) * W;
                for (i64 j = 127; j < 137; ++j)
                    if (row_offset + j < hs * W) add_flat(s, row_offset + j);
            }
            break;
        case 3: {
            add_flat(0, 0);
            add_flat(0, W - 1);
            if (S > 1) {  // "else if (myRank == numRank - 1)": never for strip 0 itself
                i64 hs = dec.strip_starts[S] - dec.strip_starts[S - 1];
                add_flat(S - 1, (hs - 1) * W);
                add_flat(S - 1, (hs - 1) * W + W - 1);
            }
            break;
        }
        case 4:
            add_flat(0, 0);
            add_flat(0, 1);
            add_flat(0, W - 1);
            break;
        case 5:
            p.fill = Fill::Random;
            break;
        default:
            throw ContractError(unknown_pattern_message(pattern), 255);
    }
    return p;
}

}  // namespace gol
