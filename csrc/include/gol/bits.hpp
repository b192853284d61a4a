// gol-mi355x: bit-sliced Game of Life arithmetic shared by the CPU stepper and the HIP kernels.
//
// Rule (reference gol-with-cuda.cu:239-257): an alive cell survives with 2 or 3 live neighbours,
// a dead cell is born with exactly 3 — B3/S23.  With T = the 3x3 block sum *including* the centre
// this is   next = (T == 3) | (alive & (T == 4)).
//
// Bit-sliced evaluation for 64 (or 32) cells at once:
//   1. per row, the horizontal sum h = left + centre + right  (2 bits: s0 = xor3, s1 = maj)
//   2. T = h(row-1) + h(row) + h(row+1):
//        x0 = xor3(s0's), cy = maj(s0's), u0 = xor3(s1's), u1 = maj(s1's)
//        T  = x0 + 2*(cy + u0 + 2*u1) = x0 + 2*y
//      T == 3  <=>  x0 & (y == 1)  <=>  x0 & ~u1 & (u0 ^ cy)
//      T == 4  <=> ~x0 & (y == 2)  <=> ~x0 & (u1 ? ~u0 & ~cy : u0 & cy)
// Every step is a 3-input boolean function, i.e. one v_bitop3_b32 on gfx950.
#pragma once

#include "gol/common.hpp"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GOL_HD __host__ __device__ __forceinline__
#else
#define GOL_HD inline
#endif

namespace gol {

// 8-bit truth table of a 3-input boolean function, in v_bitop3's operand convention
// (operand a = 0xF0, b = 0xCC, c = 0xAA).
template <typename F>
constexpr unsigned lut3(F f) {
    return (unsigned)(f(0xF0u, 0xCCu, 0xAAu) & 0xFFu);
}

constexpr unsigned kLutXor3 = 0x96;  // a ^ b ^ c
constexpr unsigned kLutMaj = 0xE8;   // majority(a, b, c)
constexpr unsigned kLutY1 = lut3([](unsigned u1, unsigned u0, unsigned cy) { return ~u1 & (u0 ^ cy); });
constexpr unsigned kLutY2 = lut3([](unsigned u1, unsigned u0, unsigned cy) {
    return (u1 & ~u0 & ~cy) | (~u1 & u0 & cy);
});
constexpr unsigned kLutBorn4 = lut3([](unsigned x0, unsigned x, unsigned y2) { return ~x0 & x & y2; });
constexpr unsigned kLutOut = lut3([](unsigned x0, unsigned y1, unsigned t) { return (x0 & y1) | t; });

// Host/reference evaluation of a 3-input LUT on 64-bit words.
GOL_HD u64 bitop3_ref(u64 a, u64 b, u64 c, unsigned lut) {
    u64 r = 0;
    for (unsigned i = 0; i < 8; ++i) {
        if (!((lut >> i) & 1u)) continue;
        u64 ma = (i & 4u) ? a : ~a, mb = (i & 2u) ? b : ~b, mc = (i & 1u) ? c : ~c;
        r |= ma & mb & mc;
    }
    return r;
}

// Horizontal 3-sum of a 64-cell word given its neighbouring words in the row.
GOL_HD void hsum64(u64 prev, u64 cur, u64 next, u64& s0, u64& s1) {
    u64 L = (cur << 1) | (prev >> 63);
    u64 R = (cur >> 1) | (next << 63);
    s0 = L ^ cur ^ R;
    s1 = (L & cur) | (L & R) | (cur & R);
}

// B3/S23 from three horizontal sums (rows above, centre, below) and the centre word.
GOL_HD u64 rule64(u64 a0, u64 a1, u64 b0, u64 b1, u64 c0, u64 c1, u64 x) {
    u64 x0 = a0 ^ b0 ^ c0;
    u64 cy = (a0 & b0) | (a0 & c0) | (b0 & c0);
    u64 u0 = a1 ^ b1 ^ c1;
    u64 u1 = (a1 & b1) | (a1 & c1) | (b1 & c1);
    u64 y1 = ~u1 & (u0 ^ cy);
    u64 y2 = (u1 & ~u0 & ~cy) | (~u1 & u0 & cy);
    return (x0 & y1) | (~x0 & x & y2);
}

// Extract `n` (1..64) bits of a row starting at column s (no wrap; s + n <= row width).
GOL_HD u64 extract_bits(const u64* row, i64 s, int n) {
    i64 i = s >> 6;
    int off = (int)(s & 63);
    u64 v = row[i] >> off;
    if (off && off + n > 64) v |= row[i + 1] << (64 - off);
    return n >= 64 ? v : (v & ((1ull << n) - 1ull));
}

// 64 cells of a periodic row of width w starting at (any) column `start`, i.e. columns
// start .. start+63 taken mod w.  Used to refresh the ghost bits of an x-periodic row.
GOL_HD u64 wrap64(const u64* row, i64 w, i64 start) {
    i64 s = start % w;
    if (s < 0) s += w;
    u64 res = 0;
    int got = 0;
    while (got < 64) {
        i64 avail = w - s;
        int n = (int)(avail < (i64)(64 - got) ? avail : (i64)(64 - got));
        res |= extract_bits(row, s, n) << got;
        got += n;
        s = 0;
    }
    return res;
}

// Ghost words of one x-periodic row.  `row` points at word 0 of the row; words -1 and nw are the
// ghost words and bits >= w%64 of word nw-1 are ghost bits.  Only cells in [0, w) are read.
GOL_HD void wrap_row_ghosts(u64* row, i64 w, i64 nw) {
    int rem = (int)(w & 63);
    if (rem == 0) {
        u64 first = row[0], last = row[nw - 1];
        row[-1] = last;
        row[nw] = first;
        return;
    }
    u64 left = wrap64(row, w, -64);
    u64 tail = wrap64(row, w, w);  // columns w, w+1, ... (placed from bit rem upwards)
    u64 right = wrap64(row, w, 64 * nw);
    u64 keep = (1ull << rem) - 1ull;
    row[nw - 1] = (row[nw - 1] & keep) | (tail << rem);
    row[-1] = left;
    row[nw] = right;
}

// Fingerprint contribution of one (masked) word at global word index `gidx`.  The fingerprint is
// the wrapping sum over all words, so it is independent of how the board is split across ranks.
GOL_HD u64 fingerprint_word(u64 gidx, u64 word) { return word ? mix64(mix64(gidx) ^ word) : 0ull; }

}  // namespace gol
