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
//        T  = x0 + 2*(cy + u0 + 2*u1)
//   3. next = [T in {3,4}] & (x0 | alive)   (T == 3 is the odd one), where, in two 3-input steps,
//        g1 = exactly one of (x0, cy, u1)
//        [T in {3,4}] = (u0, u1, g1) in {(0,0,0), (0,1,1), (1,0,1)}
//      (an exhaustive search over 3-input gate circuits; it uses the don't-care "alive with T = 0",
//      impossible because T counts the centre.  The textbook form needs 4 steps here.)
// Every step is a 3-input boolean function, i.e. one v_bitop3_b32 on gfx950: 7 per word-half for
// the vertical sum and the rule, 2 for the row's horizontal sum.
#pragma once

#include "gol/common.hpp"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BITS_HD __host__ __device__ __forceinline__
#else
#define BITS_HD inline
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
constexpr unsigned kLutOne3 = lut3([](unsigned x0, unsigned cy, unsigned u1) {
    return (x0 & ~cy & ~u1) | (~x0 & cy & ~u1) | (~x0 & ~cy & u1);
});
constexpr unsigned kLutT34 = lut3([](unsigned u0, unsigned u1, unsigned g1) {
    return (~u0 & ~u1 & ~g1) | (~u0 & u1 & g1) | (u0 & ~u1 & g1);
});
constexpr unsigned kLutNext = lut3([](unsigned x0, unsigned alive, unsigned t34) { return t34 & (x0 | alive); });
static_assert(kLutOne3 == 0x16 && kLutT34 == 0x29 && kLutNext == 0xA8, "rule LUTs");

// Host/reference evaluation of a 3-input LUT on 64-bit words.
BITS_HD u64 bitop3_ref(u64 a, u64 b, u64 c, unsigned lut) {
    u64 r = 0;
    for (unsigned i = 0; i < 8; ++i) {
        if (!((lut >> i) & 1u)) continue;
        u64 ma = (i & 4u) ? a : ~a, mb = (i & 2u) ? b : ~b, mc = (i & 1u) ? c : ~c;
        r |= ma & mb & mc;
    }
    return r;
}

// ---------------------------------------------------------------------------------------------
// Storage format of a board word ("split"): the 64 cells of word c (columns 64c .. 64c+63) are
// stored with the EVEN columns in bits 0..31 (column 64c+2j at bit j) and the ODD columns in bits
// 32..63 (column 64c+2j+1 at bit 32+j).  An even cell's right neighbour is then the same bit of the
// odd half and an odd cell's left neighbour the same bit of the even half, so each 32-bit half
// needs ONE funnel shift for its horizontal neighbour sum instead of two.  Everything at word
// granularity (halos, plans, exchange, ghost words) is format-agnostic; only bit-level I/O
// (init, pattern cells, masks, dumps) converts with split_word / merge_word.
// ---------------------------------------------------------------------------------------------

BITS_HD u64 compact_even_bits(u64 x) {  // bits 0,2,4,.. -> 0..31
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
    return x;
}
BITS_HD u64 spread_even_bits(u64 x) {  // bits 0..31 -> 0,2,4,..
    x &= 0x00000000FFFFFFFFull;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}
// natural (bit b = column 64c+b) -> split storage
BITS_HD u64 split_word(u64 v) { return compact_even_bits(v) | (compact_even_bits(v >> 1) << 32); }
// split storage -> natural
BITS_HD u64 merge_word(u64 s) { return spread_even_bits(s) | (spread_even_bits(s >> 32) << 1); }
// storage bit of column c within its word
BITS_HD int storage_bit(i64 c) {
    const int b = (int)(c & 63);
    return (b & 1) ? 32 + (b >> 1) : (b >> 1);
}
// valid-cell mask of storage word c of a row of width w
BITS_HD u64 storage_mask(i64 c, i64 w) { return split_word(word_mask(c, w)); }

// Horizontal 3-sum (L + C + R, 2 bits per cell) of a split-format word given its row neighbours.
BITS_HD void hsum64(u64 prev, u64 cur, u64 next, u64& s0, u64& s1) {
    const u32 lo = (u32)cur, hi = (u32)(cur >> 32);
    const u32 prevhi = (u32)(prev >> 32), nextlo = (u32)next;
    const u32 Le = (hi << 1) | (prevhi >> 31);  // even cells: left = odd half shifted, right = odd half
    const u32 Ro = (lo >> 1) | (nextlo << 31);  // odd cells: left = even half, right = even half shifted
    const u32 s0e = Le ^ lo ^ hi, s1e = (Le & lo) | (Le & hi) | (lo & hi);
    const u32 s0o = lo ^ hi ^ Ro, s1o = (lo & hi) | (lo & Ro) | (hi & Ro);
    s0 = (u64)s0e | ((u64)s0o << 32);
    s1 = (u64)s1e | ((u64)s1o << 32);
}

// B3/S23 from three horizontal sums (rows above, centre, below) and the centre word.
BITS_HD u64 rule64(u64 a0, u64 a1, u64 b0, u64 b1, u64 c0, u64 c1, u64 x) {
    u64 x0 = a0 ^ b0 ^ c0;
    u64 cy = (a0 & b0) | (a0 & c0) | (b0 & c0);
    u64 u0 = a1 ^ b1 ^ c1;
    u64 u1 = (a1 & b1) | (a1 & c1) | (b1 & c1);
    u64 g1 = (x0 ^ cy ^ u1) & ~(x0 & cy & u1);    // kLutOne3
    u64 t34 = (g1 & (u0 ^ u1)) | ~(g1 | u0 | u1);  // kLutT34
    return t34 & (x0 | x);                          // kLutNext
}

// Word accessors for the bit-level helpers below: natural words as stored, or split-format
// storage words merged back to natural order on the fly.
struct NaturalRow {
    const u64* p;
    BITS_HD u64 operator[](i64 i) const { return p[i]; }
};
struct SplitRow {
    const u64* p;
    BITS_HD u64 operator[](i64 i) const { return merge_word(p[i]); }
};

// Extract `n` (1..64) bits (natural order) of a row starting at column s (no wrap; s + n <= w).
template <typename Row>
BITS_HD u64 extract_bits(Row row, i64 s, int n) {
    i64 i = s >> 6;
    int off = (int)(s & 63);
    u64 v = row[i] >> off;
    if (off && off + n > 64) v |= row[i + 1] << (64 - off);
    return n >= 64 ? v : (v & ((1ull << n) - 1ull));
}
BITS_HD u64 extract_bits(const u64* row, i64 s, int n) { return extract_bits(NaturalRow{row}, s, n); }

// 64 cells (natural order) of a periodic row of width w starting at (any) column `start`, i.e.
// columns start .. start+63 taken mod w.  Used to refresh the ghost bits of an x-periodic row.
template <typename Row>
BITS_HD u64 wrap64(Row row, i64 w, i64 start) {
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
BITS_HD u64 wrap64(const u64* row, i64 w, i64 start) { return wrap64(NaturalRow{row}, w, start); }

// Ghost words of one x-periodic row in split storage.  `row` points at word 0 of the row; words
// -1 and nw are the ghost words and columns >= w of word nw-1 are ghost cells.  Only cells in
// [0, w) are read.  (Word-aligned widths are a pure word copy, independent of the format.)
BITS_HD void wrap_row_ghosts(u64* row, i64 w, i64 nw) {
    int rem = (int)(w & 63);
    if (rem == 0) {
        u64 first = row[0], last = row[nw - 1];
        row[-1] = last;
        row[nw] = first;
        return;
    }
    const SplitRow src{row};
    u64 left = wrap64(src, w, -64);
    u64 tail = wrap64(src, w, w);  // columns w, w+1, ... (placed from bit rem upwards)
    u64 right = wrap64(src, w, 64 * nw);
    u64 keep = (1ull << rem) - 1ull;
    row[nw - 1] = split_word((merge_word(row[nw - 1]) & keep) | (tail << rem));
    row[-1] = split_word(left);
    row[nw] = split_word(right);
}

// Fingerprint contribution of one (masked) word at global word index `gidx`.  The fingerprint is
// the wrapping sum over all words, so it is independent of how the board is split across ranks.
BITS_HD u64 fingerprint_word(u64 gidx, u64 word) { return word ? mix64(mix64(gidx) ^ word) : 0ull; }

}  // namespace gol
