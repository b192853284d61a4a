// gol-mi355x: device building blocks of the B3/S23 kernels (step_kernels.hip, resident_kernel.hip).
//
// Bit-sliced arithmetic on split-format words (bits.hpp: lo = the 32 even columns, hi = the 32 odd
// columns of a 64-cell word, one word column per lane): v_bitop3_b32 three-input gates, DPP
// wave_shr/shl lane moves and v_alignbit_b32 funnel shifts.  11 VALU ops per 32 cells per generation.
#pragma once

#include <hip/hip_runtime.h>

#include "gol/bits.hpp"

namespace gol {
namespace hipk {
namespace {

template <unsigned LUT>
__device__ __forceinline__ u32 b3(u32 a, u32 b, u32 c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, LUT);
}

// lane i <- lane i-1 (lane 0 gets 0: bound_ctrl)
__device__ __forceinline__ u32 dpp_prev(u32 v) {
    return (u32)__builtin_amdgcn_mov_dpp((int)v, 0x138 /*wave_shr:1*/, 0xF, 0xF, true);
}
// lane i <- lane i+1 (lane 63 gets 0: bound_ctrl)
__device__ __forceinline__ u32 dpp_next(u32 v) {
    return (u32)__builtin_amdgcn_mov_dpp((int)v, 0x130 /*wave_shl:1*/, 0xF, 0xF, true);
}

__device__ __forceinline__ u32 rule32(u32 a0, u32 a1, u32 b0, u32 b1, u32 c0, u32 c1, u32 x) {
    const u32 x0 = b3<kLutXor3>(a0, b0, c0);
    const u32 cy = b3<kLutMaj>(a0, b0, c0);
    const u32 u0 = b3<kLutXor3>(a1, b1, c1);
    const u32 u1 = b3<kLutMaj>(a1, b1, c1);
    const u32 g1 = b3<kLutOne3>(x0, cy, u1);
    const u32 t34 = b3<kLutT34>(u0, u1, g1);
    return b3<kLutNext>(x0, x, t34);
}

// Horizontal 3-sums of one split-format word (bits.hpp: lo = even columns, hi = odd columns).
// Even cell j: left = odd cell j-1 (hi shifted up one, bit 0 from the previous lane's hi), right =
// odd cell j (hi).  Odd cell j: left = even cell j (lo), right = even cell j+1 (lo shifted down one,
// bit 31 from the next lane's lo).  2 DPP + 2 funnel shifts + 4 bitop3 per 64 cells.
__device__ __forceinline__ void hsum_split(u32 lo, u32 hi, u32& s0lo, u32& s1lo, u32& s0hi, u32& s1hi) {
    const u32 ph = dpp_prev(hi), nl = dpp_next(lo);
    const u32 Le = __builtin_amdgcn_alignbit(hi, ph, 31);  // (hi << 1) | (ph >> 31)
    const u32 Ro = __builtin_amdgcn_alignbit(nl, lo, 1);   // (lo >> 1) | (nl << 31)
    s0lo = b3<kLutXor3>(Le, lo, hi);
    s1lo = b3<kLutMaj>(Le, lo, hi);
    s0hi = b3<kLutXor3>(lo, hi, Ro);
    s1hi = b3<kLutMaj>(lo, hi, Ro);
}

// Pair-shared vertical sums (round 6).  Two vertically adjacent output rows share two of their three input
// rows, so a level can add the horizontal sums of an input row PAIR once, P = a + b in 0..6 (3 planes,
// 4 gates), and finish each of the two outputs from P, the third row's sum c and the centre cell in 4
// gates.  The finish, found by an exhaustive search over circuits of 3-input gates (tools/rule_search.c
// pair mode; no 3-gate finish exists) and checked on every input, with T = P + c (centre included):
//   g1 = f43(p0, c0, x)   g3 = f25(p1, p2, c1)   g2 = f27(p2, x, g1)   next = f42(g3, g1, g2)
// It uses only the don't-care "alive with T = 0", so the same circuit serves the output whose centre is
// the pair's upper row and the one whose centre is its lower row.
// The row loops of every kernel are unrolled by 3 (the ring slot of a row is a compile-time constant), so
// the pairs follow the slots: of the outputs centred on rows 3m, 3m+1, 3m+2 of a level, the first two
// share the pair (3m, 3m+1) and the third takes rule32: 4 + 4 + 4 + 7 = 19 v_bitop3 per word-half and
// row triple instead of 21 (20.7 instead of 22 VALU per 64 cells and generation).  (Pairing every output
// needs a row phase mod 6; unrolled by 6, the steady loops of step_temporal took 277-308 VGPRs at K = 8
// against 162.)
// Where it runs (PAIR): the LDS tile kernels' band stream and step_pipe's stages, where it measured faster
// (kbench, interleaved on one box: 8192^2 folded tile@32 1.373-1.381 -> 1.322-1.329 us/gen, 4096 x 32768
// step_pipe 10 x 2 2.351-2.363 -> 2.320-2.342, 32768^2 step_pipe 8 x 3 10.16-10.18 -> 9.88-9.90;
// profiles/pair_rule_round6.txt).  Not in step_temporal: its K = 8 loop issues 510 instead of 542 VALU
// and no s_nop, yet ran 10.55 -> 13.1 us/gen at 32768^2 (two halves 9.3 -> 11.4): the compiler's issue
// order of the level chains, not the instruction count, limits that loop (docs/PERFORMANCE.md §2).
#ifndef GOL_RULE_PAIR
#define GOL_RULE_PAIR 1
#endif
constexpr bool kRulePair = GOL_RULE_PAIR != 0;
constexpr unsigned kLutF1 = 0x43, kLutF2 = 0x27, kLutF3 = 0x25, kLutF4 = 0x42;

__device__ __forceinline__ void pair_sum(u32 a0, u32 a1, u32 b0, u32 b1, u32& p0, u32& p1, u32& p2) {
    const u32 t = a0 & b0;
    p0 = a0 ^ b0;
    p1 = b3<kLutXor3>(a1, b1, t);
    p2 = b3<kLutMaj>(a1, b1, t);
}
__device__ __forceinline__ u32 finish32(u32 p0, u32 p1, u32 p2, u32 c0, u32 c1, u32 x) {
    const u32 g1 = b3<kLutF1>(p0, c0, x);
    const u32 g3 = b3<kLutF3>(p1, p2, c1);
    const u32 g2 = b3<kLutF2>(p2, x, g1);
    return b3<kLutF4>(g3, g1, g2);
}

// The K-level register pipeline of the streaming kernels (step_temporal, step_tile's band stream,
// step_pipe's stages): level l keeps a 3-row window of horizontal sums and centre rows.
template <int K>
struct Pipe {
    u32 s0[K][3][2];  // horizontal sum bit 0, per level, ring slot, half
    u32 s1[K][3][2];  // horizontal sum bit 1
    u32 x[K][3][2];   // the level's input rows (centre cells)
};

// Push one row (lo, hi) through the K levels.  Input index i (0-based within the segment's input
// rows).  PH == i % 3 selects the ring slots at compile time.  Returns false while the pipeline is
// still filling (GUARD instantiation only); otherwise (lo, hi) is the output row i - 2K.
// Level l sees its input row j = i - 2l, in slot s = j % 3 = (PH + l) % 3.  Pair mode: row j of slot 1
// completes the pair (j-1, j) and gives output j-1 with c = row j-2; row j of slot 2 gives output j-1 from
// the same pair with c = row j; row j of slot 0 gives output j-1 with rule32.
template <int K, int PH, bool GUARD, bool PAIR = kRulePair>
__device__ __forceinline__ bool advance(Pipe<K>& P, u32& lo, u32& hi, int i) {
#pragma unroll
    for (int l = 0; l < K; ++l) {
        if (GUARD && i < 2 * l) return false;
        const int s = (PH + l) % 3;     // slot of the arriving row
        const int sp = (s + 2) % 3;     // previous row (centre of the output)
        const int spp = (s + 1) % 3;    // two rows back
        hsum_split(lo, hi, P.s0[l][s][0], P.s1[l][s][0], P.s0[l][s][1], P.s1[l][s][1]);
        P.x[l][s][0] = lo;
        P.x[l][s][1] = hi;
        // Pair mode keeps the pair's three planes in slot 0's entries (sums and centre row), which are dead
        // from the slot-1 row's output (centred on slot 0's row) until the next slot-0 row arrives: no
        // registers beyond the ring (separate planes took 208 instead of 162 VGPRs at K = 8).
        if (PAIR && s == 1) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                u32 p0, p1, p2;
                pair_sum(P.s0[l][0][h], P.s1[l][0][h], P.s0[l][1][h], P.s1[l][1][h], p0, p1, p2);
                if (!(GUARD && i < 2 * l + 2)) {
                    const u32 o = finish32(p0, p1, p2, P.s0[l][2][h], P.s1[l][2][h], P.x[l][0][h]);
                    if (h == 0) lo = o; else hi = o;
                }
                P.s0[l][0][h] = p0;
                P.s1[l][0][h] = p1;
                P.x[l][0][h] = p2;
            }
            if (GUARD && i < 2 * l + 2) return false;
            continue;
        }
        if (GUARD && i < 2 * l + 2) return false;
        if (PAIR && s == 2) {  // the pair (slot 0's entries), c = this row, centre = slot 1's row
            lo = finish32(P.s0[l][0][0], P.s1[l][0][0], P.x[l][0][0], P.s0[l][2][0], P.s1[l][2][0], P.x[l][1][0]);
            hi = finish32(P.s0[l][0][1], P.s1[l][0][1], P.x[l][0][1], P.s0[l][2][1], P.s1[l][2][1], P.x[l][1][1]);
        } else {
            lo = rule32(P.s0[l][spp][0], P.s1[l][spp][0], P.s0[l][sp][0], P.s1[l][sp][0], P.s0[l][s][0],
                        P.s1[l][s][0], P.x[l][sp][0]);
            hi = rule32(P.s0[l][spp][1], P.s1[l][spp][1], P.s0[l][sp][1], P.s1[l][sp][1], P.s0[l][s][1],
                        P.s1[l][s][1], P.x[l][sp][1]);
        }
    }
    return true;
}

}  // namespace
}  // namespace hipk
}  // namespace gol
