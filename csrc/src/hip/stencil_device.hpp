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
template <int K, int PH, bool GUARD>
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
        if (GUARD && i < 2 * l + 2) return false;
        lo = rule32(P.s0[l][spp][0], P.s1[l][spp][0], P.s0[l][sp][0], P.s1[l][sp][0], P.s0[l][s][0],
                    P.s1[l][s][0], P.x[l][sp][0]);
        hi = rule32(P.s0[l][spp][1], P.s1[l][spp][1], P.s0[l][sp][1], P.s1[l][sp][1], P.s0[l][s][1],
                    P.s1[l][s][1], P.x[l][sp][1]);
    }
    return true;
}

}  // namespace
}  // namespace hipk
}  // namespace gol
