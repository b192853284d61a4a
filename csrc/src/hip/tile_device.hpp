// gol-mi355x: the LDS tile kernels' device code (step_tile / step_tile_fold in step_kernels.hip): a
// workgroup of NW waves stages one tile of the plan plus its K-row halos into LDS with global_load_lds
// DMA and runs K generations LDS -> LDS, the last LDS pass storing to HBM.
#pragma once

#include "gol/bits.hpp"
#include "gol/hip_kernels.hpp"
#include "stencil_device.hpp"
#include "wave_runner.hpp"

namespace gol {
namespace hipk {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// ------------------------------------------------------------------------------------------
// step_tile: LDS-resident temporal blocking.  One workgroup of NW waves per plan wave: the plan
// wave's 64 lanes (segments + halo lanes, plan.hpp) define the tile columns and its `nrows` output
// rows; the tile plus K halo rows above and below (n_in = nrows + 2K rows x 64 lanes, split
// storage lo/hi planes, 512 B per row) is staged into LDS with global_load_lds DMA, then the
// K generations run LDS -> LDS: generation g computes rows [g+1, n_in-g-1), the NW waves each take
// a contiguous band of rows, stream it with a one-level register window (the same hsum/rule code
// as step_temporal), and a workgroup barrier separates generations.  The last generation stores
// straight to HBM.  Compared with step_temporal the vertical halo (2K rows) is shared by the NW
// waves of the tile instead of being paid by every wave, which is what small tiles (e.g. 8192^2,
// or a 32768^2 board strong-scaled over 8 GPUs) need; big tiles keep step_temporal (no barriers,
// no LDS traffic).  K is a runtime argument.
// ------------------------------------------------------------------------------------------
constexpr int kTileRowU32 = 128;  // one LDS row: 64 lo words then 64 hi words

template <bool LAST>
struct BandSink {
    static constexpr bool kLast = LAST;
    u32* lds;       // !LAST: destination buffer (row-major, kTileRowU32 per row)
    uint2* st;      // LAST: global store pointer of the band's first output row
    i64 st_stride;  // LAST: pitch, or 0 for halo/idle lanes (trash row)
    int row;        // !LAST: tile row of the next output
    int lane;
    __device__ __forceinline__ void put(u32 lo, u32 hi) {
        if constexpr (LAST) {
            *st = make_uint2(lo, hi);
            st += st_stride;
        } else {
            lds[row * kTileRowU32 + lane] = lo;
            lds[row * kTileRowU32 + 64 + lane] = hi;
            ++row;
        }
    }
};

// Input rows of a band: consecutive LDS rows (double-buffered tile), or (in-place tile) the band's
// LV halo rows above from a private copy, its own rows from the tile, its LV halo rows below from
// the copy.  Row indices are wave-uniform, so the select is scalar.
struct RowsLinear {
    const u32* base;
    __device__ __forceinline__ const u32* row(int i) const { return base + i * kTileRowU32; }
    __device__ __forceinline__ u32 lo(int i, int lane) const { return row(i)[lane]; }
    __device__ __forceinline__ u32 hi(int i, int lane) const { return row(i)[64 + lane]; }
};
struct RowsSplit {
    const u32* above;  // LV rows, then the rows below (and over-read slack)
    const u32* mid;    // the band's own rows in the tile
    int lv, m;         // halo depth, own rows
    __device__ __forceinline__ const u32* row(int i) const {
        return i < lv ? above + i * kTileRowU32
                      : (i < lv + m ? mid + (i - lv) * kTileRowU32 : above + (i - m) * kTileRowU32);
    }
    __device__ __forceinline__ u32 lo(int i, int lane) const { return row(i)[lane]; }
    __device__ __forceinline__ u32 hi(int i, int lane) const { return row(i)[64 + lane]; }
};

// Two register triples in the band loop for LDS passes of 4 levels (8192^2 tile@24: 1.457-1.494 ->
// 1.437-1.453 us/gen; no gain at 2 levels, profiles/pingpong_loop_ab.txt).
template <int LV>
constexpr bool tile_pingpong() {
    return LV >= 4;
}
// Stream input rows 0 .. n-1 of `in` (n >= 2*LV+1) through an LV-level register window (LV
// generations per LDS pass); outputs rows LV .. n-LV-1.
template <int LV, typename SRC, typename SINK>
__device__ __forceinline__ void tile_band(const SRC& in, int n, SINK& out, int lane) {
    Pipe<LV> P;
    u32 lo, hi;
#define TILE_ROW_STEP(PH, GUARD, IDX)                                   \
    lo = in.lo((IDX), lane);                                           \
    hi = in.hi((IDX), lane);                                           \
    if (advance<LV, PH, GUARD>(P, lo, hi, (IDX))) out.put(lo, hi);
    constexpr int i0 = ((2 * LV + 2) / 3) * 3;  // first multiple of 3 with the window full
    int i = 0;
    for (; i < i0; i += 3) {
        if (i < n) {
            TILE_ROW_STEP(0, true, i)
        }
        if (i + 1 < n) {
            TILE_ROW_STEP(1, true, i + 1)
        }
        if (i + 2 < n) {
            TILE_ROW_STEP(2, true, i + 2)
        }
    }
    // Steady state, software-pipelined: the next triple's LDS reads are issued before this triple's
    // compute, so their latency hides behind it (a workgroup of 8 waves leaves 2 waves per SIMD,
    // too few to hide it by switching waves: 35% of wave time was s_waitcnt, PMC at 8192^2).  The
    // last prefetch reads up to 3 rows past the band: still inside the tile buffers or the LDS slack
    // rows (tile_lds_bytes), and never used.
    u32 l0 = in.lo(i, lane), h0 = in.hi(i, lane);
    u32 l1 = in.lo(i + 1, lane), h1 = in.hi(i + 1, lane);
    u32 l2 = in.lo(i + 2, lane), h2 = in.hi(i + 2, lane);
    if constexpr (tile_pingpong<LV>()) {
        // Two register triples in turn (as in step_temporal's two-triple loop): each is refilled right
        // after its rows were computed, so no freshly read register is copied (a copy waits for the read
        // just issued, and with 2 waves per SIMD nothing else hides that latency).
        for (; i + 6 <= n; i += 6) {
            const u32 m0 = in.lo(i + 3, lane), g0 = in.hi(i + 3, lane);
            const u32 m1 = in.lo(i + 4, lane), g1 = in.hi(i + 4, lane);
            const u32 m2 = in.lo(i + 5, lane), g2 = in.hi(i + 5, lane);
            __builtin_amdgcn_sched_barrier(0);
            lo = l0, hi = h0;
            if (advance<LV, 0, false>(P, lo, hi, i)) out.put(lo, hi);
            lo = l1, hi = h1;
            if (advance<LV, 1, false>(P, lo, hi, i + 1)) out.put(lo, hi);
            lo = l2, hi = h2;
            if (advance<LV, 2, false>(P, lo, hi, i + 2)) out.put(lo, hi);
            l0 = in.lo(i + 6, lane), h0 = in.hi(i + 6, lane);
            l1 = in.lo(i + 7, lane), h1 = in.hi(i + 7, lane);
            l2 = in.lo(i + 8, lane), h2 = in.hi(i + 8, lane);
            __builtin_amdgcn_sched_barrier(0);
            lo = m0, hi = g0;
            if (advance<LV, 0, false>(P, lo, hi, i + 3)) out.put(lo, hi);
            lo = m1, hi = g1;
            if (advance<LV, 1, false>(P, lo, hi, i + 4)) out.put(lo, hi);
            lo = m2, hi = g2;
            if (advance<LV, 2, false>(P, lo, hi, i + 5)) out.put(lo, hi);
        }
    }
    for (; i + 3 <= n; i += 3) {
        const u32 a0 = l0, b0 = h0, a1 = l1, b1 = h1, a2 = l2, b2 = h2;
        l0 = in.lo(i + 3, lane), h0 = in.hi(i + 3, lane);
        l1 = in.lo(i + 4, lane), h1 = in.hi(i + 4, lane);
        l2 = in.lo(i + 5, lane), h2 = in.hi(i + 5, lane);
        __builtin_amdgcn_sched_barrier(0);
        lo = a0, hi = b0;
        if (advance<LV, 0, false>(P, lo, hi, i)) out.put(lo, hi);
        lo = a1, hi = b1;
        if (advance<LV, 1, false>(P, lo, hi, i + 1)) out.put(lo, hi);
        lo = a2, hi = b2;
        if (advance<LV, 2, false>(P, lo, hi, i + 2)) out.put(lo, hi);
    }
    if (i < n) {
        lo = l0, hi = h0;
        if (advance<LV, 0, false>(P, lo, hi, i)) out.put(lo, hi);
    }
    if (i + 1 < n) {
        lo = l1, hi = h1;
        if (advance<LV, 1, false>(P, lo, hi, i + 1)) out.put(lo, hi);
    }
#undef TILE_ROW_STEP
}

// Side rows per wave of the in-place tile: its 2*LV halo rows plus the band stream's over-read.
__host__ __device__ constexpr int tile_side_rows(int lv) { return 2 * lv + 4; }

// One LDS pass of `lv` generations: wave `wv` streams its band of the pass's output rows.
//   double-buffered (IP false): reads A, writes B.
//   in place (IP true): every wave first copies its band's LV halo rows above and below (rows other
//   waves are about to overwrite) into its private side rows, then, after a barrier, streams the band
//   and writes its output rows back into A.  A wave only ever writes its own band's rows and reads
//   other bands' rows only from its copy, so one tile buffer suffices: twice the rows per tile in the
//   160 KiB of LDS (one round of tiles where the double buffer needed two or three).
template <int NW, int LV, bool IP>
__device__ __forceinline__ void tile_pass(u32* A, u32* B, u32* side, u64* dst, const LaneDesc& d,
                                          const StepParams& p, int K, int g, int n_in, int wv, int lane, i64 trash_id) {
    const int lo_r = g + LV, cnt = n_in - 2 * g - 2 * LV;
    const int b = (cnt + NW - 1) / NW;
    const int r0 = lo_r + wv * b;
    const int r1 = min(r0 + b, lo_r + cnt);
    const int n = r1 - r0 + 2 * LV;
    u32* sw = side + wv * tile_side_rows(LV) * kTileRowU32;
    if constexpr (IP) {
        if (r1 > r0) {
#pragma unroll
            for (int j = 0; j < LV; ++j) {
                sw[j * kTileRowU32 + lane] = A[(r0 - LV + j) * kTileRowU32 + lane];
                sw[j * kTileRowU32 + 64 + lane] = A[(r0 - LV + j) * kTileRowU32 + 64 + lane];
                sw[(LV + j) * kTileRowU32 + lane] = A[(r1 + j) * kTileRowU32 + lane];
                sw[(LV + j) * kTileRowU32 + 64 + lane] = A[(r1 + j) * kTileRowU32 + 64 + lane];
            }
        }
        __syncthreads();  // every wave's copy is taken before any band is overwritten
    }
    if (r1 <= r0) return;
    auto stream = [&](auto& sink) {
        if constexpr (IP) {
            const RowsSplit in{sw, A + r0 * kTileRowU32, LV, r1 - r0};
            tile_band<LV>(in, n, sink, lane);
        } else {
            const RowsLinear in{A + (r0 - LV) * kTileRowU32};
            tile_band<LV>(in, n, sink, lane);
        }
    };
    if (g + LV < K) {
        BandSink<false> s{IP ? A : B, nullptr, 0, r0, lane};
        stream(s);
    } else {
        // tile row r0 is output row row0 + r0 - K; halo/idle lanes write their own trash word
        const bool out_lane = d.flags & LANE_STORE;
        uint2* st = out_lane ? reinterpret_cast<uint2*>(dst + (i64)(d.row0 + r0 - K + p.R) * p.pitch + (d.col + 1))
                             : reinterpret_cast<uint2*>(p.trash + ((trash_id * NW + wv) & (kTrashWaves - 1)) * 64 + lane);
        BandSink<true> s{nullptr, st, out_lane ? p.pitch : 0, 0, lane};
        stream(s);
    }
}


// One tile (plan wave `d` of this lane, nrows > 0): stage, K generations, store.
template <int NW, bool WRAPY, int LV, bool IP>
__device__ __forceinline__ void tile_item(const u64* __restrict__ src, u64* __restrict__ dst, const LaneDesc& d, int nrows,
                                          const StepParams& p, int K, u32* tile_lds, int wv, int lane, i64 trash_id) {
    const int n_in = nrows + 2 * K;
    u32* A = tile_lds;
    u32* B = tile_lds + n_in * kTileRowU32;  // double-buffered: the second tile buffer
    u32* side = tile_lds + n_in * kTileRowU32;  // in place: NW x tile_side_rows(LV) private rows

    // 1. stage rows row0-K .. row0+nrows+K-1 (two 4-byte DMAs per row: lo plane, hi plane)
    for (int i = wv; i < n_in; i += NW) {
        int r = d.row0 - K + i;
        if (WRAPY) r = r < 0 ? r + p.h : (r >= p.h ? r - p.h : r);
        const u32* g = reinterpret_cast<const u32*>(src + (i64)(r + p.R) * p.pitch + (d.col + 1));
        u32* l = A + i * kTileRowU32;
        __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)l, 4, 0, 0);
        __builtin_amdgcn_global_load_lds((glb_void_t*)(g + 1), (lds_void_t*)(l + 64), 4, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // 2. K generations in LDS passes of up to LV levels (the last passes take what is left); the pass
    // starting at generation g with lv levels computes tile rows [g+lv, n_in-g-lv).  More levels per
    // pass: more independent work per wave (the level pipeline) and fewer barriers, at 2*lv rows of
    // band overlap per wave.
    for (int g = 0; g < K;) {
        const int left = K - g;
        int lv = 1;
        if (LV >= 4 && left >= 4) {
            lv = 4;
            tile_pass<NW, (LV >= 4 ? 4 : 1), IP>(A, B, side, dst, d, p, K, g, n_in, wv, lane, trash_id);
        } else if (LV >= 2 && left >= 2) {
            lv = 2;
            tile_pass<NW, (LV >= 2 ? 2 : 1), IP>(A, B, side, dst, d, p, K, g, n_in, wv, lane, trash_id);
        } else {
            tile_pass<NW, 1, IP>(A, B, side, dst, d, p, K, g, n_in, wv, lane, trash_id);
        }
        g += lv;
        if (g < K) {
            __syncthreads();
            if constexpr (!IP) {
                u32* t = A;
                A = B;
                B = t;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// step_tile_fold (STEP_TILE_FOLD): the tile kernel with the tile folded in half.  A tile is 32 lanes
// wide (<= 30 output words + 2 halo lanes, plan.hpp fold plans) and twice as tall: lanes 0-31 stream
// its top half downwards, lanes 32-63 its bottom half upwards (B3/S23 is symmetric, so the level
// pipeline runs unchanged in either direction).  Virtual row j is tile row j for half 0 and tile row
// T-1-j for half 1 (T = nrows + 2K staged rows, Th = ceil(T/2)); generation g computes virtual rows
// [g+1, Th) in both halves, so the trapezoid shrinks at the tile's two outer edges only and its
// vertical halo (2K rows) is paid over twice the output rows: at 8192^2, K=24 the computed rows per
// output row drop from ~1.35 (68-row tiles) to ~1.17 (139-row tiles) at ~4% more halo lanes.
//
// LDS row j holds virtual row j of both halves in the tile kernel's layout ([lo of lanes 0-63][hi of
// lanes 0-63]), so the band stream and its sinks are step_tile's, with no per-lane row arithmetic.
// Where the halves meet, a band reads LV virtual rows past Th: row Th+x of half 0 is tile row Th+x,
// i.e. half 1's virtual row T-1-Th-x, and vice versa.  Those rows are kept as mirrors: staged with
// the same formula, and every pass that writes virtual row v in [T-Th-4, T-1-Th] also writes it to
// row T-1-v in the other half's lanes (lane ^ 32), so no lane ever reads another half's slot.
// ------------------------------------------------------------------------------------------
constexpr int kFoldMirror = 4;  // mirrored rows past the middle (the deepest LDS pass, LV <= 4)

struct FoldSink {
    static constexpr bool kLast = false;
    u32* lds;
    int row;     // virtual row of the next output
    int lane;
    int m_lo;    // rows m_lo .. tm1 - Th are mirrored to row tm1 - row
    int m_hi;
    int tm1;     // T - 1
    __device__ __forceinline__ void put(u32 lo, u32 hi) {
        lds[row * kTileRowU32 + lane] = lo;
        lds[row * kTileRowU32 + 64 + lane] = hi;
        if (row >= m_lo && row <= m_hi) {  // wave-uniform
            const int m = tm1 - row;
            lds[m * kTileRowU32 + (lane ^ 32)] = lo;
            lds[m * kTileRowU32 + 64 + (lane ^ 32)] = hi;
        }
        ++row;
    }
};

// LDS rows of one buffer of a folded tile: Th rows, the mirrors, and the band stream's over-read
__host__ __device__ constexpr int fold_buffer_rows(int T) { return (T + 1) / 2 + kFoldMirror + 4; }

// One LDS pass of a folded tile: double-buffered (IP false: reads A, writes B) or in place (IP true:
// as step_tile's in-place pass, each wave first copies its band's LV rows above and below into its
// side rows; the mirrors past the middle are such rows for the middle band, so they too are read from
// the copy while the pass rewrites them).
template <int NW, int LV, bool IP>
__device__ __forceinline__ void fold_pass(u32* A, u32* B, u32* side, u64* dst, const LaneDesc& d, const StepParams& p,
                                          int K, int g, int T, int wv, int lane, i64 trash_id) {
    const int Th = (T + 1) / 2;
    const int lo_r = g + LV, cnt = Th - g - LV;
    const int b = (cnt + NW - 1) / NW;
    const int r0 = lo_r + wv * b;
    const int r1 = min(r0 + b, lo_r + cnt);
    const int n = r1 - r0 + 2 * LV;
    u32* sw = side + wv * tile_side_rows(LV) * kTileRowU32;
    if constexpr (IP) {
        if (r1 > r0) {
#pragma unroll
            for (int j = 0; j < LV; ++j) {
                sw[j * kTileRowU32 + lane] = A[(r0 - LV + j) * kTileRowU32 + lane];
                sw[j * kTileRowU32 + 64 + lane] = A[(r0 - LV + j) * kTileRowU32 + 64 + lane];
                sw[(LV + j) * kTileRowU32 + lane] = A[(r1 + j) * kTileRowU32 + lane];
                sw[(LV + j) * kTileRowU32 + 64 + lane] = A[(r1 + j) * kTileRowU32 + 64 + lane];
            }
        }
        __syncthreads();  // every wave's copy is taken before any band is overwritten
    }
    if (r1 <= r0) return;
    auto stream = [&](auto& sink) {
        if constexpr (IP) {
            const RowsSplit in{sw, A + r0 * kTileRowU32, LV, r1 - r0};
            tile_band<LV>(in, n, sink, lane);
        } else {
            const RowsLinear in{A + (r0 - LV) * kTileRowU32};
            tile_band<LV>(in, n, sink, lane);
        }
    };
    if (g + LV < K) {
        FoldSink sk{IP ? A : B, r0, lane, T - Th - kFoldMirror, T - 1 - Th, T - 1};
        stream(sk);
    } else {
        // virtual row r0 is tile row t0, output row row0 + t0 - K; half 1 stores upwards
        const int half = lane >> 5;
        const int t0 = half ? T - 1 - r0 : r0;
        const bool out_lane = d.flags & LANE_STORE;
        uint2* st = out_lane ? reinterpret_cast<uint2*>(dst + (i64)(d.row0 + t0 - K + p.R) * p.pitch + (d.col + 1))
                             : reinterpret_cast<uint2*>(p.trash + ((trash_id * NW + wv) & (kTrashWaves - 1)) * 64 + lane);
        BandSink<true> sk{nullptr, st, out_lane ? (half ? -p.pitch : p.pitch) : 0, 0, lane};
        stream(sk);
    }
}

// One folded tile (lanes 32-63 of `d` repeat lanes 0-31; nrows > 0).
template <int NW, bool WRAPY, int LV, bool IP>
__device__ __forceinline__ void fold_item(const u64* __restrict__ src, u64* __restrict__ dst, const LaneDesc& d, int nrows,
                                          const StepParams& p, int K, u32* tile_lds, int wv, int lane, i64 trash_id) {
    const int T = nrows + 2 * K;
    const int nb = fold_buffer_rows(T);
    u32* A = tile_lds;
    u32* B = tile_lds + nb * kTileRowU32;     // double-buffered: the second buffer
    u32* side = tile_lds + nb * kTileRowU32;  // in place: NW x tile_side_rows(LV) private rows

    // 1. stage LDS rows 0 .. Th+kFoldMirror+3: row j = tile row j (half 0) / T-1-j (half 1), tile row t
    //    being board row row0-K+t; two 4-byte DMAs per row (lo plane, hi plane)
    const int half = lane >> 5;
    for (int i = wv; i < nb; i += NW) {
        const int t = half ? T - 1 - i : i;
        int r = d.row0 - K + t;
        if (WRAPY) r = r < 0 ? r + p.h : (r >= p.h ? r - p.h : r);
        const u32* g = reinterpret_cast<const u32*>(src + (i64)(r + p.R) * p.pitch + (d.col + 1));
        u32* l = A + i * kTileRowU32;
        __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)l, 4, 0, 0);
        __builtin_amdgcn_global_load_lds((glb_void_t*)(g + 1), (lds_void_t*)(l + 64), 4, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // 2. K generations in LDS passes of up to LV levels, as step_tile
    for (int g = 0; g < K;) {
        const int left = K - g;
        int lv = 1;
        if (LV >= 4 && left >= 4) {
            lv = 4;
            fold_pass<NW, (LV >= 4 ? 4 : 1), IP>(A, B, side, dst, d, p, K, g, T, wv, lane, trash_id);
        } else if (LV >= 2 && left >= 2) {
            lv = 2;
            fold_pass<NW, (LV >= 2 ? 2 : 1), IP>(A, B, side, dst, d, p, K, g, T, wv, lane, trash_id);
        } else {
            fold_pass<NW, 1, IP>(A, B, side, dst, d, p, K, g, T, wv, lane, trash_id);
        }
        g += lv;
        if (g < K) {
            __syncthreads();
            if constexpr (!IP) {
                u32* t = A;
                A = B;
                B = t;
            }
        }
    }
}

inline int tile_levels(u32 flags) { return (flags & STEP_TILE_L4) ? 4 : ((flags & STEP_TILE_L2) ? 2 : 1); }

// LDS rows of a tile with `rows` output rows at depth k: double-buffered, two copies of the tile
// (+4 rows of over-read slack); in place, one copy plus NW private side rows per wave.
inline i64 tile_lds_rows(i64 rows, int k, int nw, u32 flags) {
    if (flags & STEP_TILE_FOLD)
        return (flags & STEP_TILE_INPLACE)
                   ? (i64)fold_buffer_rows((int)(rows + 2 * (i64)k)) + (i64)nw * tile_side_rows(tile_levels(flags))
                   : 2 * (i64)fold_buffer_rows((int)(rows + 2 * (i64)k));
    if (flags & STEP_TILE_INPLACE) return rows + 2 * (i64)k + (i64)nw * tile_side_rows(tile_levels(flags));
    return 2 * (rows + 2 * (i64)k) + 4;
}
inline size_t tile_lds_bytes(i64 rows, int k, int nw, u32 flags) {
    return (size_t)tile_lds_rows(rows, k, nw, flags) * kTileRowU32 * 4;
}

}  // namespace
}  // namespace hipk
}  // namespace gol
