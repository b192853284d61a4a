// gol-mi355x: the B3/S23 stencil kernels for gfx950 (CDNA4).
//
// step_temporal<K> — the hot kernel.  Design (MI355X-first, not a port of gol_kernel,
// reference gol-with-cuda.cu:189-262, which reads 9 bytes per cell per generation from global memory):
//
//  * 1 bit per cell, 64 cells per lane: each lane owns one u64 word column of the tile (two VGPRs,
//    split storage: lo = the 32 even columns, hi = the 32 odd columns, bits.hpp) and streams DOWN
//    the rows.  A wave64 covers 64 adjacent words = 4096 cells per row; the work plan (plan.hpp)
//    packs segments of <= 62 output words plus one halo lane on each side into the 64 lanes.
//  * Horizontal neighbours: with split storage an even cell's right neighbour and an odd cell's
//    left neighbour are the same bit of the other half, so per 64 cells only two neighbour words
//    are shifted: the previous lane's hi (v_mov_b32_dpp wave_shr:1) funnelled into hi, and the next
//    lane's lo (wave_shl:1) funnelled into lo, one v_alignbit_b32 each — no LDS, no barriers.
//  * Bit-sliced counting: per row the horizontal 3-sum (xor3 / maj = 1 v_bitop3 each), then the
//    vertical 3-sum of those 2-bit sums and the rule in 7 more v_bitop3 (bits.hpp): 11 VALU ops per
//    32 cells per generation (12 with natural bit order, which needs 4 funnel shifts per word).
//  * Temporal blocking: K generation levels are chained in registers.  Level l keeps a 3-row
//    window (horizontal sums of rows r-2, r-1 and its centre row); when a row arrives at level l it
//    emits row r-1 of generation l+1 to level l+1.  One HBM pass = K generations, so the kernel is
//    VALU bound instead of HBM bound (0.25 B/cell/pass / K).  The window rotates by unrolling the
//    row loop x3, so there are no register moves.
//  * Halo semantics: a segment reads K rows above/below its output rows and the two halo words;
//    invalid bits spread one column per generation from the halo lanes' outer edges, so the output
//    lanes are exact for K <= 64.
//  * Periodic wrap without ghost traffic: when the tile is its own E/W neighbour the plan points the
//    edge segments' halo lanes at word nw-1 / word 0 (x-wrap), and when it is its own N/S neighbour
//    the load stream addresses rows modulo h (STEP_WRAP_Y).  A single-GPU run therefore needs no
//    ghost rows, ghost words, halo kernels or copies at all.
//
// step_lds — single-generation LDS-tiled variant: a 256-thread workgroup stages a (16+2) x (64+2)
// word tile + ghost ring in LDS and computes 16 x 64 output words.  Kept as a measured alternative.
#include <mutex>
#include <set>
#include <utility>

#include "gol/bits.hpp"
#include "gol/hip_kernels.hpp"
#include "stencil_device.hpp"
#include "wave_runner.hpp"

namespace gol {
namespace hipk {

namespace {

template <int K, int ROWS>
__global__ __launch_bounds__(64 * kWavesPerBlock) void step_temporal(const u64* __restrict__ src, u64* __restrict__ dst,
                                                                      const LaneDesc* __restrict__ plan, StepParams p) {
    const int wv = threadIdx.x >> 6;
    const i64 wave = (i64)blockIdx.x * kWavesPerBlock + wv;
    const int lane = threadIdx.x & 63;
    const LaneDesc d = plan[wave * kWaveLanes + lane];
    const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
    if (nrows <= 0) return;  // padding wave (uniform)
    WaveRunner<K, ROWS> w(src, dst, d, nrows, p, wave);
    w.run();
}

template <int K>
const void* kernel_for(u32 flags) {
    if (flags & STEP_SEAM) return (const void*)step_temporal<K, ROWS_SEAM>;
    return (flags & STEP_WRAP_Y) ? (const void*)step_temporal<K, ROWS_WRAP> : (const void*)step_temporal<K, ROWS_GHOST>;
}

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
                                          const StepParams& p, int K, int g, int n_in, int wv, int lane) {
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
                             : reinterpret_cast<uint2*>(p.trash + ((i64)((blockIdx.x * NW + wv) & (kTrashWaves - 1)) * 64 + lane));
        BandSink<true> s{nullptr, st, out_lane ? p.pitch : 0, 0, lane};
        stream(s);
    }
}


template <int NW, bool WRAPY, int LV, bool IP>
__global__ __launch_bounds__(64 * NW) void step_tile(const u64* __restrict__ src, u64* __restrict__ dst,
                                                     const LaneDesc* __restrict__ plan, StepParams p, int K) {
    extern __shared__ __attribute__((aligned(16))) u32 tile_lds[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaneDesc d = plan[(i64)blockIdx.x * kWaveLanes + lane];
    const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
    if (nrows <= 0) return;  // padding tile (uniform over the workgroup)
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
            tile_pass<NW, (LV >= 4 ? 4 : 1), IP>(A, B, side, dst, d, p, K, g, n_in, wv, lane);
        } else if (LV >= 2 && left >= 2) {
            lv = 2;
            tile_pass<NW, (LV >= 2 ? 2 : 1), IP>(A, B, side, dst, d, p, K, g, n_in, wv, lane);
        } else {
            tile_pass<NW, 1, IP>(A, B, side, dst, d, p, K, g, n_in, wv, lane);
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
                                          int K, int g, int T, int wv, int lane) {
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
                             : reinterpret_cast<uint2*>(p.trash + ((i64)((blockIdx.x * NW + wv) & (kTrashWaves - 1)) * 64 + lane));
        BandSink<true> sk{nullptr, st, out_lane ? (half ? -p.pitch : p.pitch) : 0, 0, lane};
        stream(sk);
    }
}

template <int NW, bool WRAPY, int LV, bool IP>
__global__ __launch_bounds__(64 * NW) void step_tile_fold(const u64* __restrict__ src, u64* __restrict__ dst,
                                                          const LaneDesc* __restrict__ plan, StepParams p, int K) {
    extern __shared__ __attribute__((aligned(16))) u32 tile_lds[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaneDesc d = plan[(i64)blockIdx.x * kWaveLanes + lane];  // lanes 32-63 repeat lanes 0-31
    const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
    if (nrows <= 0) return;  // padding tile (uniform over the workgroup)
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
            fold_pass<NW, (LV >= 4 ? 4 : 1), IP>(A, B, side, dst, d, p, K, g, T, wv, lane);
        } else if (LV >= 2 && left >= 2) {
            lv = 2;
            fold_pass<NW, (LV >= 2 ? 2 : 1), IP>(A, B, side, dst, d, p, K, g, T, wv, lane);
        } else {
            fold_pass<NW, 1, IP>(A, B, side, dst, d, p, K, g, T, wv, lane);
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

int tile_levels(u32 flags) { return (flags & STEP_TILE_L4) ? 4 : ((flags & STEP_TILE_L2) ? 2 : 1); }

// LDS rows of a tile with `rows` output rows at depth k: double-buffered, two copies of the tile
// (+4 rows of over-read slack); in place, one copy plus NW private side rows per wave.
i64 tile_lds_rows(i64 rows, int k, int nw, u32 flags) {
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

template <int NW, bool IP>
const void* tile_kernel_ip(u32 flags) {
    if (flags & STEP_TILE_L4)
        return (flags & STEP_WRAP_Y) ? (const void*)step_tile<NW, true, 4, IP> : (const void*)step_tile<NW, false, 4, IP>;
    if (flags & STEP_TILE_L2)
        return (flags & STEP_WRAP_Y) ? (const void*)step_tile<NW, true, 2, IP> : (const void*)step_tile<NW, false, 2, IP>;
    return (flags & STEP_WRAP_Y) ? (const void*)step_tile<NW, true, 1, IP> : (const void*)step_tile<NW, false, 1, IP>;
}
template <int NW, bool IP>
const void* tile_kernel_fold_ip(u32 flags) {
    if (flags & STEP_TILE_L4)
        return (flags & STEP_WRAP_Y) ? (const void*)step_tile_fold<NW, true, 4, IP> : (const void*)step_tile_fold<NW, false, 4, IP>;
    if (flags & STEP_TILE_L2)
        return (flags & STEP_WRAP_Y) ? (const void*)step_tile_fold<NW, true, 2, IP> : (const void*)step_tile_fold<NW, false, 2, IP>;
    return (flags & STEP_WRAP_Y) ? (const void*)step_tile_fold<NW, true, 1, IP> : (const void*)step_tile_fold<NW, false, 1, IP>;
}
template <int NW>
const void* tile_kernel_fold(u32 flags) {
    return (flags & STEP_TILE_INPLACE) ? tile_kernel_fold_ip<NW, true>(flags) : tile_kernel_fold_ip<NW, false>(flags);
}
template <int NW>
const void* tile_kernel(u32 flags) {
    if (flags & STEP_TILE_FOLD) return tile_kernel_fold<NW>(flags);
    return (flags & STEP_TILE_INPLACE) ? tile_kernel_ip<NW, true>(flags) : tile_kernel_ip<NW, false>(flags);
}

const void* tile_kernel_for(int nw_per_wg, u32 flags) {
    switch (nw_per_wg) {
        case 4:
            return tile_kernel<4>(flags);
        case 8:
            return tile_kernel<8>(flags);
        case 16:
            return tile_kernel<16>(flags);
        default:
            return nullptr;
    }
}

// ------------------------------------------------------------------------------------------
// LDS-tiled single-generation kernel.
// ------------------------------------------------------------------------------------------
constexpr int kLdsRows = 16, kLdsWords = 64;

__global__ __launch_bounds__(256) void step_lds(const u64* __restrict__ src, u64* __restrict__ dst, i64 pitch,
                                                int R, int h, int nw, int r0, int r1, u32 flags) {
    __shared__ u64 tile[kLdsRows + 2][kLdsWords + 3];  // +1 pad word per row against bank conflicts
    const int tr = r0 + blockIdx.y * kLdsRows;  // first output row of the tile
    const int tc = blockIdx.x * kLdsWords;      // first output word
    const bool wy = flags & STEP_WRAP_Y, wx = flags & STEP_WRAP_X;
    // stage (rows tr-1 .. tr+16) x (words tc-1 .. tc+64): 18 x 66 words
    for (int e = threadIdx.x; e < (kLdsRows + 2) * (kLdsWords + 2); e += 256) {
        const int rr = e / (kLdsWords + 2), cc = e % (kLdsWords + 2);
        int row = tr - 1 + rr, col = tc - 1 + cc;
        if (wy) row = row < 0 ? row + h : (row >= h ? row - h : row);
        if (wx) col = col < 0 ? nw - 1 : (col >= nw ? 0 : col);
        u64 v = 0;
        if (row <= h + R - 1 && col <= nw) v = src[(i64)(R + row) * pitch + (col + 1)];
        tile[rr][cc] = v;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kLdsRows * kLdsWords; e += 256) {
        const int rr = e / kLdsWords, cc = e % kLdsWords;
        const int row = tr + rr, col = tc + cc;
        if (row >= r1 || col >= nw) continue;
        u64 a0, a1, b0, b1, c0, c1;
        hsum64(tile[rr][cc], tile[rr][cc + 1], tile[rr][cc + 2], a0, a1);
        hsum64(tile[rr + 1][cc], tile[rr + 1][cc + 1], tile[rr + 1][cc + 2], b0, b1);
        hsum64(tile[rr + 2][cc], tile[rr + 2][cc + 1], tile[rr + 2][cc + 2], c0, c1);
        dst[(i64)(R + row) * pitch + (col + 1)] = rule64(a0, a1, b0, b1, c0, c1, tile[rr + 1][cc + 1]);
    }
}

}  // namespace

// Instantiated depths.  Larger K amortises HBM traffic over more generations at the cost of
// registers (10 VGPRs per level per lane) and 2K halo rows per segment.
#define FOR_EACH_STEP_DEPTH(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(12) X(16)

bool step_depth_supported(int k) {
    switch (k) {
#define DEPTH_CASE(K) \
    case K:         \
        return true;
        FOR_EACH_STEP_DEPTH(DEPTH_CASE)
#undef DEPTH_CASE
        default:
            return false;
    }
}

int max_step_depth() { return 16; }

static const void* kernel_of(int k, u32 flags) {
    switch (k) {
#define DEPTH_CASE(K) \
    case K:         \
        return kernel_for<K>(flags);
        FOR_EACH_STEP_DEPTH(DEPTH_CASE)
#undef DEPTH_CASE
        default:
            return nullptr;
    }
}

int step_blocks_per_cu(int k, u32 flags) {
    const void* f = kernel_of(k, flags);
    int nb = 0;
    if (!f || hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 64 * kWavesPerBlock, 0) != hipSuccess || nb < 1) return 1;
    return std::min(nb, 32 / kWavesPerBlock);
}

// Per-device trash buffers (StepParams::trash).
static std::mutex g_trash_mu;
static u64* g_trash[64] = {};
void ensure_trash() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) throw Error("ensure_trash: no current HIP device");
    std::lock_guard<std::mutex> lk(g_trash_mu);
    if (g_trash[dev]) return;
    void* t = nullptr;
    if (hipMalloc(&t, (size_t)kTrashWaves * 64 * sizeof(u64)) != hipSuccess) throw Error("ensure_trash: hipMalloc failed");
    g_trash[dev] = (u64*)t;
}
u64* trash_of_current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || !g_trash[dev])
        throw Error("step kernels: the device's trash buffer is not allocated (hipk::ensure_trash)");
    return g_trash[dev];
}

void launch_step(int k, const u64* src, u64* dst, const LaneDesc* plan, i64 n_waves, const StepParams& p,
                 hipStream_t s) {
    const void* f = kernel_of(k, p.flags);
    if (!f) throw Error(strprintf("no step kernel instantiated for depth %d", k));
    const dim3 grid((unsigned)(n_waves / kWavesPerBlock)), block(64 * kWavesPerBlock);
    StepParams pp = p;
    if (!pp.trash) pp.trash = trash_of_current_device();
    void* args[] = {(void*)&src, (void*)&dst, (void*)&plan, (void*)&pp};
    hipError_t e = hipLaunchKernel(f, grid, block, args, 0, s);
    if (e != hipSuccess) throw Error(strprintf("step kernel launch failed: %s", hipGetErrorString(e)));
}

i64 tile_max_rows(int k, int nw_per_wg, u32 flags) {
    const i64 lds_rows = kMaxLdsBytes / (kTileRowU32 * 4);  // 320 rows of 512 B
    if (flags & STEP_TILE_FOLD)  // rows + 2k = T with ceil(T/2) + 8 rows per buffer
        return (flags & STEP_TILE_INPLACE)
                   ? 2 * (lds_rows - (i64)nw_per_wg * tile_side_rows(tile_levels(flags)) - kFoldMirror - 4) - 1 - 2 * (i64)k
                   : 2 * (lds_rows / 2 - kFoldMirror - 4) - 1 - 2 * (i64)k;
    if (flags & STEP_TILE_INPLACE) return lds_rows - (i64)nw_per_wg * tile_side_rows(tile_levels(flags)) - 2 * (i64)k;
    return (lds_rows - 4) / 2 - 2 * (i64)k;
}

static const void* tile_kernel_checked(int nw_per_wg, u32 flags) {
    const void* f = tile_kernel_for(nw_per_wg, flags);
    if (!f) throw Error(strprintf("step_tile: unsupported waves per workgroup %d (4, 8 or 16)", nw_per_wg));
    // allow the full 160 KiB of dynamic LDS, once per (device, kernel variant): thread-mode ranks on
    // different GPUs launch concurrently, and the attribute is per device
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> attr_set;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) throw Error("step_tile: no current HIP device");
    std::lock_guard<std::mutex> lk(mu);
    if (attr_set.insert({dev, f}).second) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsBytes);
        if (e != hipSuccess) {
            attr_set.erase({dev, f});
            throw Error(strprintf("step_tile: hipFuncSetAttribute: %s", hipGetErrorString(e)));
        }
    }
    return f;
}

int tile_blocks_per_cu(int nw_per_wg, i64 rows, int k, u32 flags) {
    const void* f = tile_kernel_checked(nw_per_wg, flags);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 64 * nw_per_wg, tile_lds_bytes(rows, k, nw_per_wg, flags)) !=
            hipSuccess ||
        nb < 1)
        return 1;
    return std::min(nb, 8);
}

void launch_step_tile(int nw_per_wg, int k, const u64* src, u64* dst, const LaneDesc* plan, i64 n_tiles, i64 rows,
                      const StepParams& p, hipStream_t s) {
    if (k < 1 || k > 64) throw Error(strprintf("step_tile: depth %d outside 1..64", k));
    const i64 rmax = tile_max_rows(k, nw_per_wg, p.flags);
    if (rows < 1 || rows > rmax)
        throw Error(strprintf("step_tile: %lld rows per tile exceed the LDS capacity (max %lld at depth %d)",
                              (long long)rows, (long long)rmax, k));
    // folded tiles: the staged mirror and over-read rows past the middle are tile rows < T
    // (K + nrows/2 >= 8) and every pass but the last recomputes the mirrored rows (nrows >= 6): the
    // plan's segments are >= rows/2 >= 14 rows (engine and kbench: regions of >= kFoldMinRows/2 rows)
    if ((p.flags & STEP_TILE_FOLD) && rows < kFoldMinRows)
        throw Error(strprintf("step_tile: a folded tile plan needs at least %d rows (got %lld)", kFoldMinRows,
                              (long long)rows));
    const void* f = tile_kernel_checked(nw_per_wg, p.flags);
    StepParams pp = p;
    if (!pp.trash) pp.trash = trash_of_current_device();
    int kk = k;
    void* args[] = {(void*)&src, (void*)&dst, (void*)&plan, (void*)&pp, (void*)&kk};
    hipError_t e = hipLaunchKernel(f, dim3((unsigned)n_tiles), dim3(64 * nw_per_wg), args,
                                   tile_lds_bytes(rows, k, nw_per_wg, p.flags), s);
    if (e != hipSuccess) throw Error(strprintf("step_tile launch failed: %s", hipGetErrorString(e)));
}


void launch_step_lds(const u64* src, u64* dst, const Layout& L, i64 r0, i64 r1, u32 flags, hipStream_t s) {
    if (r1 <= r0) return;
    const dim3 grid((unsigned)ceil_div(L.nw, kLdsWords), (unsigned)ceil_div(r1 - r0, kLdsRows)), block(256);
    hipLaunchKernelGGL(step_lds, grid, block, 0, s, src, dst, L.pitch, L.R, (int)L.h, (int)L.nw, (int)r0, (int)r1,
                       flags);
}

}  // namespace hipk
}  // namespace gol
