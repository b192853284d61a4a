// gol-mi355x: the streaming wave of the register-pipeline kernel (step_temporal in step_kernels.hip): one
// wave streams one plan segment (64 word columns, nrows + 2K input rows) through the K-level register
// pipeline of stencil_device.hpp and stores its output rows.  Kernel boundaries order the passes.
#pragma once

#include "gol/bits.hpp"
#include "gol/hip_kernels.hpp"
#include "stencil_device.hpp"

namespace gol {
namespace hipk {
namespace {

// A row load of the wave runner: a plain dereference, written in place.  (Routing the loads through
// an inline helper once changed the K = 12 kernel's schedule -- 256 VGPRs with AGPR spills and a
// vmcnt(0) before the stores in the row loop, the pass 119 -> 163 us at 32768^2 -- although the helper
// inlines to the same load.)
#define ROW_LOAD_INTO(dst) ((dst) = *ld)

// Row prefetch: a register triple loaded one row-triple ahead, pinned above the compute with a
// sched_barrier (otherwise the scheduler sinks the loads to the end of the loop body).  (An LDS
// DMA ring and a skewed level pipeline were built and measured slower; docs/PERFORMANCE.md §2.)
// Row sources of the load stream (kernel template ROWS):
//   ROWS_GHOST  rows -R .. h+R-1 of the source buffer (ghost rows filled by exchanges / earlier passes)
//   ROWS_WRAP   rows are periodic (the tile is its own N/S neighbour): row h is row 0
//   ROWS_SEAM   rows < 0 come from p.above, rows >= h from p.below, rows 0..h-1 from the source
//               buffer: the first pass of a sub-tile superstep reads the neighbouring half's edge rows
//               in place (and the torus wrap), so no seam copy precedes it
enum { ROWS_GHOST = 0, ROWS_WRAP = 1, ROWS_SEAM = 2 };

// Prefetch depth in rows.  Deep passes (K >= 5) are VALU bound and keep one row-triple in flight
// (registers are what limits their occupancy).  Shallow passes are memory bound: a whole-board pass
// at K <= 4 costs ~70 us at 32768^2 whatever K is, i.e. ~3.8 TB/s, limited by the bytes each wave
// keeps in flight, so they prefetch two row-triples ahead.
template <int K>
constexpr int prefetch_rows() {
    return K <= 4 ? 6 : 3;
}
// Deep passes whose one-triple steady loop the compiler schedules with a wait on the fresh prefetch
// (see WaveRunner::run) use the two-triple loop: K = 6, 7 and 12.  Measured at 32768^2, two halves
// (profiles/pingpong_loop_ab.txt): K=7 12.2 -> 10.9 us/gen, K=12 12.8 -> 10.6, K=6 12.0 -> 11.8;
// K=5 and 8 do not gain.
// step_temporal's rule: rule32, or (GOL_TEMPORAL_PAIR=1, experiment) the pair-shared rule of stencil_device.hpp
// with the two-triple loop at K = 8 as well: in the one-triple loop the compiler waits for the fresh prefetch
// (s_waitcnt vmcnt(0) 60 instructions after the loads, 24% slower: profiles/pair_rule_round6.txt).  With the
// prefetch kept and 9% fewer instructions per row it still only ties at K = 8 and loses 2-4% at K = 5, 6, 12
// (profiles/temporal_pair_round6.txt): this streaming kernel is not bound by its gate count.
#ifndef GOL_TEMPORAL_PAIR
#define GOL_TEMPORAL_PAIR 0
#endif
constexpr bool kTemporalPair = GOL_TEMPORAL_PAIR != 0 && kRulePair;
constexpr unsigned kPingpongMask = (1u << 6) | (1u << 7) | (1u << 12) | (kTemporalPair ? (1u << 8) : 0u);
// ... and, for the ghost-row variant only (the sub-tile passes after the first), K = 5
constexpr unsigned kPingpongGhostMask = 1u << 5;
template <int K, int ROWS>
constexpr bool pingpong_loop() {
    return K < 32 && (((kPingpongMask >> K) & 1) != 0 || (ROWS == 0 && ((kPingpongGhostMask >> K) & 1) != 0));
}

template <int K, int ROWS>
struct WaveRunner {
    static constexpr int D = prefetch_rows<K>();
    const StepParams& p;
    const LaneDesc& d;
    const int n;   // row iterations: nrows + 2K
    const i64 hp;  // h * pitch
    const uint2* ld;
    const u64* own0;  // ROWS_SEAM: row 0 of the source buffer
    uint2* st;
    i64 st_stride;  // pitch for output lanes, 0 for halo/idle lanes (they write a trash slot)
    int lrow;       // tile row of the next load (ROWS_WRAP, ROWS_SEAM; wave-uniform)
    uint2 pf[D];
    Pipe<K> P;

    __device__ __forceinline__ void next_row() {
        ld += p.pitch;
        if (ROWS == ROWS_WRAP) {  // rows are periodic: row h is row 0 (branch-free select)
            ++lrow;
            const bool w = lrow == p.h;
            lrow = w ? 0 : lrow;
            ld = w ? ld - hp : ld;
        } else if (ROWS == ROWS_SEAM) {  // switch sources at rows 0 and h
            ++lrow;
            ld = lrow == 0 ? reinterpret_cast<const uint2*>(own0 + (d.col + 1)) : ld;
            ld = lrow == p.h ? reinterpret_cast<const uint2*>(p.below + (d.col + 1)) : ld;
        }
    }

    __device__ __forceinline__ WaveRunner(const u64* src, u64* dst, const LaneDesc& d_, int nrows, const StepParams& p_,
                                          i64 wave_id)
        : p(p_), d(d_), n(nrows + 2 * K), hp((i64)p_.h * p_.pitch) {
        lrow = d.row0 - K;
        if (ROWS == ROWS_WRAP && lrow < 0) lrow += p.h;
        if (ROWS == ROWS_SEAM) {
            own0 = src + (i64)p.R * p.pitch;
            const u64* b = lrow < 0 ? p.above + (i64)lrow * p.pitch
                                    : (lrow >= p.h ? p.below + (i64)(lrow - p.h) * p.pitch : own0 + (i64)lrow * p.pitch);
            ld = reinterpret_cast<const uint2*>(b + (d.col + 1));
        } else {
            ld = reinterpret_cast<const uint2*>(src + (i64)(lrow + p.R) * p.pitch + (d.col + 1));
        }
        // Every lane stores every row (no branch: the row loop stays one basic block, so the
        // scheduler can interleave consecutive rows).  Halo/idle lanes write a trash word of their
        // own (wave mod kTrashWaves, lane), which nothing reads.  (They used to share one trash row
        // per plan column: thousands of waves storing to the same few words every row, a hot spot
        // that held shallow memory-bound passes at ~55% of the HBM streaming rate.)
        const bool out = d.flags & LANE_STORE;
        st = out ? reinterpret_cast<uint2*>(dst + (i64)(d.row0 + p.R) * p.pitch + (d.col + 1))
                 : reinterpret_cast<uint2*>(p.trash + ((i64)(wave_id & (kTrashWaves - 1)) * 64 + (threadIdx.x & 63)));
        st_stride = out ? p.pitch : 0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            ROW_LOAD_INTO(pf[j]);
            next_row();
        }
    }

    // Next input row (lo, hi) in order.
    template <int PH>
    __device__ __forceinline__ void fetch(u32& lo, u32& hi) {
        uint2 x;
        if constexpr (D == 3) {
            x = pf[PH];
            ROW_LOAD_INTO(pf[PH]);  // prefetch 3 rows ahead (the allocation has slack rows past the halo)
        } else {
            x = pf[0];  // a queue of D rows (the shift is register renaming in the unrolled code)
#pragma unroll
            for (int j = 0; j + 1 < D; ++j) pf[j] = pf[j + 1];
            ROW_LOAD_INTO(pf[D - 1]);
        }
        next_row();
        lo = x.x;
        hi = x.y;
    }

    template <int PH, bool GUARD>
    __device__ __forceinline__ void compute_store(u32 lo, u32 hi, int i) {
        if (!advance<K, PH, GUARD, kTemporalPair>(P, lo, hi, i)) return;  // (stencil_device.hpp, PAIR)
        *st = make_uint2(lo, hi);
        st += st_stride;
    }

    template <int PH, bool GUARD>
    __device__ __forceinline__ void body(int i) {
        if (GUARD && i >= n) return;
        u32 lo, hi;
        fetch<PH>(lo, hi);
        compute_store<PH, GUARD>(lo, hi, i);
    }

    __device__ __forceinline__ void run() {
        constexpr int i0 = ((2 * K + 2) / 3) * 3;  // first multiple of 3 at which the pipeline is full
        int i = 0;
        for (; i < i0; i += 3) {
            body<0, true>(i);
            body<1, true>(i + 1);
            body<2, true>(i + 2);
        }
        if constexpr (D == 6) {
            // Shallow (memory-bound) passes: each row's registers are consumed and then refilled with
            // the row six ahead, so six loads stay in flight per wave and no register copy has to
            // wait for an outstanding load (copying a prefetched register forces the wait: the
            // queue shift of the fill phase collapses the prefetch distance to one triple).
#define ROW6_STEP(J)                                          \
    compute_store<(J) % 3, false>(pf[J].x, pf[J].y, i + (J)); \
    ROW_LOAD_INTO(pf[J]);                                             \
    next_row();                                              \
    __builtin_amdgcn_sched_barrier(0);
            for (; i + 6 <= n; i += 6) {
                ROW6_STEP(0) ROW6_STEP(1) ROW6_STEP(2) ROW6_STEP(3) ROW6_STEP(4) ROW6_STEP(5)
            }
#undef ROW6_STEP
            // fewer than six rows left, in pf[0..] in order
            if (i < n) compute_store<0, false>(pf[0].x, pf[0].y, i);
            if (i + 1 < n) compute_store<1, false>(pf[1].x, pf[1].y, i + 1);
            if (i + 2 < n) compute_store<2, false>(pf[2].x, pf[2].y, i + 2);
            if (i + 3 < n) compute_store<0, false>(pf[3].x, pf[3].y, i + 3);
            if (i + 4 < n) compute_store<1, false>(pf[4].x, pf[4].y, i + 4);
        } else {
            if constexpr (pingpong_loop<K, ROWS>()) {
                // Two register triples in turn (rows i..i+2 in pf, i+3..i+5 in q): each is refilled
                // right after its rows were computed, so no prefetched register is ever copied.  (With
                // the one-triple loop below the compiler copies the new pf[2] into the register of the
                // old one at some depths, right after its last use: that copy waits for the load just
                // issued, s_waitcnt vmcnt(0), and the prefetch is lost.)
                uint2 q[3];
                for (; i + 6 <= n; i += 6) {
                    ROW_LOAD_INTO(q[0]);
                    next_row();
                    ROW_LOAD_INTO(q[1]);
                    next_row();
                    ROW_LOAD_INTO(q[2]);
                    next_row();
                    __builtin_amdgcn_sched_barrier(0);
                    compute_store<0, false>(pf[0].x, pf[0].y, i);
                    compute_store<1, false>(pf[1].x, pf[1].y, i + 1);
                    compute_store<2, false>(pf[2].x, pf[2].y, i + 2);
                    ROW_LOAD_INTO(pf[0]);
                    next_row();
                    ROW_LOAD_INTO(pf[1]);
                    next_row();
                    ROW_LOAD_INTO(pf[2]);
                    next_row();
                    __builtin_amdgcn_sched_barrier(0);
                    compute_store<0, false>(q[0].x, q[0].y, i + 3);
                    compute_store<1, false>(q[1].x, q[1].y, i + 4);
                    compute_store<2, false>(q[2].x, q[2].y, i + 5);
                }
            }
            for (; i + 3 <= n; i += 3) {
                // hoist the whole next triple's loads above this triple's compute
                const uint2 x0 = pf[0], x1 = pf[1], x2 = pf[2];
                ROW_LOAD_INTO(pf[0]);
                next_row();
                ROW_LOAD_INTO(pf[1]);
                next_row();
                ROW_LOAD_INTO(pf[2]);
                next_row();
                __builtin_amdgcn_sched_barrier(0);
                compute_store<0, false>(x0.x, x0.y, i);
                compute_store<1, false>(x1.x, x1.y, i + 1);
                compute_store<2, false>(x2.x, x2.y, i + 2);
            }
            if (i < n) body<0, false>(i);
            if (i + 1 < n) body<1, false>(i + 1);
        }
    }
};

}  // namespace
}  // namespace hipk
}  // namespace gol
