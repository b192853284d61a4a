// gol-mi355x: step_resident — a whole run of generations in ONE launch, the board resident in VGPRs.
//
// Small boards (8192^2 = BASELINE config 2) cannot fill 256 CUs with streaming segments tall enough to
// amortise a K-deep halo, and the LDS tile kernel pays a band warm-up per LDS pass and a re-staging per
// kernel pass (docs/PERFORMANCE.md §8).  Here one workgroup per CU owns a tile of the plan (64 lanes,
// one word column each, plan.hpp) for the whole launch; its NW waves each keep a band of B rows of the
// tile in registers (lo/hi split words, bits.hpp) and advance it one generation at a time:
//
//   * per generation: each band computes the horizontal 3-sums of its first and last rows, publishes
//     them in LDS (double-buffered by generation parity), one workgroup barrier, reads the
//     neighbouring bands' edge sums, and applies B3/S23 to its B rows (11 VALU ops per 32 cells, the
//     same circuit as step_temporal, stencil_device.hpp) — no band overlap, no recomputed halo rows
//     inside the tile;
//   * the tile carries a K-row halo above and below (the trapezoid: generation g of a superstep
//     computes extended rows [g, T-g), whole bands outside are skipped).  Every K generations
//     (a superstep) the tile publishes its output rows to HBM, signals a per-tile counter, waits only
//     for the tiles that own words of its halo (host-built neighbour lists), and reloads its halo:
//     no kernel boundary, no grid barrier, no re-staging of its own rows;
//   * hand-offs follow the inter-workgroup visibility rules of MI355X_MICROARCH.md: write-through
//     (sc1) stores of the published rows, s_waitcnt vmcnt(0) in every wave, a workgroup barrier, one
//     lane's agent-scope release and relaxed counter store; the consumer polls relaxed agent loads, one
//     agent-scope acquire, a barrier, then sc1 loads;
//   * every wait is bounded (s_memrealtime, rp.timeout_ticks): a tile that is not co-resident (the host
//     checks occupancy x CUs >= tiles before launching) or a stuck neighbour makes the waiting tiles
//     record an error in `status` and exit, so the grid always drains;
//   * the launch's supersteps alternate between the two board buffers and their count is odd, so the
//     result is in `dst` (the first superstep never writes `src`, which slower tiles may still be
//     loading); the counters are per tile and count supersteps over all launches, so a captured graph
//     replays correctly (no per-launch epoch argument).
// Reference: gol-with-cuda.cu:189-262 (one thread per byte cell, one launch and a device sync per
// generation, gol-with-cuda.cu:264-284).
#include <mutex>
#include <set>
#include <utility>

#include "gol/hip_kernels.hpp"
#include "stencil_device.hpp"

namespace gol {
namespace hipk {

namespace {

struct Hs {  // horizontal 3-sum planes of one row (bit 0 / bit 1, even / odd columns)
    u32 s0l, s1l, s0h, s1h;
};

__device__ __forceinline__ Hs hs_of(u32 lo, u32 hi) {
    Hs r;
    hsum_split(lo, hi, r.s0l, r.s1l, r.s0h, r.s1h);
    return r;
}

__device__ __forceinline__ void rule_row(const Hs& a, const Hs& b, const Hs& c, u32& lo, u32& hi) {
    const u32 nl = rule32(a.s0l, a.s1l, b.s0l, b.s1l, c.s0l, c.s1l, lo);
    const u32 nh = rule32(a.s0h, a.s1h, b.s0h, b.s1h, c.s0h, c.s1h, hi);
    lo = nl;
    hi = nh;
}

__device__ __forceinline__ u64 load_sc1(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_sc1(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NW, int B, bool WRAPY>
__global__ __launch_bounds__(64 * NW) void step_resident(u64* __restrict__ src, u64* __restrict__ dst,
                                                         const LaneDesc* __restrict__ plan,
                                                         const u32* __restrict__ nbr_off,
                                                         const u32* __restrict__ nbr, u32* __restrict__ counters,
                                                         u32* __restrict__ status, ResidentParams rp) {
    // [generation parity][band][first / last row][lane] edge sums (64 KiB at 16 waves), then a flag
    extern __shared__ uint4 resident_lds[];
    auto edge = reinterpret_cast<uint4(*)[NW][2][64]>(resident_lds);
    int& abort_all = *reinterpret_cast<int*>(resident_lds + 2 * NW * 2 * 64);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaneDesc d = plan[(i64)blockIdx.x * kWaveLanes + lane];
    const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
    if (nrows <= 0) return;  // padding tile (uniform over the workgroup)
    const int K = rp.kmax;  // halo rows above / below = the deepest superstep of the launch
    const int T = nrows + 2 * K;
    const int b0 = wv * B;
    const bool out_lane = (d.flags & LANE_STORE) != 0;
    if (threadIdx.x == 0) abort_all = 0;  // (LDS starts undefined; the first generation's barrier orders it)
    // word of extended row e (tile row d.row0 - K + e) of this lane's column in `buf`.  The row index
    // passes through an opaque scalar move, so the compiler recomputes each address where it is used
    // (once per superstep) instead of keeping 2 x B 64-bit addresses per buffer live across the
    // generation loop.
    auto at = [&](u64* buf, int e0) -> u64* {
        int e;
        asm volatile("s_mov_b32 %0, %1" : "=s"(e) : "s"(e0));
        int r = d.row0 - K + e;
        if (WRAPY) r = r < 0 ? r + rp.h : (r >= rp.h ? r - rp.h : r);
        return buf + (i64)(r + rp.R) * rp.pitch + (d.col + 1);
    };
    u32 lo[B], hi[B];
#pragma unroll
    for (int i = 0; i < B; ++i) {
        lo[i] = hi[i] = 0;
        if (b0 + i < T) {  // wave-uniform
            const u64 v = *at(src, b0 + i);
            lo[i] = (u32)v;
            hi[i] = (u32)(v >> 32);
        }
    }
    // supersteps every tile has completed in earlier launches (equal on all tiles between launches)
    const u32 base = __hip_atomic_load(&counters[blockIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int s = 1; s <= rp.S; ++s) {
        const int ks = rp.G / rp.S + (s <= rp.G % rp.S ? 1 : 0);
        for (int g = 1; g <= ks; ++g) {
            const int par = g & 1;
            // bands holding input rows [g-1, T-g+1) of this generation publish their edge sums and
            // compute; the others (outside the trapezoid) only keep the barrier
            const bool active = b0 + B > g - 1 && b0 < T - g + 1;
            if (!active) {  // (a path that leaves the band's registers alone: no merge copies)
                __syncthreads();
                continue;
            }
            const Hs first = hs_of(lo[0], hi[0]);
            const Hs last = B > 1 ? hs_of(lo[B - 1], hi[B - 1]) : first;
            edge[par][wv][0][lane] = make_uint4(first.s0l, first.s1l, first.s0h, first.s1h);
            edge[par][wv][1][lane] = make_uint4(last.s0l, last.s1l, last.s0h, last.s1h);
            __syncthreads();
            uint4 ua = make_uint4(0, 0, 0, 0), ub = make_uint4(0, 0, 0, 0);
            if (wv > 0) ua = edge[par][wv - 1][1][lane];
            if (wv < NW - 1) ub = edge[par][wv + 1][0][lane];
            const Hs above{ua.x, ua.y, ua.z, ua.w}, below{ub.x, ub.y, ub.z, ub.w};
            if constexpr (B == 1) {
                rule_row(above, first, below, lo[0], hi[0]);
            } else {
                // interior rows 1 .. B-2 first (the neighbours' edge sums arrive meanwhile); every
                // row's sums are taken from its old value before that row is overwritten
                const Hs h1 = B > 2 ? hs_of(lo[1], hi[1]) : last;  // sums of row 1
                Hs prev = first, cur = h1;
#pragma unroll
                for (int i = 1; i + 1 < B; ++i) {
                    const Hs nx = i + 2 < B ? hs_of(lo[i + 1], hi[i + 1]) : last;
                    rule_row(prev, cur, nx, lo[i], hi[i]);
                    prev = cur;
                    cur = nx;
                    // one row at a time: hoisting every row's sums above the rules would hold 4 x B
                    // more VGPRs
                    __builtin_amdgcn_sched_barrier(0);
                }
                const Hs hb2 = B > 2 ? prev : first;  // sums of row B-2
                rule_row(above, first, h1, lo[0], hi[0]);
                rule_row(hb2, last, below, lo[B - 1], hi[B - 1]);
            }
        }
        // ---- superstep end: publish the output rows (extended rows K .. K+nrows-1) ----
        // (rp.S is odd: supersteps S, S-2, ... write dst, the others src; the first writes dst)
        u64* X = ((rp.S - s) & 1) ? src : dst;
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const int r = b0 + i - K;
            if (r >= 0 && r < nrows && out_lane) store_sc1(at(X, b0 + i), (u64)lo[i] | ((u64)hi[i] << 32));
        }
        if (s == rp.S) break;  // the kernel boundary publishes the last one
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const u32 want = base + (u32)s;
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&counters[blockIdx.x], want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // ---- wait for the tiles that own words of this tile's halo (bounded) ----
        if (wv == 0) {
            const u32 n0 = nbr_off[blockIdx.x], n1 = nbr_off[blockIdx.x + 1];
            const u64 t0 = __builtin_amdgcn_s_memrealtime();
            bool timed_out = false;
            for (;;) {
                bool mine = true;
                for (u32 j = n0 + (u32)lane; j < n1; j += 64)
                    mine = mine && __hip_atomic_load(&counters[nbr[j]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
                if (__all(mine)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > rp.timeout_ticks) {
                    timed_out = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (timed_out && lane == 0) {
                abort_all = 1;
                atomicOr(status, 1u);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (abort_all) return;  // (uniform: read after the barrier)
        // ---- reload the halo: every row this lane does not own (halo rows, halo-lane columns) ----
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const int e = b0 + i, r = e - K;
            if (e < T && !(out_lane && r >= 0 && r < nrows)) {
                const u64 v = load_sc1(at(X, e));
                lo[i] = (u32)v;
                hi[i] = (u32)(v >> 32);
            }
        }
    }
}

template <int NW, int B>
const void* resident_kernel_wrap(bool wrapy) {
    return wrapy ? (const void*)step_resident<NW, B, true> : (const void*)step_resident<NW, B, false>;
}

template <int NW>
const void* resident_kernel_nw(int B, bool wrapy) {
    switch (B) {
        case 2: return resident_kernel_wrap<NW, 2>(wrapy);
        case 3: return resident_kernel_wrap<NW, 3>(wrapy);
        case 4: return resident_kernel_wrap<NW, 4>(wrapy);
        case 5: return resident_kernel_wrap<NW, 5>(wrapy);
        case 6: return resident_kernel_wrap<NW, 6>(wrapy);
        case 8: return resident_kernel_wrap<NW, 8>(wrapy);
        case 10: return resident_kernel_wrap<NW, 10>(wrapy);
        case 12: return resident_kernel_wrap<NW, 12>(wrapy);
        case 16: return resident_kernel_wrap<NW, 16>(wrapy);
        default: return nullptr;
    }
}

const void* resident_kernel(int nw, int B, bool wrapy) {
    switch (nw) {
        case 8: return resident_kernel_nw<8>(B, wrapy);
        case 16: return resident_kernel_nw<16>(B, wrapy);
        default: return nullptr;
    }
}

size_t resident_lds_bytes(int nw) { return (size_t)(2 * nw * 2 * 64 + 1) * sizeof(uint4); }

// the kernel's dynamic LDS exceeds the 64 KiB default at 16 waves: raise the limit once per
// (device, kernel variant)
const void* resident_kernel_checked(int nw, int B, bool wrapy) {
    const void* f = resident_kernel(nw, B, wrapy);
    if (!f) throw Error(strprintf("step_resident: no kernel for %d waves x %d band rows", nw, B));
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) throw Error("step_resident: no current HIP device");
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert({dev, f}).second) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)resident_lds_bytes(nw));
        if (e != hipSuccess) {
            done.erase({dev, f});
            throw Error(strprintf("step_resident: hipFuncSetAttribute: %s", hipGetErrorString(e)));
        }
    }
    return f;
}

}  // namespace

int resident_band_rows(int rows_needed) {
    for (int b : {2, 3, 4, 5, 6, 8, 10, 12, 16})
        if (b >= rows_needed) return b;
    return 0;
}

int resident_blocks_per_cu(int nw, int B, bool wrapy) {
    const void* f = resident_kernel_checked(nw, B, wrapy);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 64 * nw, resident_lds_bytes(nw)) != hipSuccess) return 0;
    return nb;
}

void launch_step_resident(int nw, int B, bool wrapy, u64* src, u64* dst, const LaneDesc* plan, i64 n_tiles,
                          const u32* nbr_off, const u32* nbr, u32* counters, u32* status, const ResidentParams& rp,
                          hipStream_t s) {
    const void* f = resident_kernel_checked(nw, B, wrapy);
    if (rp.S < 1 || (rp.S & 1) == 0 || rp.G < rp.S || rp.kmax < (rp.G + rp.S - 1) / rp.S)
        throw Error(strprintf("step_resident: bad superstep cut (G %d, S %d, kmax %d)", rp.G, rp.S, rp.kmax));
    ResidentParams p = rp;
    void* args[] = {(void*)&src, (void*)&dst,     (void*)&plan,   (void*)&nbr_off,
                    (void*)&nbr, (void*)&counters, (void*)&status, (void*)&p};
    const hipError_t e =
        hipLaunchKernel(f, dim3((unsigned)n_tiles), dim3(64 * nw), args, resident_lds_bytes(nw), s);
    if (e != hipSuccess) throw Error(strprintf("step_resident launch failed: %s", hipGetErrorString(e)));
}

}  // namespace hipk
}  // namespace gol
