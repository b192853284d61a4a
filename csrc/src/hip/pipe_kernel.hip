// gol-mi355x: step_pipe — a level-pipelined workgroup: K = NW x L generations per pass, the waves of
// one workgroup chained through LDS rings.
//
// The streaming kernel (step_temporal) gets its K levels from one wave, so a small board (8192^2 =
// BASELINE config 2, or a strong-scaled 4096-row strip) cannot be cut into segments tall enough to
// amortise the 2K-row halo over the ~3000 waves the chip needs; the LDS tile kernel (step_tile) shares
// the halo between the waves of a workgroup but splits each generation into row bands, which pays a
// band warm-up of ~2 LV rows per band and LDS pass, a workgroup barrier per LDS pass and the tile's
// staging (docs/PERFORMANCE.md §8).  Here the waves of a workgroup split the LEVELS instead of the
// rows: wave w owns generations w L + 1 .. (w + 1) L of the whole segment and streams it top to bottom
// with the step_temporal register pipeline (stencil_device.hpp Pipe / advance, 11 VALU ops per 32
// cells per generation); the rows it emits at level (w + 1) L go into an LDS ring that wave w + 1
// reads as its input stream.  So:
//   * the segment's vertical halo (2K rows) is paid once per workgroup, like the tile kernel, and the
//     trapezoid is the same (stage w streams nrows + 2K - 2 w L rows);
//   * no band overlap and no workgroup barrier at all: a wave waits only for its own producer (ring
//     rows published) and its own consumer (ring slots freed), through two LDS counters per ring,
//     checked once per row triple and cached in SGPRs, so the pipeline runs at the pace of the
//     aggregate VALU issue of its NW waves;
//   * wave 0 streams the segment from HBM with a 6-row register prefetch (the rows reach it one
//     level group ahead of everyone else, so its loads need the deeper queue), the last wave stores the
//     output rows to HBM; nothing is staged.
// Visibility inside the workgroup: LDS operations of one wave are performed in order, so a ring row
// written before the producer's counter store is visible to a consumer that observed the counter (the
// counter accesses are workgroup-scope release/acquire atomics, which also keep the compiler from
// moving ring accesses across them).  No wait is unbounded in a bad way: every producer/consumer pair
// is a chain (wave w depends on w - 1 and w + 1 only), all NW waves of a workgroup are co-resident,
// and every stage streams exactly the rows its consumer expects, so the chain always drains.
// Reference: gol-with-cuda.cu:189-262 (one thread per byte cell, one launch and a device sync per
// generation, gol-with-cuda.cu:264-284).
#include <mutex>
#include <set>
#include <type_traits>
#include <utility>
#include <vector>

#include "gol/hip_kernels.hpp"
#include "stencil_device.hpp"

namespace gol {
namespace hipk {

namespace {

// Ring geometry (measured, docs/PERFORMANCE.md §13: a 3-row register queue with 18-row rings ran
// 10.55 us/gen at 32768^2 where a 6-row queue or per-row counters were slower)
constexpr int kPipeSync = 3;       // rows between counter updates
constexpr int kPipeU = 3;          // rows of every stage's register queue (its prefetch distance)
constexpr int kPipeRing = 18;      // rows per LDS ring between compute stages (>= kPipeU + 3, multiple of 6)
constexpr int kPipeLoadAhead = 12; // rows the loader keeps in flight (2 DMAs per row, <= 31)
constexpr int kPipeRing0 = 18;     // rows of the loader's ring (>= kPipeLoadAhead + kPipeU + 3)
constexpr int kRowU32 = 128;    // one ring row: 64 lo words, then 64 hi words (LDS DMA writes planes)

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// Ring counters.  Relaxed LDS atomics plus compiler barriers, no hardware waits: the LDS performs a
// wave's DS operations in order, so ring rows written before a counter store are in LDS before the
// store is, and a consumer's ring reads, issued after it saw the counter, come after it.  (Release /
// acquire atomics would add s_waitcnt lgkmcnt(0) and, in the loader, vmcnt(0) — a wait for every DMA
// in flight.)
// In the loader the counter accesses are inline asm: the compiler treats any LDS access after an LDS
// DMA as possibly aliasing it and would wait for every DMA in flight (vmcnt(0)) before each of them.
__device__ __forceinline__ u32 lds_addr(const void* p) {
    return (u32)(size_t)(const __attribute__((address_space(3))) void*)p;
}
template <bool ASM = false>
__device__ __forceinline__ u32 ctr_load(const u32* c) {
    u32 v;
    if constexpr (ASM) {
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(c)) : "memory");
    } else {
        v = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return __builtin_amdgcn_readfirstlane(v);
}
template <bool ASM = false>
__device__ __forceinline__ void ctr_store(u32* c, u32 v) {
    asm volatile("" ::: "memory");
    if constexpr (ASM) {
        asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(c)), "v"(v) : "memory");
    } else {
        __hip_atomic_store(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// Set when a wait gave up (pipe_fault()): the board is invalid then, but every wave still drains.
__device__ u32 g_pipe_fault;

#ifdef GOL_PIPE_STAMPS
// Diagnostic build (tools/kbench.cpp KB_PIPE_STAMPS=1, build flag -DGOL_PIPE_STAMPS): per wave, s_memtime
// cycles of its role [0], spent in its input waits [1] (compute stages: the producer's counter; the loader:
// s_waitcnt vmcnt for its DMAs), in its output waits [2] (the consumer's counter; the loader: a free ring
// slot), and the number of waits that found the counter short [3].
constexpr int kPipeStampWaves = 1 << 16;
__device__ u64 g_pipe_stamps[kPipeStampWaves * 4];
#define PIPE_STAMPS 1
#else
#define PIPE_STAMPS 0
#endif
struct WaitAcc {  // (PIPE_STAMPS only: cycles waited, waits entered)
    u64 cy = 0, n = 0;
};
constexpr u64 kPipeWaitTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz): no real wait is that long

// wait until *c >= need (the cached value first: counters only grow).  Bounded: after 2 s (or once
// any wave of the device has given up) the wait returns as if satisfied and records the fault, so a
// broken pipeline cannot hang the GPU.
template <bool ASM = false>
__device__ __forceinline__ void ctr_wait(const u32* c, u32& cached, u32 need, WaitAcc* acc = nullptr) {
    if (cached < need) {
        const u64 s0 = PIPE_STAMPS && acc ? __builtin_amdgcn_s_memtime() : 0;
        cached = ctr_load<ASM>(c);
        if (PIPE_STAMPS && acc && cached < need) acc->n += 1;
        if (cached < need) {
            const u64 t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                __builtin_amdgcn_s_sleep(1);
                cached = ctr_load<ASM>(c);
                if (cached >= need) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > kPipeWaitTicks ||
                    __hip_atomic_load(&g_pipe_fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                    if ((threadIdx.x & 63) == 0) atomicOr(&g_pipe_fault, 1u);
                    cached = need;
                    break;
                }
            }
        }
        if (PIPE_STAMPS && acc) acc->cy += __builtin_amdgcn_s_memtime() - s0;
    }
    asm volatile("" ::: "memory");  // ring accesses stay after the wait
}

// Wave 0: streams the segment's n rows (row0 - K .. row0 + nrows + K - 1 of the source buffer, rows
// modulo h with WRAPY, else its ghost rows) into ring 0 with LDS DMA (global_load_lds, one 4-byte
// DMA per plane), kPipeLoadAhead rows in flight.  DMAs complete in order, so "row i has landed" is
// s_waitcnt vmcnt(2 (rows issued after it)).  Rows past the stream may be fetched (the allocation's
// slack rows or the wrap keep them in bounds) and are never published.
template <bool WRAPY>
__device__ __forceinline__ void loader(const u64* src, const LaneDesc& d, const StepParams& p, int K, int n, u32* ring,
                                       u32* prod, const u32* cons, WaitAcc* acc_in = nullptr, WaitAcc* acc_out = nullptr) {
    int lrow = d.row0 - K;
    if (WRAPY && lrow < 0) lrow += p.h;
    const u32* g = reinterpret_cast<const u32*>(src + (i64)(lrow + p.R) * p.pitch + (d.col + 1));
    const i64 step = 2 * p.pitch, wrapback = 2 * (i64)p.h * p.pitch;
    u32 freed = 0;
    int slot = 0;
    auto issue = [&](int j) {
        if (j >= kPipeRing0) ctr_wait<true>(cons, freed, (u32)(j + 1 - kPipeRing0), acc_out);  // slot j % ring free
        u32* l = ring + slot * kRowU32;
        __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)l, 4, 0, 0);
        __builtin_amdgcn_global_load_lds((glb_void_t*)(g + 1), (lds_void_t*)(l + 64), 4, 0, 0);
        slot = slot + 1 == kPipeRing0 ? 0 : slot + 1;
        g += step;
        if (WRAPY) {
            ++lrow;
            const bool w = lrow == p.h;
            lrow = w ? 0 : lrow;
            g = w ? g - wrapback : g;
        }
    };
    for (int j = 0; j < kPipeLoadAhead; ++j) issue(j);
    int i = 0;
    for (; i + kPipeLoadAhead < n; ++i) {
        const u64 s0 = PIPE_STAMPS && acc_in ? __builtin_amdgcn_s_memtime() : 0;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (kPipeLoadAhead - 1)) : "memory");
        if (PIPE_STAMPS && acc_in) acc_in->cy += __builtin_amdgcn_s_memtime() - s0;
        ctr_store<true>(prod, (u32)(i + 1));
        issue(i + kPipeLoadAhead);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ctr_store<true>(prod, (u32)n);
}

// Compile-time loop: f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>).
template <class F, int... R>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, R...>) {
    (f(std::integral_constant<int, R>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// A compute stage's input: the previous wave's rows from its ring of RIN slots.  Every stage's loops
// are unrolled so that each row's slot is a compile-time constant: ring accesses are one DS
// instruction with an immediate offset and no address arithmetic.
template <int RIN>
struct RingIn {
    const u32* ring;  // this lane's lo word of slot 0 (hi at +64)
    const u32* prod;  // rows the producer has published
    u32* cons;        // rows this wave has consumed (their slots are free)
    u32 avail = 0;    // cached *prod
    u32 pv = 0;       // an early read of *prod (peek), used by the next ensure
    WaitAcc acc;      // (PIPE_STAMPS)
    __device__ __forceinline__ void peek() { pv = __hip_atomic_load(prod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
    // rows < need are published (the peeked value first, then a bounded wait)
    __device__ __forceinline__ void ensure(u32 need, bool peeked = false) {
        if (peeked) avail = max(avail, (u32)__builtin_amdgcn_readfirstlane(pv));
        ctr_wait(prod, avail, need, PIPE_STAMPS ? &acc : nullptr);
    }
    template <int SLOT>
    __device__ __forceinline__ uint2 read() const {
        return make_uint2(ring[(SLOT % RIN) * kRowU32], ring[(SLOT % RIN) * kRowU32 + 64]);
    }
    // rows < n have been used (their reads completed): their slots may be refilled
    __device__ __forceinline__ void consumed(u32 n) { ctr_store(cons, n); }
};

// A stage's output: the next wave's ring (kSlots = kPipeRing), or the destination buffer.
struct RingOut {
    static constexpr int kSlots = kPipeRing;
    u32* ring;
    u32* prod;
    const u32* cons;  // the consumer's progress
    u32 freed = 0;    // cached *cons
    u32 cv = 0;       // an early read of *cons
    WaitAcc acc;      // (PIPE_STAMPS)
    __device__ __forceinline__ void peek() { cv = __hip_atomic_load(cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
    // slots of rows < end are free (rows < end - kSlots consumed)
    __device__ __forceinline__ void reserve(u32 end, bool peeked = false) {
        if (end <= (u32)kSlots) return;
        if (peeked) freed = max(freed, (u32)__builtin_amdgcn_readfirstlane(cv));
        ctr_wait(cons, freed, end - kSlots, PIPE_STAMPS ? &acc : nullptr);
    }
    template <int SLOT>
    __device__ __forceinline__ void put(u32 lo, u32 hi) {
        ring[(SLOT % kSlots) * kRowU32] = lo;
        ring[(SLOT % kSlots) * kRowU32 + 64] = hi;
    }
    __device__ __forceinline__ void publish(u32 rows) { ctr_store(prod, rows); }
};

struct GlobalOut {
    static constexpr int kSlots = 1;
    WaitAcc acc;  // (never waits)
    uint2* st;
    i64 stride;  // pitch, or 0 for halo/idle lanes (their own trash word)
    __device__ __forceinline__ void peek() {}
    __device__ __forceinline__ void reserve(u32, bool = false) {}
    template <int SLOT>
    __device__ __forceinline__ void put(u32 lo, u32 hi) {
        *st = make_uint2(lo, hi);
        st += stride;
    }
    __device__ __forceinline__ void publish(u32) {}
};

// Stream n input rows through an L-level pipeline: outputs rows L .. n-L-1 of the stream (n - 2L
// rows; input row r emits output row r - 2L).  Rows are held in a 6-row register queue q (row x in
// q[(x - i0) % 6]) refilled one triple at a time, kPipeU rows ahead.
template <int L, int RIN, class Out>
__device__ __forceinline__ void stage(RingIn<RIN>& in, Out& out, int n) {
    constexpr int U = RIN;                        // steady rows per iteration: the slot pattern repeats
    constexpr int i0 = ((2 * L + 2) / 3) * 3;     // fill rows (first multiple of 3 with the window full)
    static_assert(U % 6 == 0 && U % kPipeU == 0 && U % Out::kSlots == 0 && i0 < RIN && kPipeU % 3 == 0, "slot pattern");
    Pipe<L> P;
    u32 lo, hi;
    // fill: rows 0 .. i0-1 one by one, outputs published per row
    static_for<i0>([&](auto R) {
        constexpr int r = decltype(R)::value;
        if (r < n) {
            in.ensure((u32)(r + 1));
            const uint2 v = in.template read<r>();
            lo = v.x;
            hi = v.y;
            // released row by row: the producer may need the slot before the fill ends (the loader
            // publishes row x only after issuing row x + kPipeLoadAhead)
            in.consumed((u32)(r + 1));
            if constexpr (r < 2 * L) {
                advance<L, r % 3, true>(P, lo, hi, r);
            } else {
                advance<L, r % 3, false>(P, lo, hi, r);
                out.reserve((u32)(r - 2 * L + 1));
                out.template put<r - 2 * L>(lo, hi);
                out.publish((u32)(r - 2 * L + 1));
            }
        }
    });
    if (n <= i0) {
        in.consumed((u32)n);
        return;
    }
    in.consumed((u32)i0);
    uint2 q[kPipeU];
    in.ensure((u32)min(i0 + kPipeU, n));
    static_for<kPipeU>([&](auto J) {
        constexpr int j = decltype(J)::value;
        q[j] = i0 + j < n ? in.template read<i0 + j>() : make_uint2(0, 0);
    });
    // U rows from row i (i - i0 a multiple of U, so every slot below is a constant); TAIL: stop at n
    // Synchronisation every S rows (kPipeSync): at a group's first row the output slots are
    // reserved and both counters are read early (peek); at its last row the outputs are published, the
    // inputs released, and the queue registers of the group refilled kPipeU rows ahead.
    constexpr int S = kPipeSync;
    static_assert(kPipeU % S == 0 && 3 % S == 0, "sync group");
    auto body = [&](auto tail, int i) {
        constexpr bool TAIL = decltype(tail)::value;
        static_for<U>([&](auto R) {
            constexpr int r = decltype(R)::value;
            if (TAIL && i + r >= n) return;
            if constexpr (r % S == 0) {
                if (!TAIL) {
                    out.reserve((u32)(i + r - 2 * L + S), true);
                    in.peek();
                    out.peek();
                }
            }
            if (TAIL) out.reserve((u32)(i + r - 2 * L + 1));
            lo = q[r % kPipeU].x;
            hi = q[r % kPipeU].y;
            advance<L, r % 3, false>(P, lo, hi, i + r);
            out.template put<i0 - 2 * L + r>(lo, hi);
            if (TAIL || r % S == S - 1) out.publish((u32)(i + r - 2 * L + 1));
            if constexpr (r % S == S - 1) {
                in.consumed((u32)(i + r + 1));
                constexpr int a = r - (S - 1) + kPipeU;  // rows i+a .. i+a+S-1 refill q[(r-S+1) % kPipeU ..]
                const int nx = i + a;
                if (!TAIL || nx + S <= n) {  // (wave-uniform; the steady loop never reads past n)
                    in.ensure((u32)(nx + S), !TAIL);
                    static_for<S>([&](auto J) {
                        constexpr int j = decltype(J)::value;
                        q[(r - (S - 1) + j) % kPipeU] = in.template read<i0 + a + j>();
                    });
                } else if (nx < n) {
                    in.ensure((u32)n);
                    static_for<S>([&](auto J) {
                        constexpr int j = decltype(J)::value;
                        if (nx + j < n) q[(r - (S - 1) + j) % kPipeU] = in.template read<i0 + a + j>();
                    });
                }
                if (S == 3 || r % 3 == 2) __builtin_amdgcn_sched_barrier(0);
            }
        });
    };
    int i = i0;
    for (; i + U + kPipeU <= n; i += U) body(std::false_type{}, i);
    body(std::true_type{}, i);  // fewer than U + kPipeU rows left: two tail passes
    if (i + U < n) body(std::true_type{}, i + U);
    in.consumed((u32)n);
}

// NW waves: wave 0 loads, waves 1 .. NW-1 compute L generations each (K = (NW - 1) L per pass).
// At most 102 VGPRs (5 waves per SIMD): two workgroups of 9 waves per CU at any L (unbounded, L = 4
// took 167 VGPRs and ran one workgroup per CU)
template <int NW, int L, bool WRAPY>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(5))) void step_pipe(const u64* __restrict__ src, u64* __restrict__ dst,
                                                     const LaneDesc* __restrict__ plan, StepParams p) {
    // Progress (no wait cycle): a consumer that has released rows < c waits for at most rows < c + kPipeU
    // (+ the producer's publish group of 3); the producer of those rows needs slots of rows < c + kPipeU + 3
    // (compute ring: kPipeRing >= kPipeU + 3) or, the loader, of rows < c + kPipeU + kPipeLoadAhead.
    static_assert(NW >= 2 && kPipeRing >= kPipeU + 3 && kPipeU % 3 == 0 &&
                      kPipeRing0 >= kPipeLoadAhead + kPipeU && kPipeLoadAhead <= 31,
                  "ring sizes");
    extern __shared__ __attribute__((aligned(16))) u32 pipe_lds[];
    constexpr int K = (NW - 1) * L;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaneDesc d = plan[(i64)blockIdx.x * kWaveLanes + lane];
    const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
    if (nrows <= 0) return;  // padding tile (uniform over the workgroup)
    // ring 0 (loader -> wave 1), rings 1 .. NW-2 (wave w -> wave w + 1), then prod[NW], cons[NW]
    auto ring_of = [&](int r) { return pipe_lds + (r == 0 ? 0 : (kPipeRing0 + (r - 1) * kPipeRing) * kRowU32); };
    u32* ctr = pipe_lds + (kPipeRing0 + (NW - 2) * kPipeRing) * kRowU32;
    if (threadIdx.x < 2 * NW) ctr[threadIdx.x] = 0;
    __syncthreads();
#if PIPE_STAMPS
    const u64 t_start = __builtin_amdgcn_s_memtime();
    auto stamp = [&](const WaitAcc& a, const WaitAcc& b) {
        const i64 slot = ((i64)blockIdx.x * NW + wv) * 4;
        if (lane == 0 && slot + 3 < (i64)kPipeStampWaves * 4) {
            g_pipe_stamps[slot] = __builtin_amdgcn_s_memtime() - t_start;
            g_pipe_stamps[slot + 1] = a.cy;
            g_pipe_stamps[slot + 2] = b.cy;
            g_pipe_stamps[slot + 3] = a.n + b.n;
        }
    };
#endif
    if (wv == 0) {
#if PIPE_STAMPS
        WaitAcc ai, ao;
        loader<WRAPY>(src, d, p, K, nrows + 2 * K, ring_of(0), ctr, ctr + NW, &ai, &ao);
        stamp(ai, ao);
#else
        loader<WRAPY>(src, d, p, K, nrows + 2 * K, ring_of(0), ctr, ctr + NW);
#endif
        return;
    }
    const int st = wv - 1;                     // compute stage
    const int n = nrows + 2 * K - 2 * st * L;  // its input rows
    auto run = [&](auto in) {
        in.ring = ring_of(st) + lane;
        in.prod = ctr + st;
        in.cons = ctr + NW + st;
        if (wv == NW - 1) {
            const bool out_lane = d.flags & LANE_STORE;
            GlobalOut o;
            o.st = out_lane ? reinterpret_cast<uint2*>(dst + (i64)(d.row0 + p.R) * p.pitch + (d.col + 1))
                            : reinterpret_cast<uint2*>(p.trash + ((i64)((blockIdx.x * NW + wv) & (kTrashWaves - 1)) * 64 + lane));
            o.stride = out_lane ? p.pitch : 0;
            stage<L>(in, o, n);
#if PIPE_STAMPS
            stamp(in.acc, o.acc);
#endif
        } else {
            RingOut o;
            o.ring = ring_of(wv) + lane;
            o.prod = ctr + wv;
            o.cons = ctr + NW + wv;
            stage<L>(in, o, n);
#if PIPE_STAMPS
            stamp(in.acc, o.acc);
#endif
        }
    };
    if (st == 0)
        run(RingIn<kPipeRing0>{});
    else
        run(RingIn<kPipeRing>{});
}

template <int NW, int L>
const void* pipe_kernel_wrap(bool wrapy) {
    return wrapy ? (const void*)step_pipe<NW, L, true> : (const void*)step_pipe<NW, L, false>;
}
template <int NW>
const void* pipe_kernel_nw(int L, bool wrapy) {
    switch (L) {
        case 1: return pipe_kernel_wrap<NW, 1>(wrapy);
        case 2: return pipe_kernel_wrap<NW, 2>(wrapy);
        case 3: return pipe_kernel_wrap<NW, 3>(wrapy);
        case 4: return pipe_kernel_wrap<NW, 4>(wrapy);
        default: return nullptr;
    }
}
const void* pipe_kernel(int nw, int L, bool wrapy) {
    switch (nw) {
        case 5: return pipe_kernel_nw<5>(L, wrapy);
        case 7: return pipe_kernel_nw<7>(L, wrapy);
        case 9: return pipe_kernel_nw<9>(L, wrapy);
        case 11: return pipe_kernel_nw<11>(L, wrapy);
        case 13: return pipe_kernel_nw<13>(L, wrapy);
        case 16: return pipe_kernel_nw<16>(L, wrapy);
        default: return nullptr;
    }
}

const void* pipe_kernel_checked(int nw, int L, bool wrapy) {
    const void* f = pipe_kernel(nw, L, wrapy);
    if (!f) throw Error(strprintf("step_pipe: no kernel for %d waves x %d levels", nw, L));
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) throw Error("step_pipe: no current HIP device");
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert({dev, f}).second) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pipe_lds_bytes(nw));
        if (e != hipSuccess) {
            done.erase({dev, f});
            throw Error(strprintf("step_pipe: hipFuncSetAttribute: %s", hipGetErrorString(e)));
        }
    }
    return f;
}

}  // namespace

#ifdef GOL_PIPE_STAMPS
std::vector<u64> pipe_stamps(size_t waves) {
    std::vector<u64> v(std::min<size_t>(waves, (size_t)kPipeStampWaves) * 4);
    if (hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_pipe_stamps), v.size() * sizeof(u64)) != hipSuccess)
        throw Error("step_pipe: cannot read the stamps");
    return v;
}
#endif

bool pipe_fault() {
    u32 v = 0, z = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_pipe_fault), sizeof(v)) != hipSuccess)
        throw Error("step_pipe: cannot read the fault flag");
    if (v && hipMemcpyToSymbol(HIP_SYMBOL(g_pipe_fault), &z, sizeof(z)) != hipSuccess)
        throw Error("step_pipe: cannot clear the fault flag");
    return v != 0;
}

size_t pipe_lds_bytes(int nw) {
    return ((size_t)(kPipeRing0 + (nw - 2) * kPipeRing) * kRowU32 + 2 * (size_t)nw) * sizeof(u32);
}

bool pipe_supported(int nw, int L) { return pipe_kernel(nw, L, true) != nullptr; }

int pipe_blocks_per_cu(int nw, int L, bool wrapy) {
    const void* f = pipe_kernel_checked(nw, L, wrapy);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 64 * nw, pipe_lds_bytes(nw)) != hipSuccess) return 0;
    return nb;
}

void launch_step_pipe(int nw, int L, const u64* src, u64* dst, const LaneDesc* plan, i64 n_tiles, const StepParams& p,
                      hipStream_t s) {
    const void* f = pipe_kernel_checked(nw, L, (p.flags & STEP_WRAP_Y) != 0);
    if (p.flags & STEP_SEAM) throw Error("step_pipe: seam sources are not supported");
    StepParams pp = p;
    if (!pp.trash) pp.trash = trash_of_current_device();
    void* args[] = {(void*)&src, (void*)&dst, (void*)&plan, (void*)&pp};
    const hipError_t e = hipLaunchKernel(f, dim3((unsigned)n_tiles), dim3(64 * nw), args, pipe_lds_bytes(nw), s);
    if (e != hipSuccess) throw Error(strprintf("step_pipe launch failed: %s", hipGetErrorString(e)));
}

}  // namespace hipk
}  // namespace gol
