// gol-mi355x: step_flow — a whole superstep (several register-pipeline passes) as ONE launch, its
// work items scheduled by data dependencies instead of kernel boundaries.
//
// The pass kernels (step_temporal, step_kernels.hip) run a superstep of G generations as G / K
// launches: every launch streams the board once through K levels of the register pipeline and the
// next pass starts only when the LAST wave of the previous one has finished.  On MI355X the co-resident
// waves of a SIMD do not finish together (VALU issue is arbitrated by age), so every pass boundary
// idles most wave slots while its slowest waves drain, and the first waves of the next pass start
// late (docs/PERFORMANCE.md §6: ~20 us of a 20-generation superstep).  Here:
//
//  * A superstep's passes are cut into work items (FlowItem, plan.hpp build_flow_plan): one plan wave
//    of one pass each (the same segments and lane layout as step_temporal's plans), listed in ONE
//    global ticket order: every item of pass j comes before any item of pass j + 1, and inside a pass
//    the items run down the board in row bands (with the torus wrap, pass j starts one band further
//    down than pass j - 1, so its first items read only the rows pass j - 1 finished first).
//  * A persistent grid of waves (one full round of resident slots) takes tickets from device
//    counters; a wave that draws item t waits for the items t depends on (host-computed: the items of
//    pass j - 1 that WRITE rows it reads, and those that READ rows it overwrites — two buffers
//    alternate, so pass j + 1 writes the buffer pass j reads), streams the item with the
//    step_temporal wave (wave_runner.hpp), and publishes its completion flag.  So an early-finishing
//    wave starts on pass j + 1 as soon as its neighbourhood of pass j is done, instead of idling at a
//    kernel boundary; only the superstep's end drains.
//  * Ticket sequences.  One device-wide counter costs ~12 ns per draw, serialised (same-address
//    atomics: tools/ticket_probe.hip, profiles/ticket_probe.txt), and a superstep draws ~15000 tickets
//    (items plus each wave's final draw): ~180 us, the whole budget.  So item t belongs to sequence
//    t % nseq, and sequence s is drawn only by the waves running on XCD s (HW_REG_XCC_ID; nseq = the
//    device's XCDs): eight counters in parallel, ~2.5 ns per draw device-wide.
//  * Deadlock freedom (no residency assumption, no cooperative launch): an item depends only on items
//    with SMALLER tickets, and each sequence is drawn in increasing order by running waves, which work
//    on a drawn item without waiting for anything but its dependencies.  Let t be the smallest
//    unfinished item and s its sequence; its dependencies are finished.  If t is drawn, its wave runs it
//    (with PF, the item the wave is still on is an earlier one of sequence s: finished).  If not, every
//    drawn item of sequence s is smaller, hence finished, so the waves of XCD s are free and the next
//    draw on s is t: XCD s has a wave of the launch (the hardware deals workgroups to every XCD, none
//    exits before its sequence is drawn out, and nothing else holds its CUs for ever).  By induction
//    every item finishes.  Engines sharing a device (thread ranks) use one sequence (nseq = 1): then the
//    argument needs no XCD at all (another engine's grid may hold an XCD).  Every wait is also bounded
//    (2 s of s_memrealtime), after which the wave records a fault (FlowCtl::fault, read by the engine
//    at every board readout) and goes on, so a bug cannot hang the GPU.
//  * Cross-CU visibility (MI355X_MICROARCH.md, "inter-workgroup visibility", valid hand-off forms):
//    every board-row load and store of an item is an agent-scope relaxed atomic, `global_load/store
//    ... sc1` (write-through stores, loads that bypass the CU's L1); a wave's stores are complete at
//    its `s_waitcnt vmcnt(0)`, after which ONE lane stores the item's flag (`sc1`); a consumer polls
//    flags with `sc1` loads and issues its row loads only after every flag matched.  Flags hold the
//    launch's epoch (host-counted, FlowArgs::epoch), so they are never reset between launches, and the
//    ticket counters are double-buffered by epoch parity: launch e zeroes the ones launch e + 1 draws
//    from (no completion count, no last-wave-out reset).  (No scalar-cache stores or atomics anywhere:
//    every store and atomic here is a vector memory instruction.)
//  * Kernel boundaries still order supersteps (exchanges and readouts see finished boards).  The epoch
//    is a launch argument, so a flow launch is not replayed from a captured graph (it is one launch per
//    superstep: a graph replay costs more than a direct launch, MI355X_MICROARCH.md graph-replay-floor).
//
// Reference: the generation loop gol-main.c:93-116 and its per-generation launch + device sync,
// gol-with-cuda.cu:264-284.
#include <mutex>
#include <set>
#include <utility>

#include "gol/hip_kernels.hpp"
#include "stencil_device.hpp"
#include "wave_runner.hpp"
#include "tile_device.hpp"

namespace gol {
namespace hipk {

namespace {

constexpr u64 kFlowWaitTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz): no real wait is that long

// Wait until every dependency of an item carries the running launch's epoch.  One lane per
// dependency (64 per sweep), `sc1` loads, a short sleep between polls.  Every branch here is on a
// wave-uniform value (ballot, readfirstlane): a branch on a per-lane atomic load (each lane's load is
// its own atomic, so the compiler must treat the value as divergent) makes the loops divergent, and
// the structurizer then moved lane 0's flag store and next ticket draw out of step with the other
// lanes' item loop (seen in the ISA of the first version).
__device__ __forceinline__ void flow_wait(const FlowArgs& a, u32 dep_off, u32 ndeps, u32 target, int lane) {
    for (u32 b = 0; b < ndeps; b += 64) {
        const bool act = b + (u32)lane < ndeps;
        const u32 dep = act ? a.deps[dep_off + b + (u32)lane] : 0u;
        u64 t0 = 0;
        for (int spin = 0;; ++spin) {
            const u32 v = act ? __hip_atomic_load(&a.flags[dep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : target;
            const bool ready = (int)(v - target) >= 0;
            if (__builtin_amdgcn_ballot_w64(!ready) == 0) break;
            if (spin == 0) {
                t0 = __builtin_amdgcn_s_memrealtime();
            } else if ((spin & 15) == 0) {  // (the time limit, or a fault elsewhere: every 16th poll)
                const u32 fault = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&a.ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (__builtin_amdgcn_s_memrealtime() - t0 > kFlowWaitTicks || fault != 0) {
                    __hip_atomic_store(&a.ctl->fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (all lanes, one word)
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(4);
        }
    }
    asm volatile("" ::: "memory");  // the item's loads stay after the wait
}

// Exchange-overlapped launches: an item that reads ghost cells waits for the comm stream's flag
// (hipStreamWriteValue32 of the launch's epoch after the RCCL group), then acquires at agent scope
// before its loads.  The flag is a single word polled with system-scope loads (the write comes from
// another queue's packet processor, not from a wave).
__device__ __forceinline__ void flow_wait_exch(const FlowArgs& a) {
    u64 t0 = 0;
    for (int spin = 0;; ++spin) {
        const u32 v = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&a.ctl->exch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        if ((int)(v - a.epoch) >= 0) break;
        if (spin == 0) t0 = __builtin_amdgcn_s_memrealtime();
        const u32 fault = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&a.ctl->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (__builtin_amdgcn_s_memrealtime() - t0 > kFlowWaitTicks || fault != 0) {
            __hip_atomic_store(&a.ctl->fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (all lanes, one word)
            break;
        }
        __builtin_amdgcn_s_sleep(8);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The ticket sequence of the calling wave (kFlowSeqs = one per XCD, or one for all) and its counter for
// this launch; block 0's first wave zeroes the counters of the next launch (double-buffered by epoch).
__device__ __forceinline__ u32* flow_sequence(const FlowArgs& a, u32& seq, int lane) {
    seq = 0;
    if (a.nseq > 1) {
        u32 xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        seq = xcc % a.nseq;
    }
    if (blockIdx.x == 0 && threadIdx.x < 64)  // (wave 0 of block 0: lanes 0-7 one counter each, the rest repeat them)
        __hip_atomic_store(&a.ctl->next[(a.epoch + 1u) & 1u][lane & (kFlowSeqs - 1)][0], 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return &a.ctl->next[a.epoch & 1u][seq][0];
}

// Draw the next item of the wave's sequence: item seq + nseq x (draw number); >= n_items when the
// sequence is drawn out.  An all-lane atomic adding 1 from lane 0 and 0 from the others.
__device__ __forceinline__ u32 flow_draw(const FlowArgs& a, u32* ctr, u32 seq, int lane) {
    const u32 i = __hip_atomic_fetch_add(ctr, lane == 0 ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(i) * a.nseq + seq;
}

template <int K, int ROWS, bool COH = true>
__device__ __forceinline__ void flow_item(const u64* src, u64* dst, const LaneDesc& d, int nrows, const StepParams& p,
                                          i64 wave) {
    WaveRunner<K, ROWS, COH> w(src, dst, d, nrows, p, wave);
    w.run();
}

// The depths one flow kernel instantiates (a superstep's cut uses any of them).
#define FLOW_DEPTHS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8)

// Three waves per SIMD, as step_temporal<8> (163 VGPRs): the persistent item loop around the
// pipelines needs ~190 by default, and capping it spills 3-5 registers to scratch, reloaded once per
// item (outside the row loops).
// PF: a wave draws its NEXT ticket when it starts an item, so the draw's latency (a contended atomic,
// ~1 us under load) hides behind the item instead of preceding the next one.  The deadlock argument
// holds: a wave holding a drawn-but-unstarted ticket is working on a smaller one.
// (KONLY, COH: measurement variants of the GOL_FLOW_EXPERIMENTS build only — one depth instantiated,
// plain row loads and stores; the production kernel is KONLY = 0, COH = true.)
template <int ROWS, bool PF, int KONLY = 0, bool COH = true>
__global__ __launch_bounds__(64 * kWavesPerBlock) __attribute__((amdgpu_waves_per_eu(3))) void step_flow(FlowArgs a,
                                                                                                    StepParams p) {
    const int lane = threadIdx.x & 63;
    const i64 wave = (i64)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const u32 target = a.epoch;
    // (No lane-conditional code in this loop: a `lane == 0` branch around the ticket draw or the flag
    // store let the compiler thread that condition across the loop's back edge, and lanes 1-63 went on
    // re-running ticket 0 — the first version hung.  The draw is an all-lane atomic adding 1 from lane
    // 0 and 0 from the others; the flag is stored by every lane to the same word.)
    u32 seq = 0;
    u32* ctr = flow_sequence(a, seq, lane);
    u32 t = flow_draw(a, ctr, seq, lane);
    for (;;) {
        if (t >= a.n_items) break;
        u32 t_next = 0;  // (PF: a per-lane register until the item's end, so no wait is forced here)
        if constexpr (PF)
            t_next = __hip_atomic_fetch_add(ctr, lane == 0 ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the item's fields as wave-uniform values (they steer every branch below)
        const FlowItem* ip = a.items + t;
        const u32 depth = __builtin_amdgcn_readfirstlane(ip->depth);
        const u32 pass = __builtin_amdgcn_readfirstlane(ip->pass);
        const u32 dep_off = __builtin_amdgcn_readfirstlane(ip->dep_off);
        const u32 ndeps = __builtin_amdgcn_readfirstlane(ip->ndeps);
        flow_wait(a, dep_off, ndeps, target, lane);
        if (pass & FLOW_ITEM_EXCH) flow_wait_exch(a);
        const LaneDesc d = a.lanes[(i64)t * kWaveLanes + lane];
        const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
        const bool odd = pass & 1u;
        const u64* src = odd ? a.b : a.a;
        u64* dst = odd ? a.a : a.b;
        if (nrows > 0) {
            if constexpr (KONLY > 0) {
                if (depth == KONLY) flow_item<KONLY, ROWS, COH>(src, dst, d, nrows, p, wave);
            } else {
                switch (depth) {
#define DEPTH_CASE(K)                                             \
    case K:                                                     \
        flow_item<K, ROWS>(src, dst, d, nrows, p, wave);        \
        break;
                    FLOW_DEPTHS(DEPTH_CASE)
#undef DEPTH_CASE
                    default:
                        break;
                }
            }
        }
        // every store of the item has left the wave (write-through) before its flag does
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&a.flags[t], target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (PF)
            t = __builtin_amdgcn_readfirstlane(t_next) * a.nseq + seq;
        else
            t = flow_draw(a, ctr, seq, lane);
    }
}

// ---- tile items: one workgroup of NW waves per item (step_tile / step_tile_fold's device code) ----
// The ticket is drawn by wave 0 and broadcast through an LDS word past the tile buffers; wave 0 also
// waits for the item's dependencies, then a barrier releases the workgroup.  Every branch is on a
// workgroup-uniform value (barrier-published LDS word, readfirstlane), and only wave-granular code is
// conditional (wv == 0).  The deadlock argument is the wave kernel's with workgroups for waves.
template <int NW, bool WRAPY, int LV, bool IP, bool FOLD>
__global__ __launch_bounds__(64 * NW) void step_flow_tile(FlowArgs a, StepParams p, u32 ticket_slot) {
    extern __shared__ __attribute__((aligned(16))) u32 tile_lds[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u32* s_ticket = tile_lds + ticket_slot;
    const u32 target = a.epoch;
    u32 seq = 0;
    u32* ctr = flow_sequence(a, seq, lane);
    for (;;) {
        if (wv == 0) {
            const u32 t = flow_draw(a, ctr, seq, lane);
            if (t < a.n_items) {
                const FlowItem* ip = a.items + t;
                flow_wait(a, __builtin_amdgcn_readfirstlane(ip->dep_off), __builtin_amdgcn_readfirstlane(ip->ndeps),
                          target, lane);
                if (__builtin_amdgcn_readfirstlane(ip->pass) & FLOW_ITEM_EXCH) flow_wait_exch(a);
            }
            *s_ticket = t;  // (every lane, the same word)
        }
        __syncthreads();
        const u32 t = __builtin_amdgcn_readfirstlane(*s_ticket);
        __syncthreads();  // every wave has read the slot before wave 0 may rewrite it
        if (t >= a.n_items) break;
        const FlowItem* ip = a.items + t;
        const int K = (int)__builtin_amdgcn_readfirstlane(ip->depth);
        const u32 pass = __builtin_amdgcn_readfirstlane(ip->pass);
        const LaneDesc d = a.lanes[(i64)t * kWaveLanes + lane];
        const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
        const bool odd = pass & 1u;
        const u64* src = odd ? a.b : a.a;
        u64* dst = odd ? a.a : a.b;
        if (nrows > 0) {
            if constexpr (FOLD)
                fold_item<NW, WRAPY, LV, IP, true>(src, dst, d, nrows, p, K, tile_lds, wv, lane, blockIdx.x);
            else
                tile_item<NW, WRAPY, LV, IP, true>(src, dst, d, nrows, p, K, tile_lds, wv, lane, blockIdx.x);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's output rows have left it
        __syncthreads();                                   // ... and every other wave's
        if (wv == 0) __hip_atomic_store(&a.flags[t], target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// tile variants of the flow kernel: double-buffered tiles with 4 generations per LDS pass, or in place
// with 2 (the engine's defaults for 8 waves, step_kernels.hip tile_bits), folded or plain
template <bool WRAPY, bool FOLD>
const void* flow_tile_variant(u32 flags) {
    if (flags & STEP_TILE_INPLACE)
        return (flags & STEP_TILE_L2) ? (const void*)step_flow_tile<8, WRAPY, 2, true, FOLD> : nullptr;
    return (flags & STEP_TILE_L4) ? (const void*)step_flow_tile<8, WRAPY, 4, false, FOLD> : nullptr;
}
const void* flow_tile_kernel_for(int nw_per_wg, u32 flags) {
    if (nw_per_wg != 8) return nullptr;
    const bool fold = flags & STEP_TILE_FOLD;
    if (flags & STEP_WRAP_Y) return fold ? flow_tile_variant<true, true>(flags) : flow_tile_variant<true, false>(flags);
    return fold ? flow_tile_variant<false, true>(flags) : flow_tile_variant<false, false>(flags);
}

const void* flow_kernel_for(u32 flags, u32 variant = 0) {
#ifdef GOL_FLOW_EXPERIMENTS
    // bit 1: only depth 8 instantiated; bit 2 (with bit 1): plain loads and stores (y-wrapped tiles only)
    if ((variant & 6u) == 2u) return (const void*)step_flow<ROWS_WRAP, false, 8, true>;
    if ((variant & 6u) == 6u) return (const void*)step_flow<ROWS_WRAP, false, 8, false>;
#endif
    if (variant & 1u)
        return (flags & STEP_WRAP_Y) ? (const void*)step_flow<ROWS_WRAP, true> : (const void*)step_flow<ROWS_GHOST, true>;
    return (flags & STEP_WRAP_Y) ? (const void*)step_flow<ROWS_WRAP, false> : (const void*)step_flow<ROWS_GHOST, false>;
}

}  // namespace

bool flow_depth_supported(int k) {
    switch (k) {
#define DEPTH_CASE(K) \
    case K:         \
        return true;
        FLOW_DEPTHS(DEPTH_CASE)
#undef DEPTH_CASE
        default:
            return false;
    }
}

int flow_max_depth() { return 8; }

int flow_blocks_per_cu(u32 flags) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, flow_kernel_for(flags), 64 * kWavesPerBlock, 0) != hipSuccess ||
        nb < 1)
        return 1;
    return std::min(nb, 32 / kWavesPerBlock);
}

void launch_step_flow(const FlowArgs& a, i64 n_blocks, const StepParams& p, hipStream_t s) {
    if (p.flags & STEP_SEAM) throw Error("step_flow: seam-reading passes are not supported");
    if (n_blocks < 1) throw Error("step_flow: empty grid");
    StepParams pp = p;
    if (!pp.trash) pp.trash = trash_of_current_device();
    FlowArgs aa = a;
    void* args[] = {(void*)&aa, (void*)&pp};
    hipError_t e = hipLaunchKernel(flow_kernel_for(p.flags, a.variant), dim3((unsigned)n_blocks), dim3(64 * kWavesPerBlock),
                                   args, 0, s);
    if (e != hipSuccess) throw Error(strprintf("step_flow launch failed: %s", hipGetErrorString(e)));
}

bool flow_tile_supported(int nw_per_wg, u32 flags) { return flow_tile_kernel_for(nw_per_wg, flags) != nullptr; }

// LDS of a flow tile item: the tile kernel's (tile_lds_bytes), then the 16-byte ticket slot
static size_t flow_tile_lds_bytes(i64 rows, int k, int nw, u32 flags) { return tile_lds_bytes(rows, k, nw, flags) + 16; }

i64 flow_tile_max_rows(int k, int nw_per_wg, u32 flags) {
    // the largest rows whose tile plus the ticket slot fit the 160 KiB
    i64 r = tile_max_rows(k, nw_per_wg, flags);
    while (r > 0 && flow_tile_lds_bytes(r, k, nw_per_wg, flags) > kMaxLdsBytes) --r;
    return r;
}

static const void* flow_tile_checked(int nw_per_wg, u32 flags) {
    const void* f = flow_tile_kernel_for(nw_per_wg, flags);
    if (!f) throw Error(strprintf("step_flow: no tile variant for %d waves per workgroup, flags 0x%x", nw_per_wg, flags));
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> attr_set;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) throw Error("step_flow: no current HIP device");
    std::lock_guard<std::mutex> lk(mu);
    if (attr_set.insert({dev, f}).second) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLdsBytes);
        if (e != hipSuccess) {
            attr_set.erase({dev, f});
            throw Error(strprintf("step_flow: hipFuncSetAttribute: %s", hipGetErrorString(e)));
        }
    }
    return f;
}

int flow_tile_blocks_per_cu(int nw_per_wg, i64 rows, int kmax, u32 flags) {
    const void* f = flow_tile_checked(nw_per_wg, flags);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 64 * nw_per_wg, flow_tile_lds_bytes(rows, kmax, nw_per_wg, flags)) !=
            hipSuccess ||
        nb < 1)
        return 1;
    return std::min(nb, 8);
}

void launch_step_flow_tile(int nw_per_wg, const FlowArgs& a, i64 n_blocks, i64 rows, int kmax, const StepParams& p,
                           hipStream_t s) {
    if (n_blocks < 1) throw Error("step_flow: empty grid");
    if (kmax < 1 || kmax > 64) throw Error(strprintf("step_flow: tile depth %d outside 1..64", kmax));
    const size_t bytes = flow_tile_lds_bytes(rows, kmax, nw_per_wg, p.flags);
    if (rows < 1 || bytes > kMaxLdsBytes)
        throw Error(strprintf("step_flow: %lld-row tiles at depth %d exceed the LDS", (long long)rows, kmax));
    if ((p.flags & STEP_TILE_FOLD) && rows < kFoldMinRows)
        throw Error(strprintf("step_flow: a folded tile plan needs at least %d rows", kFoldMinRows));
    const void* f = flow_tile_checked(nw_per_wg, p.flags);
    StepParams pp = p;
    if (!pp.trash) pp.trash = trash_of_current_device();
    FlowArgs aa = a;
    u32 slot = (u32)(tile_lds_bytes(rows, kmax, nw_per_wg, p.flags) / 4);
    void* args[] = {(void*)&aa, (void*)&pp, (void*)&slot};
    const hipError_t e = hipLaunchKernel(f, dim3((unsigned)n_blocks), dim3(64 * nw_per_wg), args, bytes, s);
    if (e != hipSuccess) throw Error(strprintf("step_flow (tiles) launch failed: %s", hipGetErrorString(e)));
}

bool flow_fault(FlowCtl* ctl, hipStream_t s) {
    u32 v = 0;
    if (hipMemcpyAsync(&v, &ctl->fault, sizeof(v), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        throw Error("flow_fault: cannot read the control block");
    if (v == 0) return false;
    // clear it, and the ticket counters of the faulted launch (its waves all left); the exchange flag
    // holds an epoch and stays
    if (hipMemsetAsync(ctl->next, 0, sizeof(ctl->next), s) != hipSuccess ||
        hipMemsetAsync(&ctl->fault, 0, sizeof(u32), s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        throw Error("flow_fault: cannot reset the control block");
    return true;
}

}  // namespace hipk
}  // namespace gol
