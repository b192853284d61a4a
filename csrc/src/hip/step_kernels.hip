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
#include "tile_device.hpp"

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

template <int NW, bool WRAPY, int LV, bool IP>
__global__ __launch_bounds__(64 * NW) void step_tile(const u64* __restrict__ src, u64* __restrict__ dst,
                                                     const LaneDesc* __restrict__ plan, StepParams p, int K) {
    extern __shared__ __attribute__((aligned(16))) u32 tile_lds[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaneDesc d = plan[(i64)blockIdx.x * kWaveLanes + lane];
    const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
    if (nrows <= 0) return;  // padding tile (uniform over the workgroup)
    tile_item<NW, WRAPY, LV, IP>(src, dst, d, nrows, p, K, tile_lds, wv, lane, blockIdx.x);
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
    fold_item<NW, WRAPY, LV, IP>(src, dst, d, nrows, p, K, tile_lds, wv, lane, blockIdx.x);
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
