// gol-mi355x: host API of the hand-written gfx950 kernels (implemented in src/hip/*.hip).
//
// Kernel inventory (reference has one kernel, gol_kernel, gol-with-cuda.cu:189-262):
//   step_temporal<K>  — K generations of B3/S23 per pass over a bit-packed tile: wave64 column
//                       streaming, bit-sliced v_bitop3/v_alignbit adders, DPP wave_shr/shl lane
//                       exchange, K-deep register pipeline (temporal blocking), periodic wrap by
//                       load addressing.  Replaces gol_kernel + the per-generation sync/swap.
//   step_lds          — single-generation LDS-tiled variant (tile + ghost words staged in LDS);
//                       kept as a measured alternative (GOL_KERNEL=lds).
//   fill_ghost_cols   — x-periodic ghost words for widths that are not a multiple of 64.
//   fill_ghost_rows   — y-periodic ghost rows for a tile shorter than the halo depth.
//   init_fill/set_cells — device-side pattern init (reference: host loops over managed memory).
//   copy_regions      — batched strided copies: 2-D halo pack/unpack and self-neighbour copies.
//   reduce_board      — population + decomposition-invariant fingerprint.
//   naive_byte_step   — byte-per-cell, thread-per-cell yardstick of the reference's algorithm class
//                       (no printf), used only by the benchmark for comparison.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "gol/geometry.hpp"
#include "gol/plan.hpp"

namespace gol {
namespace hipk {

enum : u32 {
    STEP_WRAP_X = 1u << 0,  // LDS kernel: tile is its own E/W neighbour (w % 64 == 0); the temporal
                            // kernel gets x-wrap from its plan (build_plan(..., xwrap = true))
    STEP_WRAP_Y = 1u << 1,  // tile is its own N/S neighbour: rows are read modulo h, no ghost rows
    STEP_TILE_L2 = 1u << 4, // tile kernel: two generations per LDS pass (half the barriers)
    STEP_TILE_L4 = 1u << 6, // tile kernel: four generations per LDS pass
    STEP_TILE_INPLACE = 1u << 7,  // tile kernel: one tile buffer updated in place (twice the rows)
    STEP_TILE_FOLD = 1u << 8,     // tile kernel: 32-lane tiles folded in half (fold plans, plan.hpp)
    STEP_SEAM = 1u << 5,    // temporal kernel: rows < 0 are read from StepParams::above, rows >= h
                            // from StepParams::below (sub-tile first pass: the other half's edges)
};

// Rows the HIP engine allocates past the bottom halo: the temporal kernel's 3-row prefetch overrun
// + the trash row its halo lanes store into (and the tile kernel's over-read slack).
constexpr int kSlackRows = 32;

struct StepParams {
    i64 pitch;
    i32 h;
    i32 nw;
    i32 R;
    u32 flags;
    // STEP_SEAM: row r < 0 of the source is at above + r * pitch, row r >= h at below + (r - h) * pitch
    // (word c at + c + 1, like the source buffer's rows)
    const u64* above = nullptr;
    const u64* below = nullptr;
    // Where lanes that store nothing (halo / idle lanes) write instead: kTrashWaves x 64 words, one
    // word per (wave mod kTrashWaves, lane).  Filled in by the launch functions (ensure_trash).
    u64* trash = nullptr;
};
constexpr int kTrashWaves = 1024;
// Allocate the current device's trash buffer (call once per device before any launch or capture;
// thread safe).
void ensure_trash();
u64* trash_of_current_device();  // (throws when ensure_trash has not run on this device)

// Supported temporal depths (template instantiations).
bool step_depth_supported(int k);
// Resident 256-thread workgroups per CU of step_temporal<k> for the given STEP_* flags.
int step_blocks_per_cu(int k, u32 flags);
int max_step_depth();
// Launch K generations: src -> dst over the waves of `plan` (n_waves * 64 LaneDescs in device memory).
void launch_step(int k, const u64* src, u64* dst, const LaneDesc* plan, i64 n_waves, const StepParams& p,
                 hipStream_t s);
// LDS-resident temporal kernel (step_tile): one workgroup of `nw_per_wg` (4, 8, 16) waves per plan
// wave; `rows` = the plan's rows per chunk (<= tile_max_rows(k), the 160 KiB LDS limit).
constexpr size_t kMaxLdsBytes = 160 * 1024;
// Least chunk height of a folded-tile plan (STEP_TILE_FOLD): its segments are >= 14 rows tall.
constexpr int kFoldMinRows = 28;
i64 tile_max_rows(int k, int nw_per_wg, u32 flags);
int tile_blocks_per_cu(int nw_per_wg, i64 rows, int k, u32 flags);
void launch_step_tile(int nw_per_wg, int k, const u64* src, u64* dst, const LaneDesc* plan, i64 n_tiles, i64 rows,
                      const StepParams& p, hipStream_t s);
// step_resident (resident_kernel.hip): a run of G generations in one launch, one workgroup of `nw`
// (8, 16) waves per tile of `plan` (one tile per CU, all co-resident), each wave holding B rows of
// the tile's extended rows (nrows + 2 kmax) in registers; S supersteps (odd) of <= kmax generations,
// between which tiles exchange halos through HBM with their neighbour tiles (CSR nbr_off / nbr,
// plan.hpp resident_neighbours) and per-tile counters.  The result is in dst.
struct ResidentParams {
    i64 pitch;
    i32 h;
    i32 R;
    i32 G;       // generations of this launch
    i32 S;       // supersteps (odd), of G / S or G / S + 1 generations
    i32 kmax;    // halo rows of the tiles: >= ceil(G / S)
    u64 timeout_ticks;  // bound of every neighbour wait, in s_memrealtime ticks (100 MHz)
};
int resident_band_rows(int rows_needed);  // supported band height >= rows_needed (0: none)
int resident_blocks_per_cu(int nw, int B, bool wrapy);
void launch_step_resident(int nw, int B, bool wrapy, u64* src, u64* dst, const LaneDesc* plan, i64 n_tiles,
                          const u32* nbr_off, const u32* nbr, u32* counters, u32* status, const ResidentParams& rp,
                          hipStream_t s);
// step_pipe (pipe_kernel.hip): K = nw x L generations per launch, one workgroup of `nw` (4, 8, 12,
// 16) waves per plan wave (a segment of the plan, as step_tile), wave w computing levels
// w L + 1 .. (w + 1) L of the whole segment and handing its rows to wave w + 1 through an LDS ring.
size_t pipe_lds_bytes(int nw);
bool pipe_supported(int nw, int L);
int pipe_blocks_per_cu(int nw, int L, bool wrapy);
// True (and cleared) when a step_pipe wait timed out since the last call: the board is invalid.
bool pipe_fault();
#ifdef GOL_PIPE_STAMPS
// Diagnostic build: per-wave wait stamps of the last step_pipe launch (pipe_kernel.hip g_pipe_stamps)
std::vector<u64> pipe_stamps(size_t waves);
#endif
void launch_step_pipe(int nw, int L, const u64* src, u64* dst, const LaneDesc* plan, i64 n_tiles, const StepParams& p,
                      hipStream_t s);
// Single-generation LDS-tiled kernel over output rows [r0, r1) (all words).
void launch_step_lds(const u64* src, u64* dst, const Layout& L, i64 r0, i64 r1, u32 flags, hipStream_t s);

void launch_fill_ghost_cols(u64* buf, const Layout& L, i64 r_lo, i64 r_hi, hipStream_t s);
void launch_fill_ghost_rows(u64* buf, const Layout& L, hipStream_t s);

struct InitParams {
    i64 row0;     // global row of tile row 0
    i64 gword0;   // global word index of tile word 0
    i64 gwords;   // words per global row
    u64 seed;
    int fill;     // 0 zero, 1 ones, 2 random
};
void launch_init_fill(u64* buf, const Layout& L, const InitParams& ip, hipStream_t s);
// cells: device array of (row, col) tile coordinates
void launch_set_cells(u64* buf, const Layout& L, const i64* cells, i64 n, hipStream_t s);

struct CopyDesc {
    const u64* src;
    u64* dst;
    i64 src_stride;  // words between rows
    i64 dst_stride;
    i32 rows;
    i32 words;
};
void launch_copy_regions(const CopyDesc* descs, int n, i64 max_elems, hipStream_t s);

// out[0] += population, out[1] += fingerprint (wrapping sums); out must be zeroed by the caller.
void launch_reduce_board(const u64* buf, const Layout& L, i64 grow0, i64 gword0, i64 gwords, u64* out,
                         hipStream_t s);

// Yardstick: one byte per cell, one thread per cell, x-wrap + two ghost rows (reference class).
void launch_naive_byte_step(const u8* src, u8* dst, i64 w, i64 h, const u8* above, const u8* below, int threads,
                            hipStream_t s);

}  // namespace hipk
}  // namespace gol
