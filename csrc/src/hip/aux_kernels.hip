// gol-mi355x: auxiliary gfx950 kernels — init, ghost refresh, halo pack/unpack, reductions and the
// byte-per-cell yardstick.  None of these is on the per-generation hot path of a single-GPU run.
//
// Reference counterparts: pattern init runs host loops over managed memory (gol-with-cuda.cu:85-88,
// 111-114, 134-141, 161-166) and ghost rows are copied on the host once (gol-with-cuda.cu:40-47);
// here everything stays in HBM and is done by small device kernels.
#include "gol/bits.hpp"
#include "gol/hip_kernels.hpp"

namespace gol {
namespace hipk {

namespace {

__global__ void k_init_fill(u64* __restrict__ buf, i64 pitch, int R, i64 h, i64 nw, i64 w, InitParams ip) {
    const i64 n = h * nw;
    for (i64 e = (i64)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (i64)gridDim.x * blockDim.x) {
        const i64 r = e / nw, c = e - r * nw;
        u64 v = 0;
        if (ip.fill == 1)
            v = ~0ull;
        else if (ip.fill == 2)
            v = random_word(ip.seed, ip.row0 + r, ip.gword0 + c, ip.gwords);
        buf[(r + R) * pitch + c + 1] = split_word(v & word_mask(c, w));  // split storage (bits.hpp)
    }
}

__global__ void k_set_cells(u64* __restrict__ buf, i64 pitch, int R, const i64* __restrict__ cells, i64 n) {
    const i64 e = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const i64 r = cells[2 * e], c = cells[2 * e + 1];
    atomicOr((unsigned long long*)&buf[(r + R) * pitch + (c >> 6) + 1], 1ull << storage_bit(c));
}

__global__ void k_fill_ghost_cols(u64* __restrict__ buf, i64 pitch, int R, i64 w, i64 nw, i64 r_lo, i64 r_hi) {
    const i64 r = r_lo + (i64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= r_hi) return;
    wrap_row_ghosts(buf + (r + R) * pitch + 1, w, nw);
}

__global__ void k_fill_ghost_rows(u64* __restrict__ buf, i64 pitch, int R, i64 h) {
    // ghost row g in [-R,0) U [h,h+R) <- row g mod h (full pitch, including ghost words)
    const i64 n = 2 * (i64)R * pitch;
    for (i64 e = (i64)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (i64)gridDim.x * blockDim.x) {
        const i64 j = e / pitch, c = e - j * pitch;
        const i64 g = j < R ? -R + j : h + (j - R);
        i64 srow = g % h;
        if (srow < 0) srow += h;
        buf[(g + R) * pitch + c] = buf[(srow + R) * pitch + c];
    }
}

__global__ void k_copy_regions(const CopyDesc* __restrict__ descs) {
    const CopyDesc d = descs[blockIdx.y];
    const i64 n = (i64)d.rows * d.words;
    for (i64 e = (i64)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (i64)gridDim.x * blockDim.x) {
        const i64 r = e / d.words, c = e - r * d.words;
        d.dst[r * d.dst_stride + c] = d.src[r * d.src_stride + c];
    }
}

// Block-level reduction of (population, fingerprint); one atomic pair per block.
__global__ __launch_bounds__(256) void k_reduce_board(const u64* __restrict__ buf, i64 pitch, int R, i64 h, i64 nw,
                                                      i64 w, i64 grow0, i64 gword0, i64 gwords,
                                                      unsigned long long* __restrict__ out) {
    u64 pop = 0, fp = 0;
    const i64 n = h * nw;
    for (i64 e = (i64)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (i64)gridDim.x * blockDim.x) {
        const i64 r = e / nw, c = e - r * nw;
        const u64 v = merge_word(buf[(r + R) * pitch + c + 1]) & word_mask(c, w);  // natural order
        pop += (u64)__popcll(v);
        fp += fingerprint_word((u64)(grow0 + r) * (u64)gwords + (u64)(gword0 + c), v);
    }
    // wave reduction (64 lanes) then across the 4 waves through LDS
    for (int off = 32; off > 0; off >>= 1) {
        pop += __shfl_down(pop, off, 64);
        fp += __shfl_down(fp, off, 64);
    }
    __shared__ u64 sp[4], sf[4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sp[wv] = pop;
        sf[wv] = fp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 a = 0, b = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
            a += sp[i];
            b += sf[i];
        }
        atomicAdd(&out[0], (unsigned long long)a);
        atomicAdd(&out[1], (unsigned long long)b);
    }
}

// Reference-class yardstick: one thread per byte-cell, grid-stride, global loads only.
__global__ void k_naive_byte_step(const u8* __restrict__ src, u8* __restrict__ dst, i64 w, i64 h,
                                  const u8* __restrict__ above, const u8* __restrict__ below) {
    const i64 n = w * h;
    for (i64 e = (i64)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (i64)gridDim.x * blockDim.x) {
        const i64 y = e / w, x = e - y * w;
        const i64 x0 = x == 0 ? w - 1 : x - 1, x2 = x == w - 1 ? 0 : x + 1;
        const u8* up = y == 0 ? above : src + (y - 1) * w;
        const u8* mid = src + y * w;
        const u8* dn = y == h - 1 ? below : src + (y + 1) * w;
        const int nb = up[x0] + up[x] + up[x2] + mid[x0] + mid[x2] + dn[x0] + dn[x] + dn[x2];
        dst[e] = (u8)(nb == 3 || (mid[x] && nb == 2));
    }
}

unsigned grid_for(i64 n, int block = 256, i64 cap = 256 * 16) {
    i64 g = ceil_div(n, block);
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

}  // namespace

void launch_init_fill(u64* buf, const Layout& L, const InitParams& ip, hipStream_t s) {
    hipLaunchKernelGGL(k_init_fill, dim3(grid_for(L.h * L.nw)), dim3(256), 0, s, buf, L.pitch, L.R, L.h, L.nw, L.w,
                       ip);
}

void launch_set_cells(u64* buf, const Layout& L, const i64* cells, i64 n, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_set_cells, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, buf, L.pitch, L.R, cells, n);
}

void launch_fill_ghost_cols(u64* buf, const Layout& L, i64 r_lo, i64 r_hi, hipStream_t s) {
    if (r_hi <= r_lo) return;
    hipLaunchKernelGGL(k_fill_ghost_cols, dim3((unsigned)ceil_div(r_hi - r_lo, 256)), dim3(256), 0, s, buf, L.pitch,
                       L.R, L.w, L.nw, r_lo, r_hi);
}

void launch_fill_ghost_rows(u64* buf, const Layout& L, hipStream_t s) {
    hipLaunchKernelGGL(k_fill_ghost_rows, dim3(grid_for(2 * (i64)L.R * L.pitch)), dim3(256), 0, s, buf, L.pitch, L.R,
                       L.h);
}

void launch_copy_regions(const CopyDesc* descs, int n, i64 max_elems, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_copy_regions, dim3(grid_for(max_elems, 256, 1024), (unsigned)n), dim3(256), 0, s, descs);
}

void launch_reduce_board(const u64* buf, const Layout& L, i64 grow0, i64 gword0, i64 gwords, u64* out,
                         hipStream_t s) {
    hipLaunchKernelGGL(k_reduce_board, dim3(grid_for(L.h * L.nw, 256, 2048)), dim3(256), 0, s, buf, L.pitch, L.R, L.h,
                       L.nw, L.w, grow0, gword0, gwords, (unsigned long long*)out);
}

void launch_naive_byte_step(const u8* src, u8* dst, i64 w, i64 h, const u8* above, const u8* below, int threads,
                            hipStream_t s) {
    if (threads < 64 || threads > 1024) threads = 256;
    hipLaunchKernelGGL(k_naive_byte_step, dim3(grid_for(w * h, threads, 256 * 64)), dim3(threads), 0, s, src, dst, w,
                       h, above, below);
}

}  // namespace hipk
}  // namespace gol
