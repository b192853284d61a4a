// Standalone timing harness for the temporal stencil kernel (single tile, periodic, balanced plan).
// Used to A/B compiler flags / code variants of step_kernels.hip without rebuilding the framework:
//   hipcc --offload-arch=gfx950 -O3 -Icsrc/include [variant flags] tools/kbench.cpp \
//         csrc/src/hip/step_kernels.hip csrc/src/hip/aux_kernels.hip csrc/src/core/plan.cpp \
//         csrc/src/core/geometry.cpp csrc/src/core/config.cpp -o build/kbench_<variant>
//   build/kbench_<variant> [N=32768] [K=8] [gens=960] [pf=0|1] [skew] [tile_nw] [rows] [tile_lv]
//   (KB_PIPE=L with tile_nw = NW: step_pipe, K = (NW - 1) L)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gol/hip_kernels.hpp"
#include "gol/plan.hpp"

using namespace gol;

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
            exit(1);                                                            \
        }                                                                       \
    } while (0)


int main(int argc, char** argv) {
    const i64 N = argc > 1 ? atoll(argv[1]) : 32768;
    const int K = argc > 2 ? atoi(argv[2]) : 8;
    const int gens = argc > 3 ? atoi(argv[3]) : 960;
    const int pf = argc > 4 ? atoi(argv[4]) : 0;
    const int skew = argc > 5 ? atoi(argv[5]) : 0;
    const int tile_nw = argc > 6 ? atoi(argv[6]) : 0;  // >0: step_tile with this many waves per workgroup
    const i64 rows_arg = argc > 7 ? atoll(argv[7]) : 0;
    const i64 W = getenv("KB_W") ? atoll(getenv("KB_W")) : N;  // board columns (default square)
    Layout L(N, W, K);
    const size_t bytes = (size_t)(L.words() + hipk::kSlackRows * L.pitch) * 8;
    u64 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    hipk::InitParams ip{0, 0, L.nw, 0x5EED, 2};
    hipk::launch_init_fill(a, L, ip, 0);
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int tile_lv = argc > 8 ? atoi(argv[8]) : 1;  // tile kernel: generations per LDS pass
    const bool fold = tile_nw > 0 && getenv("KB_FOLD") && atoi(getenv("KB_FOLD"));  // folded 32-lane tiles
    // KB_PIPE=L: step_pipe with tile_nw waves (one loader + tile_nw - 1 stages of L generations; K must
    // be (tile_nw - 1) L), KB_PIPE_WG workgroups per CU in the plan (default 1)
    const int pipe_l = tile_nw > 0 && getenv("KB_PIPE") ? atoi(getenv("KB_PIPE")) : 0;
    const int pipe_wg = getenv("KB_PIPE_WG") ? atoi(getenv("KB_PIPE_WG")) : 1;
    if (pipe_l > 0 && K != (tile_nw - 1) * pipe_l) {
        fprintf(stderr, "KB_PIPE: K must be (tile_nw - 1) x L = %d\n", (tile_nw - 1) * pipe_l);
        return 1;
    }
    (void)pf;
    (void)skew;  // the LDS-ring prefetch and skewed pipeline variants were removed (measured slower)
    const u32 flags = hipk::STEP_WRAP_Y |
                      (tile_lv == 2 ? hipk::STEP_TILE_L2 : 0u) | (tile_lv == 4 ? hipk::STEP_TILE_L4 : 0u) |
                      (getenv("KB_INPLACE") && atoi(getenv("KB_INPLACE")) ? hipk::STEP_TILE_INPLACE : 0u) |
                      (fold ? hipk::STEP_TILE_FOLD : 0u);
    std::vector<Region> rg = {{0, N, 0, L.nw}};
    i64 rows = rows_arg;
    if (pipe_l > 0) {
        if (rows <= 0) rows = balanced_rows_per_chunk(rg, L.nw, N, K, (i64)pipe_wg * prop.multiProcessorCount, 1, true);
    } else if (tile_nw > 0) {
        const i64 rmax = hipk::tile_max_rows(K, tile_nw, flags);
        if (rows > rmax) rows = rmax;
        for (i64 rounds = 1; rows <= 0; ++rounds) {
            const i64 r = balanced_rows_per_chunk(rg, L.nw, N, K, rounds * prop.multiProcessorCount, fold ? hipk::kFoldMinRows : 1, true, fold);
            if (r <= rmax) rows = r;
        }
    } else if (rows <= 0) {
        i64 bpc = hipk::step_blocks_per_cu(K, flags);
        if (getenv("KB_BPC")) bpc = std::min<i64>(bpc, atoi(getenv("KB_BPC")));  // waves per SIMD of the plan
        const i64 resident = bpc * kWavesPerBlock * prop.multiProcessorCount;
        rows = balanced_rows_per_chunk(rg, L.nw, N, K, resident, 2 * K, true);
    }
    PlanStats st;
    const int xcds = getenv("KB_XCDS") ? atoi(getenv("KB_XCDS")) : 8;  // 1: plain row-major order
    std::vector<LaneDesc> lanes = build_plan(rg, L.nw, N, rows, K, true, &st, tile_nw > 0 ? 1 : kWavesPerBlock, xcds, fold);
    {
        const std::string bad = validate_plan(lanes, L.nw, N, L.R, K, true);
        if (!bad.empty()) {
            fprintf(stderr, "unsafe plan: %s\n", bad.c_str());
            return 1;
        }
    }
    LaneDesc* dplan;
    CK(hipMalloc(&dplan, lanes.size() * sizeof(LaneDesc)));
    CK(hipMemcpy(dplan, lanes.data(), lanes.size() * sizeof(LaneDesc), hipMemcpyHostToDevice));
    hipk::ensure_trash();
    hipk::StepParams sp{L.pitch, (i32)L.h, (i32)L.nw, L.R, flags};
    const int steps = gens / K;
    // KB_SPLIT2=1 (temporal only, timing experiment): the board as two half-height regions, each
    // with its own one-round plan sized for the whole GPU, launched on two streams with no
    // cross-stream ordering (like two ranks sharing the GPU between exchanges).  The board values
    // are meaningless; only the time is.
    // KB_SPLIT2=n (temporal only; 1 means 2): the board as n equal row bands, each with its own
    // one-round plan sized for the whole GPU, launched on n streams with no cross-stream ordering.
    // (with KB_PIPE: each band runs step_pipe, its plan sized for KB_PIPE_WG workgroups per CU)
    const int nsplit = ((tile_nw == 0 || pipe_l > 0) && getenv("KB_SPLIT2")) ? std::max(0, atoi(getenv("KB_SPLIT2"))) : 0;
    const bool split2 = nsplit > 0;
    const int nparts = nsplit == 1 ? 2 : nsplit;
    std::vector<LaneDesc*> dplan2(std::max(nparts, 1), nullptr);
    std::vector<i64> waves2(std::max(nparts, 1), 0);
    std::vector<hipStream_t> ss(std::max(nparts, 1), nullptr);
    if (split2) {
        for (int h = 0; h < nparts; ++h) {
            std::vector<Region> r2 = {{h * (N / nparts), h == nparts - 1 ? N : (h + 1) * (N / nparts), 0, L.nw}};
            i64 bpc = hipk::step_blocks_per_cu(K, flags);
            if (getenv("KB_BPC")) bpc = std::min<i64>(bpc, atoi(getenv("KB_BPC")));
            const i64 rr = pipe_l > 0 ? balanced_rows_per_chunk(r2, L.nw, N, K, (i64)pipe_wg * prop.multiProcessorCount, 1, true)
                                      : balanced_rows_per_chunk(r2, L.nw, N, K, bpc * kWavesPerBlock * prop.multiProcessorCount, 2 * K, true);
            PlanStats st2;
            std::vector<LaneDesc> l2 = build_plan(r2, L.nw, N, rr, K, true, &st2, pipe_l > 0 ? 1 : kWavesPerBlock, xcds);
            CK(hipMalloc(&dplan2[h], l2.size() * sizeof(LaneDesc)));
            CK(hipMemcpy(dplan2[h], l2.data(), l2.size() * sizeof(LaneDesc), hipMemcpyHostToDevice));
            waves2[h] = st2.waves;
            CK(hipStreamCreateWithFlags(&ss[h], hipStreamNonBlocking));
        }
    }
    auto launch = [&](const u64* s, u64* d) {
        if (split2) {
            for (int h = 0; h < nparts; ++h)
                if (pipe_l > 0)
                    hipk::launch_step_pipe(tile_nw, pipe_l, s, d, dplan2[h], waves2[h], sp, ss[h]);
                else
                    hipk::launch_step(K, s, d, dplan2[h], waves2[h], sp, ss[h]);
        } else if (pipe_l > 0)
            hipk::launch_step_pipe(tile_nw, pipe_l, s, d, dplan, st.waves, sp, 0);
        else if (tile_nw > 0)
            hipk::launch_step_tile(tile_nw, K, s, d, dplan, st.waves, rows, sp, 0);
        else
            hipk::launch_step(K, s, d, dplan, st.waves, sp, 0);
    };
    for (int w = 0; w < 4; ++w) {
        launch(a, b);
        std::swap(a, b);
    }
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipDeviceSynchronize());
        const auto h0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, 0));
        for (int s = 0; s < steps; ++s) {
            launch(a, b);
            std::swap(a, b);
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (split2) {  // the null-stream events do not order the non-blocking streams: host time
            CK(hipDeviceSynchronize());
            ms = (float)(std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count() * 1e3);
        }
        if (ms < best) best = ms;
    }
    CK(hipGetLastError());
#ifdef GOL_PIPE_STAMPS
    // KB_PIPE_STAMPS=1 (build with -DGOL_PIPE_STAMPS): one more step_pipe launch, then its per-wave wait stamps
    // averaged by wave role (0 = loader, 1.. = compute stages): s_memtime cycles of the role, of its input
    // waits (stages: the producer's counter; loader: its DMA vmcnt waits), of its output waits (the consumer's
    // counter / a free loader slot), and waits that found the counter short, per workgroup.
    if (pipe_l > 0 && getenv("KB_PIPE_STAMPS") && atoi(getenv("KB_PIPE_STAMPS"))) {
        CK(hipDeviceSynchronize());
        launch(a, b);
        CK(hipDeviceSynchronize());
        const std::vector<u64> v = hipk::pipe_stamps((size_t)st.waves * tile_nw);
        const size_t nwg = v.size() / 4 / tile_nw;
        printf("stamps: %zu workgroups x %d waves (cycles per wave, mean over workgroups)\n", nwg, tile_nw);
        for (int w = 0; w < tile_nw; ++w) {
            double t = 0, wi = 0, wo = 0, nn = 0;
            size_t cnt = 0;
            for (size_t g = 0; g < nwg; ++g) {
                const u64* q = &v[(g * tile_nw + w) * 4];
                if (q[0] == 0) continue;  // padding workgroup
                t += (double)q[0], wi += (double)q[1], wo += (double)q[2], nn += (double)q[3];
                ++cnt;
            }
            if (!cnt) continue;
            printf("  wave %2d %-8s total %9.0f  in-wait %9.0f (%4.1f%%)  out-wait %9.0f (%4.1f%%)  short waits %7.1f\n", w,
                   w == 0 ? "loader" : "stage", t / cnt, wi / cnt, 100.0 * wi / t, wo / cnt, 100.0 * wo / t, nn / cnt);
        }
    }
#endif
    if (pipe_l > 0 && hipk::pipe_fault()) {
        fprintf(stderr, "step_pipe: a ring wait timed out\n");
        return 3;
    }
    if (getenv("KB_CHECK") && atoi(getenv("KB_CHECK")) && tile_nw > 0) {
        // K generations from the same random board: this tile kernel vs K single-generation passes of
        // the temporal kernel (its own one-round plan); every word of the board must match
        hipk::launch_init_fill(a, L, ip, 0);
        launch(a, b);
        std::vector<u64> got((size_t)(L.words())), ref((size_t)(L.words()));
        CK(hipMemcpy(got.data(), b, got.size() * 8, hipMemcpyDeviceToHost));
        const i64 r1 = balanced_rows_per_chunk(rg, L.nw, N, 1, 4 * kWavesPerBlock * prop.multiProcessorCount, 2, true);
        PlanStats s1;
        std::vector<LaneDesc> l1 = build_plan(rg, L.nw, N, r1, 1, true, &s1, kWavesPerBlock, xcds);
        LaneDesc* dp1;
        CK(hipMalloc(&dp1, l1.size() * sizeof(LaneDesc)));
        CK(hipMemcpy(dp1, l1.data(), l1.size() * sizeof(LaneDesc), hipMemcpyHostToDevice));
        hipk::StepParams s1p{L.pitch, (i32)L.h, (i32)L.nw, L.R, hipk::STEP_WRAP_Y};
        hipk::launch_init_fill(a, L, ip, 0);
        for (int g = 0; g < K; ++g) {
            hipk::launch_step(1, a, b, dp1, s1.waves, s1p, 0);
            std::swap(a, b);
        }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), a, ref.size() * 8, hipMemcpyDeviceToHost));
        i64 bad = 0;
        for (i64 r = 0; r < N; ++r)
            for (i64 c = 0; c < L.nw; ++c) {
                const size_t o = (size_t)((r + L.R) * L.pitch + c + 1);
                if (got[o] != ref[o]) ++bad;
            }
        printf("check: %lld of %lld words differ\n", (long long)bad, (long long)(N * L.nw));
        if (bad) return 2;
    }
    const double per_gen_us = best * 1e3 / (steps * K);
    const int bpc = pipe_l > 0 ? hipk::pipe_blocks_per_cu(tile_nw, pipe_l, true) : tile_nw > 0 ? hipk::tile_blocks_per_cu(tile_nw, rows, K, flags) : hipk::step_blocks_per_cu(K, flags);
    printf("{\"N\": %lld, \"K\": %d, \"skew\": %d, \"pf\": %d, \"tile_nw\": %d, \"rows\": %lld, \"waves\": %lld, "
           "\"blocks_per_cu\": %d, \"us_per_gen\": %.3f, \"cells_per_s\": %.4e}\n",
           (long long)N, K, skew, pf, tile_nw, (long long)rows, (long long)st.waves, bpc, per_gen_us,
           (double)N * W / (per_gen_us * 1e-6));
    return 0;
}
