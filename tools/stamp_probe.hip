// stamp_probe: when do the waves of one step_temporal pass start and finish?  (The drain at the end of
// a pass — waves of one SIMD finishing at different times — is what a superstep of several passes
// loses at every pass boundary.)  One K = 8 pass over an N^2 periodic tile with the engine's one-round
// plan, run through the production wave code (wave_runner.hpp), each wave stamping s_memrealtime at
// its start and end with its hardware slot (HW_ID: SE, CU, SIMD, wave; XCC_ID).  Prints the finish
// times by the wave's age rank on its SIMD (0 = dispatched first) and by dispatch third of the grid.
//   build/stamp_probe [N=32768] [weights=1: build_plan age_weights, one per dispatch class of the grid]
//                     [reps=3] [blocks_per_cu=0: the occupancy limit]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "gol/hip_kernels.hpp"
#include "gol/plan.hpp"
#include "../csrc/src/hip/stencil_device.hpp"
#include "../csrc/src/hip/wave_runner.hpp"

using namespace gol;
using namespace gol::hipk;

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ __launch_bounds__(64 * kWavesPerBlock) void stamped(const u64* __restrict__ src, u64* __restrict__ dst,
                                                               const LaneDesc* __restrict__ plan, StepParams p,
                                                               u64* stamps) {
    const int wv = threadIdx.x >> 6;
    const i64 wave = (i64)blockIdx.x * kWavesPerBlock + wv;
    const int lane = threadIdx.x & 63;
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    const LaneDesc d = plan[wave * kWaveLanes + lane];
    const int nrows = __builtin_amdgcn_readfirstlane(d.nrows);
    if (nrows > 0) {
        WaveRunner<8, ROWS_WRAP> w(src, dst, d, nrows, p, wave);
        w.run();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u64 t1 = __builtin_amdgcn_s_memrealtime();
    u32 hw = 0, xcc = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    if (lane < 4) {
        const u64 v = lane == 0 ? t0 : lane == 1 ? t1 : lane == 2 ? (u64)hw : (u64)xcc;
        stamps[wave * 4 + lane] = v;
    }
}

int main(int argc, char** argv) {
    const i64 N = argc > 1 ? atoll(argv[1]) : 32768;
    std::vector<double> hts;
    {
        const std::string s = argc > 2 ? argv[2] : "1";
        for (size_t q = 0; q < s.size();) {
            size_t e = s.find(',', q);
            if (e == std::string::npos) e = s.size();
            hts.push_back(atof(s.substr(q, e - q).c_str()));
            q = e + 1;
        }
    }
    Layout L(N, N, 8);
    const size_t bytes = (size_t)(L.words() + kSlackRows * L.pitch) * 8;
    u64 *a, *b, *trash, *stamps;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&trash, (size_t)kTrashWaves * 64 * 8));
    CK(hipMemset(a, 0x5A, bytes));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, stamped, 64 * kWavesPerBlock, 0));
    if (argc > 4 && atoi(argv[4]) > 0) bpc = std::min(bpc, atoi(argv[4]));
    const i64 resident = (i64)bpc * prop.multiProcessorCount * kWavesPerBlock;
    std::vector<Region> rg = {{0, N, 0, L.nw}};
    const i64 rows = balanced_rows_per_chunk(rg, L.nw, N, 8, resident, 16, true);
    PlanStats st;
    const bool weighted = hts.size() > 1;
    std::string wtxt;
    for (double x : hts) wtxt += (wtxt.empty() ? "" : ",") + std::to_string(x).substr(0, 4);
    std::vector<LaneDesc> lanes = build_plan(rg, L.nw, N, rows, 8, true, &st, kWavesPerBlock, 8, false, weighted ? &hts : nullptr);
    const i64 waves = (i64)lanes.size() / kWaveLanes;
    printf("stamp_probe: %lld^2, K 8, %d blocks/CU, plan %lld waves of %lld rows (resident %lld), weights %s\n",
           (long long)N, bpc, (long long)waves, (long long)rows, (long long)resident, wtxt.c_str());
    if (waves > resident) printf("  (more waves than resident slots: not one round)\n");
    LaneDesc* dplan = nullptr;
    CK(hipMalloc(&dplan, lanes.size() * sizeof(LaneDesc)));
    CK(hipMemcpy(dplan, lanes.data(), lanes.size() * sizeof(LaneDesc), hipMemcpyHostToDevice));
    CK(hipMalloc(&stamps, (size_t)waves * 4 * 8));
    StepParams p{L.pitch, (i32)L.h, (i32)L.nw, L.R, STEP_WRAP_Y};
    p.trash = trash;
    const int blocks = (int)(waves / kWavesPerBlock);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(stamped, dim3(blocks), dim3(64 * kWavesPerBlock), 0, 0, a, b, dplan, p, stamps);
    CK(hipDeviceSynchronize());
    const int nrep = argc > 3 ? atoi(argv[3]) : 3;
    std::vector<double> spans;
    for (int rep = 0; rep < nrep; ++rep) {
        hipLaunchKernelGGL(stamped, dim3(blocks), dim3(64 * kWavesPerBlock), 0, 0, a, b, dplan, p, stamps);
        CK(hipDeviceSynchronize());
        std::vector<u64> s((size_t)waves * 4);
        CK(hipMemcpy(s.data(), stamps, s.size() * 8, hipMemcpyDeviceToHost));
        u64 t_min = ~0ull, t_max = 0;
        for (i64 w = 0; w < waves; ++w) {
            t_min = std::min(t_min, s[w * 4]);
            t_max = std::max(t_max, s[w * 4 + 1]);
        }
        // age rank of each wave on its SIMD: order of start stamps among the waves of one (xcc, se, cu, simd)
        std::map<std::tuple<u32, u32, u32, u32>, std::vector<std::pair<u64, i64>>> simd;
        double busy = 0;
        for (i64 w = 0; w < waves; ++w) {
            const u32 hw = (u32)s[w * 4 + 2], xcc = (u32)s[w * 4 + 3];
            const u32 simd_id = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            simd[std::make_tuple(xcc, se, cu * 2 + sh, simd_id)].push_back({s[w * 4], w});
            busy += (double)(s[w * 4 + 1] - s[w * 4]);
        }
        std::vector<int> rank((size_t)waves, 0);
        size_t max_per_simd = 0;
        for (auto& kv : simd) {
            std::sort(kv.second.begin(), kv.second.end());
            for (size_t i = 0; i < kv.second.size(); ++i) rank[(size_t)kv.second[i].second] = (int)i;
            max_per_simd = std::max(max_per_simd, kv.second.size());
        }
        const double span = (double)(t_max - t_min) * 1e-2;  // us (100 MHz)
        spans.push_back(span);
        printf("rep %d: pass %.1f us, %zu SIMDs (<= %zu waves each), slot busy %.0f%%\n", rep, span, simd.size(),
               max_per_simd, 100.0 * busy * 1e-2 / (span * (double)waves));
        auto stats = [&](const char* what, auto&& key, int nkeys) {
            for (int k = 0; k < nkeys; ++k) {
                std::vector<double> st_, en;
                for (i64 w = 0; w < waves; ++w)
                    if (key(w) == k) {
                        st_.push_back((double)(s[w * 4] - t_min) * 1e-2);
                        en.push_back((double)(s[w * 4 + 1] - t_min) * 1e-2);
                    }
                if (en.empty()) continue;
                std::sort(st_.begin(), st_.end());
                std::sort(en.begin(), en.end());
                auto q = [](const std::vector<double>& v, double f) { return v[(size_t)(f * (double)(v.size() - 1))]; };
                printf("  %s %d: %5zu waves  start p50 %6.1f max %6.1f | end min %6.1f p10 %6.1f p50 %6.1f p90 %6.1f max %6.1f us\n",
                       what, k, en.size(), q(st_, 0.5), st_.back(), en[0], q(en, 0.1), q(en, 0.5), q(en, 0.9), en.back());
            }
        };
        stats("age rank", [&](i64 w) { return rank[(size_t)w]; }, (int)max_per_simd);
        stats("dispatch class", [&](i64 w) { return (int)(bpc * (w / kWavesPerBlock) / blocks); }, bpc);
        // segment heights by dispatch class
        for (int c = 0; c < bpc; ++c) {
            double sr = 0;
            i64 n = 0;
            for (i64 w = 0; w < waves; ++w)
                if ((int)(bpc * (w / kWavesPerBlock) / blocks) == c && lanes[(size_t)w * kWaveLanes].nrows > 0) {
                    sr += lanes[(size_t)w * kWaveLanes].nrows;
                    ++n;
                }
            printf("  dispatch class %d: mean segment %.1f rows\n", c, n ? sr / (double)n : 0.0);
        }
    }
    // back-to-back passes (event timed): the rate a superstep of such passes runs at
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 20; ++i)
            hipLaunchKernelGGL(stamped, dim3(blocks), dim3(64 * kWavesPerBlock), 0, 0, (i & 1) ? b : a, (i & 1) ? a : b, dplan, p, stamps);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
    }
    std::sort(spans.begin(), spans.end());
    printf("bpc %d weights %s: stamped pass span median %.1f us; 20 back-to-back passes %.1f us/pass = %.3f us/gen\n",
           bpc, wtxt.c_str(), spans.empty() ? 0.0 : spans[spans.size() / 2], best * 1e3 / 20, best * 1e3 / 160);
    return 0;
}
