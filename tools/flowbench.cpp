// Standalone harness for step_flow (csrc/src/hip/flow_kernel.hip): one square periodic tile, a
// superstep of G generations cut into the given passes, run as ONE dependency-driven launch, checked
// word by word against the same passes run as separate step_temporal launches, then timed:
//   build/flowbench [N=32768] [cut=8,8,4] [reps=20] [items_per_round=1.0] [blocks_per_cu=0 (auto)]
// KB_XFLOW=0 skips the flow launches (times the pass launches only).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gol/hip_kernels.hpp"
#include "gol/plan.hpp"

using namespace gol;

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

template <typename T>
T* upload(const std::vector<T>& v) {
    T* d = nullptr;
    CK(hipMalloc(&d, std::max<size_t>(1, v.size()) * sizeof(T)));
    if (!v.empty()) CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const i64 N = argc > 1 ? atoll(argv[1]) : 32768;
    std::vector<int> cut;
    {
        std::string s = argc > 2 ? argv[2] : "8,8,4";
        for (size_t p = 0; p < s.size();) {
            size_t q = s.find(',', p);
            if (q == std::string::npos) q = s.size();
            cut.push_back(atoi(s.substr(p, q - p).c_str()));
            p = q + 1;
        }
    }
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    const double per_round = argc > 4 ? atof(argv[4]) : 1.0;
    int bpc = argc > 5 ? atoi(argv[5]) : 0;
    int G = 0;
    for (int k : cut) G += k;
    Layout L(N, N, 8);
    const size_t bytes = (size_t)(L.words() + hipk::kSlackRows * L.pitch) * 8;
    u64 *a, *b, *c, *d;
    for (u64** p : {&a, &b, &c, &d}) {
        CK(hipMalloc(p, bytes));
        CK(hipMemset(*p, 0, bytes));
    }
    hipk::InitParams ip{0, 0, L.nw, 0x5EED, 2};
    hipk::launch_init_fill(a, L, ip, 0);
    CK(hipMemcpy(c, a, bytes, hipMemcpyDeviceToDevice));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipk::ensure_trash();
    const u32 flags = hipk::STEP_WRAP_Y;
    hipk::StepParams sp{L.pitch, (i32)L.h, (i32)L.nw, L.R, flags};
    std::vector<Region> rg = {{0, N, 0, L.nw}};

    // the passes as separate step_temporal launches (their own one-round plans): reference + timing
    std::vector<LaneDesc*> pplan;
    std::vector<i64> pwaves;
    for (int k : cut) {
        const i64 res = (i64)hipk::step_blocks_per_cu(k, flags) * kWavesPerBlock * cus;
        const i64 rows = balanced_rows_per_chunk(rg, L.nw, N, k, res, 2 * k, true);
        PlanStats st;
        std::vector<LaneDesc> ln = build_plan(rg, L.nw, N, rows, k, true, &st, kWavesPerBlock, 8);
        pplan.push_back(upload(ln));
        pwaves.push_back(st.waves);
    }
    auto run_passes = [&](u64*& x, u64*& y) {
        for (size_t j = 0; j < cut.size(); ++j) {
            hipk::launch_step(cut[j], x, y, pplan[j], pwaves[j], sp, 0);
            std::swap(x, y);
        }
    };

    // the flow plan
    if (bpc <= 0) bpc = hipk::flow_blocks_per_cu(flags);
    const i64 resident = (i64)bpc * kWavesPerBlock * cus;
    std::vector<FlowPass> fps;
    // KB_LAST_PR: items per round of the LAST pass (finer items there shorten the superstep's drain)
    const double last_pr = getenv("KB_LAST_PR") ? atof(getenv("KB_LAST_PR")) : per_round;
    for (size_t j = 0; j < cut.size(); ++j) {
        const int k = cut[j];
        const double pr = j + 1 == cut.size() ? last_pr : per_round;
        const i64 target = std::max<i64>(1, (i64)(pr * (double)resident));
        fps.push_back({k, rg, balanced_rows_per_chunk(rg, L.nw, N, k, target, 2 * k, true)});
    }
    FlowPlan fp;
    const auto hb0 = std::chrono::steady_clock::now();
    const std::string err = build_flow_plan(fps, L.nw, N, true, true, fp);
    const double build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - hb0).count();
    if (!err.empty()) {
        fprintf(stderr, "flow plan: %s\n", err.c_str());
        return 1;
    }
    for (size_t j = 0; j < cut.size(); ++j) {
        std::vector<LaneDesc> part(fp.lanes.begin() + (size_t)fp.pass_begin[j] * kWaveLanes,
                                   fp.lanes.begin() + (size_t)fp.pass_begin[j + 1] * kWaveLanes);
        const std::string bad = validate_plan(part, L.nw, N, L.R, cut[j], true);
        if (!bad.empty()) {
            fprintf(stderr, "unsafe flow pass %zu: %s\n", j, bad.c_str());
            return 1;
        }
    }
    hipk::FlowArgs fa{};
    fa.lanes = upload(fp.lanes);
    fa.items = upload(fp.items);
    fa.deps = upload(fp.deps);
    fa.flags = upload(std::vector<u32>(fp.items.size(), 0u));
    fa.ctl = upload(std::vector<hipk::FlowCtl>(1, hipk::FlowCtl{}));
    fa.n_items = (u32)fp.items.size();
    // ticket sequences: KB_FLOW_SEQS (default: the device's XCDs)
    int xccs = 1;
    CK(hipDeviceGetAttribute(&xccs, hipDeviceAttributeNumberOfXccs, 0));
    fa.nseq = (u32)std::max(1, std::min(getenv("KB_FLOW_SEQS") ? atoi(getenv("KB_FLOW_SEQS")) : xccs, hipk::kFlowSeqs));
    fa.variant = getenv("KB_FLOW_PF") ? (u32)atoi(getenv("KB_FLOW_PF")) : 0u;  // 1: ticket prefetch
    double avg_deps = fp.items.empty() ? 0 : (double)fp.deps.size() / (double)fp.items.size();
    printf("flow plan: %zu items, %u..%zu deps (max %u, avg %.1f), rows/pass:", fp.items.size(), 0u, fp.deps.size(),
           fp.max_deps, avg_deps);
    for (const FlowPass& p : fps) printf(" %lld", (long long)p.rows);
    printf(", grid %d blocks/CU (%lld waves), %u ticket sequences, host build %.1f ms\n", bpc, (long long)resident,
           fa.nseq, build_ms);
    auto run_flow = [&](u64*& x, u64*& y) {
        fa.a = x;
        fa.b = y;
        ++fa.epoch;
        hipk::launch_step_flow(fa, (i64)bpc * cus, sp, 0);
        if (cut.size() & 1) std::swap(x, y);
    };
    const bool xflow = !getenv("KB_XFLOW") || atoi(getenv("KB_XFLOW"));

    // correctness: one superstep each way from the same board, then 3 more
    int bad_words = 0;
    if (xflow) {
        for (int round = 0; round < 4; ++round) {
            run_passes(c, d);
            CK(hipDeviceSynchronize());
            fprintf(stderr, "[flowbench] round %d: passes done, launching flow\n", round);
            run_flow(a, b);
            // bounded wait (a hang is reported with the control block, read from the host-visible copy)
            const auto tw = std::chrono::steady_clock::now();
            while (hipStreamQuery(0) == hipErrorNotReady) {
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count() > 20) {
                    fprintf(stderr, "[flowbench] flow launch still running after 20 s\n");
                    return 4;
                }
            }
            CK(hipDeviceSynchronize());
            fprintf(stderr, "[flowbench] round %d: flow done\n", round);
            if (hipk::flow_fault(fa.ctl, 0)) {
                fprintf(stderr, "flow: a dependency wait timed out\n");
                return 3;
            }
            std::vector<u64> x((size_t)L.words()), y((size_t)L.words());
            CK(hipMemcpy(x.data(), a, x.size() * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(y.data(), c, y.size() * 8, hipMemcpyDeviceToHost));
            for (i64 r = 0; r < N; ++r)
                for (i64 w = 0; w < L.nw; ++w) {
                    const size_t o = (size_t)((r + L.R) * L.pitch + w + 1);
                    if (x[o] != y[o]) ++bad_words;
                }
            printf("check superstep %d: %d words differ\n", round, bad_words);
            if (bad_words) return 2;
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_it = [&](auto&& fn, const char* what) {
        for (int w = 0; w < 3; ++w) fn(a, b);
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) fn(a, b);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        // single supersteps from an idle GPU, host wall (the driver's 20-generation case)
        std::vector<double> one;
        for (int r = 0; r < 15; ++r) {
            CK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            fn(a, b);
            CK(hipDeviceSynchronize());
            one.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(one.begin(), one.end());
        printf("%-8s G=%d: back-to-back %.3f us/gen; one superstep from idle (host wall) min %.1f med %.1f us = %.3f us/gen\n",
               what, G, best * 1e3 / (reps * G), one[0], one[one.size() / 2], one[one.size() / 2] / G);
    };
    time_it(run_passes, "passes");
    if (xflow) time_it(run_flow, "flow");
    if (xflow && hipk::flow_fault(fa.ctl, 0)) {
        fprintf(stderr, "flow: a dependency wait timed out during timing\n");
        return 3;
    }
    return 0;
}
