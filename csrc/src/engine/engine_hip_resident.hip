// gol-mi355x: HipEngine — the resident kernel (step_resident): plans, neighbour lists, launches.
#include "hip_engine.hpp"

namespace gol {
namespace hipeng {

// A plan of tiles (one workgroup each, all co-resident) for in-kernel halo exchanges every `kin`
// generations.  Tile heights: one round of tiles per CU when a tile's extended rows (nrows + 2 kin)
// fit 16 waves x 8 rows (the band height whose registers do not spill, 89 VGPRs), else two rounds of
// shorter tiles per CU at 16 x 4 rows (43 VGPRs, 8 waves per SIMD); tiles = 0 when neither fits.
const HipEngine::ResPlan& HipEngine::res_plan(int kin) {
    auto it = res_plans_.find(kin);
    if (it != res_plans_.end()) return it->second;
    ResPlan rp;
    rp.kin = kin;
    const std::vector<Region> rg = {{0, L_.h, 0, L_.nw}};
    const bool wrapy = true;  // resident_eligible(): the rank is its own N/S neighbour
    for (int per_cu : {1, 2}) {
        const int bmax = per_cu == 1 ? 8 : 4;
        const i64 rows = balanced_rows_per_chunk(rg, L_.nw, L_.h, kin, (i64)per_cu * cus_, 1, true);
        if (rows + 2 * (i64)kin > 16 * (i64)bmax) continue;
        const int B = hipk::resident_band_rows((int)ceil_div(rows + 2 * (i64)kin, 16));
        if (B <= 0 || B > bmax) continue;
        if (hipk::resident_blocks_per_cu(16, B, wrapy) < per_cu) continue;
        std::vector<LaneDesc> lanes = build_plan(rg, L_.nw, L_.h, rows, kin, true, nullptr, 1, cfg_.plan_xcds);
        const i64 tiles = (i64)lanes.size() / kWaveLanes;
        if (tiles > (i64)per_cu * cus_) continue;  // all tiles must be co-resident
        i64 tallest = 0;
        for (size_t w = 0; w < (size_t)tiles; ++w) tallest = std::max<i64>(tallest, lanes[w * kWaveLanes].nrows);
        if (tallest + 2 * (i64)kin > 16 * (i64)B) continue;
        std::string bad = validate_plan(lanes, L_.nw, L_.h, L_.R, kin, true);
        std::vector<u32> off, idx;
        if (bad.empty()) bad = resident_neighbours(lanes, L_.nw, L_.h, kin, true, off, idx);
        if (!bad.empty()) throw Error(strprintf("refusing to launch an unsafe resident plan (depth %d): %s", kin, bad.c_str()));
        if (idx.empty()) idx.push_back(0);  // (a valid allocation; off[] bounds every read)
        HIP_CHECK(hipMalloc(&rp.d, lanes.size() * sizeof(LaneDesc)));
        upload(rp.d, lanes.data(), lanes.size() * sizeof(LaneDesc));
        HIP_CHECK(hipMalloc(&rp.nbr_off, off.size() * sizeof(u32)));
        upload(rp.nbr_off, off.data(), off.size() * sizeof(u32));
        HIP_CHECK(hipMalloc(&rp.nbr, idx.size() * sizeof(u32)));
        upload(rp.nbr, idx.data(), idx.size() * sizeof(u32));
        HIP_CHECK(hipMalloc(&rp.counters, (size_t)tiles * sizeof(u32)));
        HIP_CHECK(hipMemsetAsync(rp.counters, 0, (size_t)tiles * sizeof(u32), s_comp_));
        if (!res_status_) {
            HIP_CHECK(hipMalloc(&res_status_, sizeof(u32)));
            HIP_CHECK(hipMemsetAsync(res_status_, 0, sizeof(u32), s_comp_));
        }
        HIP_CHECK(hipStreamSynchronize(s_comp_));
        rp.tiles = tiles;
        rp.B = B;
        rp.rows = rows;
        break;
    }
    return res_plans_.emplace(kin, rp).first->second;
}

void HipEngine::res_launch(int G, u64* src, u64* dst, hipStream_t s) {
    const ResPlan& rp = res_plan(res_kin_);
    if (rp.tiles == 0) throw Error(strprintf("the resident kernel does not fit this board at depth %d", res_kin_));
    int S = (G + rp.kin - 1) / rp.kin;
    S += (S % 2 == 0);  // odd: the result lands in dst
    hipk::ResidentParams p{};
    p.pitch = L_.pitch;
    p.h = (i32)L_.h;
    p.R = L_.R;
    p.G = G;
    p.S = S;
    p.kmax = (G + S - 1) / S;
    // 2 s of s_memrealtime (100 MHz): a neighbour wait never takes that long (GOL_RESIDENT_TIMEOUT_TICKS:
    // test knob, e.g. 0 makes the first unsatisfied wait time out)
    p.timeout_ticks = (u64)env_int("GOL_RESIDENT_TIMEOUT_TICKS", 200000000ll);
    hipk::launch_step_resident(rp.nw, rp.B, true, src, dst, rp.d, rp.tiles, rp.nbr_off, rp.nbr, rp.counters,
                               res_status_, p, s);
}

void HipEngine::check_res_status() {
    // every launch enqueued so far must be done before its fault words are read (pipe_fault reads its
    // flag with a null-stream copy, which the engine's non-blocking streams do not order)
    if (pipe_used_ || res_status_) synchronize();
    if (pipe_used_ && hipk::pipe_fault())
        throw Error("step_pipe: a ring wait timed out (a stage never got its rows); the board is invalid");
    if (!res_status_) return;
    u32 v = 0;
    HIP_CHECK(hipMemcpyAsync(&v, res_status_, sizeof(u32), hipMemcpyDeviceToHost, s_comp_));
    HIP_CHECK(hipStreamSynchronize(s_comp_));
    if (v != 0)
        throw Error("step_resident: a tile timed out waiting for its neighbours (tiles not co-resident?); the board "
                    "is invalid");
}

float HipEngine::time_resident(int kin, int G) {
    const ResPlan& rp = res_plan(kin);
    if (rp.tiles == 0) return 1e30f;
    if (!res_scratch_[0])
        for (auto& b : res_scratch_) HIP_CHECK(hipMalloc(&b, alloc_bytes_));
    const int saved = res_kin_;
    res_kin_ = kin;
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipMemcpyAsync(res_scratch_[0], buf_[cur_], alloc_bytes_, hipMemcpyDeviceToDevice, s_comp_));
    res_launch(G, res_scratch_[0], res_scratch_[1], s_comp_);  // warm-up
    HIP_CHECK(hipEventRecord(e0, s_comp_));
    for (int i = 0; i < 3; ++i) res_launch(G, res_scratch_[i & 1], res_scratch_[(i & 1) ^ 1], s_comp_);
    HIP_CHECK(hipEventRecord(e1, s_comp_));
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    res_kin_ = saved;
    // A candidate whose launches timed out (a tile gave up waiting for its neighbours: not co-resident
    // on this box, or the test knob above) is dropped, as a step_pipe candidate whose ring wait timed
    // out is: read and clear the status, and re-zero this plan's counters (the tiles that gave up left
    // theirs behind the others', so later launches would wait for supersteps that never come).  Only a
    // forced GOL_KERNEL=resident makes it fatal.
    u32 v = 0;
    HIP_CHECK(hipMemcpyAsync(&v, res_status_, sizeof(u32), hipMemcpyDeviceToHost, s_comp_));
    HIP_CHECK(hipStreamSynchronize(s_comp_));
    if (v != 0) {
        HIP_CHECK(hipMemsetAsync(res_status_, 0, sizeof(u32), s_comp_));
        HIP_CHECK(hipMemsetAsync(rp.counters, 0, (size_t)rp.tiles * sizeof(u32), s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
        if (cfg_.kernel == "resident")
            throw Error(strprintf("GOL_KERNEL=resident: a tile timed out waiting for its neighbours (depth %d)", kin));
        fprintf(stderr, "[gol] step_resident@%d: a neighbour wait timed out in the timing; candidate dropped\n", kin);
        return 1e30f;
    }
    return ms / 3 / (float)G;
}

}  // namespace hipeng
}  // namespace gol
