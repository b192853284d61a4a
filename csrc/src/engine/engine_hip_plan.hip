// gol-mi355x: HipEngine — work plans of the kernel passes, pass cuts and the interior/boundary regions of a tile.
#include "hip_engine.hpp"

namespace gol {
namespace hipeng {

// Kernel passes of a superstep of k generations.  Once the pass costs are measured
// (measure_pass_costs), the cheapest cut over the instantiated depths <= K; before that (and with
// an explicit GOL_KERNEL_DEPTH) the fewest passes of at most K with depths as equal as possible
// (20 = 7 + 7 + 6, not 8 + 8 + 4).  A pass streams the board through HBM once whatever its
// depth, so shallow passes cost nearly as much as deep ones (32768^2: ~70-80 us for any depth
// <= 6, ~90 us at 8; profiles/kb_depth_sweep.txt).
const std::vector<int>& HipEngine::pass_depths(int k) {
    const int key = k + (dual_ ? (1 << 20) : 0) + (res_ ? (1 << 21) : 0);
    auto it = passes_.find(key);
    if (it != passes_.end()) return it->second;
    if (res_) return passes_.emplace(key, std::vector<int>{k}).first->second;  // one resident launch
    // every kind may be temporal, unless only the (any-depth) tile kernel runs; sub-tiles always
    // run the temporal kernel at its own depth
    const bool any_depth = !dual_ && (cfg_.kernel == "tile" || (tuned_ && !split_ && tile_kernel(0)));
    auto ok = [&](int d) { return any_depth || hipk::step_depth_supported(d); };
    const int K = std::max(1, dual_ ? tdepth_ : kdepth_);
    std::vector<int> ps;
    if (!pass_costs().empty() && !any_depth) {
        // cheapest cut by the measured per-depth pass times (the depths include step_pipe geometries when
        // that is the tuned kernel: measure_pass_costs)
        ps = cheapest_cut(k, pass_costs());
        if (!ps.empty()) return passes_.emplace(key, ps).first->second;
    }
    if (!dual_ && kern_[0] == "pipe" && pipe_k_ > 0 && !split_) {
        // (before the pass costs are measured) whole step_pipe passes; the remainder in step_temporal
        // passes of <= tdepth_, as equal as the instantiated depths allow (greedy otherwise)
        std::vector<int> v;
        int left = k;
        for (; left >= pipe_k_; left -= pipe_k_) v.push_back(pipe_k_);
        const size_t m = v.size();
        if (left > 0) {
            const int n = (left + tdepth_ - 1) / tdepth_;
            bool okd = true;
            for (int j = 0; j < n; ++j) {
                const int d = left / n + (j < left % n ? 1 : 0);
                okd = okd && hipk::step_depth_supported(d);
                v.push_back(d);
            }
            if (!okd) {
                v.resize(m);
                while (left > 0) {
                    const int d = supported_kernel_depth(std::min(left, tdepth_));
                    v.push_back(d);
                    left -= d;
                }
            }
        }
        return passes_.emplace(key, v).first->second;
    }
    const int n = (k + K - 1) / K;
    bool balanced = true;
    for (int j = 0; j < n; ++j) {
        const int d = k / n + (j < k % n ? 1 : 0);
        if (!ok(d)) balanced = false;
        ps.push_back(d);
    }
    if (!balanced) {  // greedy over the instantiated depths
        ps.clear();
        for (int left = k; left > 0;) {
            int d = std::min(left, K);
            if (!any_depth) d = supported_kernel_depth(d);
            ps.push_back(d);
            left -= d;
        }
    }
    return passes_.emplace(key, ps).first->second;
}

// Output regions of a pass of depth k whose output rows extend e rows beyond the tile (into
// the ghost rows, 1-D multi-pass supersteps): kind 0 full, 1 interior, 2 boundary bands.
std::vector<Region> HipEngine::regions(int kind, int k, i64 rem) const {
    const i64 h = L_.h, nw = L_.nw;
    const bool two_d = this->two_d();
    // multi-pass: earlier passes also produce the ghost rows (y neighbours) and the ghost
    // words, columns -1 and nw (x neighbours), that later passes read
    const i64 e = self_y() ? 0 : rem;
    const i64 xe = (!self_x() && rem > 0) ? 1 : 0;
    if (kind == 0 || h <= 2 * (i64)k)
        return kind == 1 ? std::vector<Region>{} : std::vector<Region>{{-e, h + e, -xe, nw + xe}};
    if (kind == 1) {
        if (two_d) return nw > 2 ? std::vector<Region>{{k, h - k, 1, nw - 1}} : std::vector<Region>{};
        return {{k, h - k, 0, nw}};
    }
    std::vector<Region> r = {{-e, k, -xe, nw + xe}, {h - k, h + e, -xe, nw + xe}};
    if (two_d) {
        if (nw > 2) {
            r.push_back({k, h - k, -xe, 1});
            r.push_back({k, h - k, nw - 1, nw + xe});
        } else {
            r.push_back({k, h - k, -xe, nw + xe});
        }
    }
    return r;
}

const DevPlan& HipEngine::plan(int kind, int k, i64 e) {
    // plans depend on e only through regions(): rows beyond the tile when y has neighbours,
    // ghost words when x has neighbours (so one plan serves every e of a local rank)
    const i64 ek = self_y() ? (self_x() ? 0 : (e > 0 ? 1 : 0)) : e;
    // tile plans also depend on the workgroup size (the LDS rows a tile may hold)
    const bool pipe = pipe_pass(kind, k), tile = tile_pass(kind, k);
    const PipeGeo* pg = pipe ? pipe_geo(k) : nullptr;
    const i64 key = (((((i64)(pipe ? pg->nw * 16 + pg->wg : 0) * 8 + occ_) * 2 + (tile ? 1 : 0)) * 32 +
                      (tile ? cfg_.tile_waves : 0)) * 4 + kind) * 100000 + (i64)ek * 100 + k;
    auto it = plans_.find(key);
    if (it != plans_.end()) return it->second;
    std::vector<Region> rg = regions(kind, k, e);
    DevPlan p;
    i64 rows = cfg_.rows_per_wave;
    if (tile) {
        // step_tile: one workgroup per plan wave, one tile per CU per round; rows are capped by
        // the 160 KiB of LDS (2k halo rows + the tile, double-buffered or in place), extra rounds
        // beyond that.  The double-buffered tile is used when one round of tiles fits it (cheaper:
        // no halo copies, one barrier per LDS pass; 8192^2: 1.45 vs 1.65 us/gen), the in-place one
        // (twice the rows) when the double buffer would need more rounds (4096 x 32768: 2.36 vs
        // 2.70, 16384^2: 4.58 vs 4.69; profiles/tile_inplace_ab.txt).  GOL_TILE_INPLACE=0/1 forces.
        const i64 rdb = hipk::tile_max_rows(k, cfg_.tile_waves, step_flags() | tile_bits(false));
        const i64 rip = hipk::tile_max_rows(k, cfg_.tile_waves, step_flags() | tile_bits(true));
        const i64 r1 = balanced_rows_per_chunk(rg, L_.nw, L_.h, k, cus_, 1, xwrap_by_plan());
        bool ip = tile_inplace_ > 0 || (tile_inplace_ < 0 && r1 > rdb && rip > rdb);
        if (tile_inplace_ < 0 && rows > 0) ip = rows > rdb;
        // Folded tiles (32 lanes wide, twice as tall, step_kernels.hip step_tile_fold) when one round of
        // them fits: 8192^2 K=24 1.43-1.45 -> 1.39-1.40 us/gen, K=32 1.46 -> 1.38 (double-buffered,
        // profiles/tile_fold_ab.txt).  GOL_TILE_FOLD=0/1 forces.
        const u32 ff = step_flags() | tile_bits(false) | hipk::STEP_TILE_FOLD;
        const i64 rfm = hipk::tile_max_rows(k, cfg_.tile_waves, ff);
        const i64 r1f = balanced_rows_per_chunk(rg, L_.nw, L_.h, k, cus_, hipk::kFoldMinRows, xwrap_by_plan(), true);
        // A folded tile needs >= kFoldMinRows / 2 rows (segments of a chunk height S are >= S / 2 rows):
        // regions thinner than that (boundary bands) and tiny boards keep plain tiles.
        i64 thinnest = 1 << 30;
        for (const Region& r : rg)
            if (r.r1 > r.r0 && r.c1 > r.c0) thinnest = std::min(thinnest, r.r1 - r.r0);
        // Folded in place (one buffer + side rows, twice the rows) only when forced (GOL_TILE_FOLD=1 with a
        // plan that needs it): on the 4096 x 32768 strip it ties the in-place tile kernel (K=32, 4 levels
        // 2.40-2.44 vs 2.42-2.44 us/gen; 240 of 256 CUs busy) and loses with 2 levels per LDS pass.
        const i64 rfmi = hipk::tile_max_rows(k, cfg_.tile_waves, step_flags() | tile_bits(true) | hipk::STEP_TILE_FOLD);
        const bool fold_ip = tile_inplace_ > 0 || (tile_inplace_ < 0 && r1f > rfm);
        const i64 fcap = fold_ip ? rfmi : rfm;
        const bool fold = r1f >= hipk::kFoldMinRows && thinnest >= hipk::kFoldMinRows / 2 &&
                          (tile_fold_ > 0 || (tile_fold_ < 0 && rows <= 0 && !fold_ip && r1f <= fcap));
        if (fold) {
            if (rows <= 0) rows = std::min(r1f, fcap);
            if (rows < hipk::kFoldMinRows || rows > fcap)
                throw Error(strprintf("GOL_TILE_FOLD: %lld rows per folded tile outside %d..%lld at depth %d",
                                      (long long)rows, hipk::kFoldMinRows, (long long)fcap, k));
            p.tflags = tile_bits(fold_ip) | hipk::STEP_TILE_FOLD;
            p.fold = true;
        }
        const i64 rmax = ip ? rip : rdb;
        if (!fold) p.tflags = tile_bits(ip);
        if (rmax < 1) throw Error(strprintf("GOL_KERNEL=tile: depth %d leaves no LDS rows", k));
        if (!fold && rows > rmax) rows = rmax;
        if (tile_rounds(kind, k, e) > kMaxTileRounds)
            throw Error(strprintf("LDS tile kernel (plan kind %d, depth %d, tuned kernels %s/%s/%s): this tile needs "
                                  "%lld rounds of LDS tiles; use the temporal kernel for boards this large",
                                  kind, k, kern_[0].c_str(), kern_[1].c_str(), kern_[2].c_str(),
                                  (long long)tile_rounds(kind, k, e)));
        if (rows <= 0) {  // (a folded plan has its rows already)
            const i64 rounds = ceil_div(r1, rmax);
            rows = rounds <= 1 ? r1
                               : std::min(rmax, balanced_rows_per_chunk(rg, L_.nw, L_.h, k, rounds * cus_, 1,
                                                                        xwrap_by_plan()));
        }
    } else if (pipe) {
        // step_pipe: one workgroup per plan wave, wg of them per CU in one round
        if (rows <= 0) rows = balanced_rows_per_chunk(rg, L_.nw, L_.h, k, (i64)pg->wg * cus_, 1, xwrap_by_plan());
    } else {
        if (rows <= 0 && cfg_.waves_target > 0)
            rows = choose_rows_per_chunk(rg, k, cfg_.waves_target, 4 * (i64)k);
        if (rows <= 0) {
            // one full round of resident waves (occupancy of this kernel instantiation)
            i64 bpc = hipk::step_blocks_per_cu(k, step_flags());
            // 256-thread blocks per CU = waves per SIMD; the tuned cap applies to the tuned depth
            // only (shallower passes are memory bound and want every resident wave)
            if (occ_ > 0 && k == kdepth_) bpc = std::min<i64>(bpc, occ_);
            const i64 resident = bpc * kWavesPerBlock * cus_;
            // big tiles: several rounds of segments near round_rows() rows (plan.hpp round_balanced_rows)
            rows = round_balanced_rows(rg, L_.nw, L_.h, k, resident, 2 * (i64)k, xwrap_by_plan(), round_rows(k));
            // (Segment heights weighted by dispatch class, plan.hpp build_plan age_weights, made every
            // pass slower: the pass is VALU-bound, profiles/stamp_age_weights.txt.)
        }
    }
    std::vector<LaneDesc> lanes = build_plan(rg, L_.nw, L_.h, rows, k, xwrap_by_plan(), &p.st,
                                             (tile || pipe) ? 1 : kWavesPerBlock, cfg_.plan_xcds, p.fold);
    const std::string bad = validate_plan(lanes, L_.nw, L_.h, L_.R, k, (step_flags() & hipk::STEP_WRAP_Y) != 0);
    if (!bad.empty()) throw Error(strprintf("refusing to launch an unsafe plan (kind %d, k %d, e %lld): %s", kind, k,
                                            (long long)e, bad.c_str()));
    p.waves = (i64)lanes.size() / kWaveLanes;
    p.rows = rows;
    HIP_CHECK(hipMalloc(&p.d, lanes.size() * sizeof(LaneDesc)));
    upload(p.d, lanes.data(), lanes.size() * sizeof(LaneDesc));
    return plans_.emplace(key, p).first->second;
}

}  // namespace hipeng
}  // namespace gol
