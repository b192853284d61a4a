// gol-mi355x: segment planner for the temporal-blocked stencil kernel (see plan.hpp).
#include "gol/plan.hpp"

#include <algorithm>
#include <cstdlib>
#include <limits>
#include <string>
#include <map>
#include <set>
#include <tuple>

namespace gol {

namespace {

struct Item {
    i64 r0, nrows, c0, nwords;
    int lanes() const { return (int)nwords + 2; }
};

// Lanes of one packed tile: a 64-lane wave, or (fold) the 32-lane half that both halves of a
// folded tile share (plan.hpp)
int pack_lanes(bool fold) { return fold ? kWaveLanes / 2 : kWaveLanes; }

}  // namespace

i64 choose_rows_per_chunk(const std::vector<Region>& regions, int k, i64 target_waves, i64 min_rows) {
    // lane-rows of output work, expressed in waves of full segments
    double seg_rows = 0;
    i64 max_rows = 1;
    for (const Region& r : regions) {
        i64 rows = r.r1 - r.r0, words = r.c1 - r.c0;
        if (rows <= 0 || words <= 0) continue;
        seg_rows += (double)rows * (double)words / kSegWords;
        max_rows = std::max(max_rows, rows);
    }
    if (seg_rows <= 0) return 1;
    i64 s = (i64)(seg_rows / (double)std::max<i64>(1, target_waves));
    s = std::max<i64>(s, std::max<i64>(min_rows, 4 * (i64)k));
    return std::max<i64>(1, std::min(s, max_rows));
}

i64 balanced_rows_per_chunk(const std::vector<Region>& regions, i64 nw, i64 h, int k, i64 resident_waves,
                            i64 min_rows, bool xwrap, bool fold) {
    i64 max_rows = 1;
    for (const Region& r : regions) max_rows = std::max(max_rows, r.r1 - r.r0);
    (void)k;
    (void)xwrap;
    // fits(S): the plan of S-row segments has at most resident_waves waves.  The full-width segments
    // alone (one wave each) bound the count from below, so a height whose bound already exceeds the
    // target is rejected without packing the plan: packing materialises every segment, which for
    // short segments of a big tile is hundreds of millions of them (a 2^20-row board's search used to
    // start by packing 1-row segments and spent minutes in the kernel autotune).
    const i64 lw = pack_lanes(fold), sw = lw - 2;
    auto fits = [&](i64 S) {
        double full = 0, narrow_lanes = 0;  // (narrow segments: their lanes incl. 2 halo lanes, packed <= lw per wave)
        for (const Region& r : regions) {
            const i64 rows = r.r1 - r.r0, words = r.c1 - r.c0;
            if (rows <= 0 || words <= 0) continue;
            full += (double)ceil_div(rows, S) * (double)(words / sw);
            if (words % sw) narrow_lanes += (double)ceil_div(rows, S) * (double)(words % sw + 2);
        }
        if (full + narrow_lanes / (double)lw > (double)resident_waves) return false;
        return plan_waves(regions, nw, h, S, fold) <= resident_waves;
    };
    i64 lo = std::max<i64>(1, std::min(min_rows, max_rows)), hi = max_rows;
    if (fits(lo)) return lo;
    if (!fits(hi)) return hi;  // cannot fit one round: fewest, tallest segments
    while (hi - lo > 1) {  // !fits(lo), fits(hi)
        i64 mid = (lo + hi) / 2;
        if (fits(mid))
            hi = mid;
        else
            lo = mid;
    }
    return hi;
}

i64 round_balanced_rows(const std::vector<Region>& regions, i64 nw, i64 h, int k, i64 resident_waves, i64 min_rows,
                        bool xwrap, i64 round_rows, i64 max_rounds) {
    const i64 r1 = balanced_rows_per_chunk(regions, nw, h, k, resident_waves, min_rows, xwrap);
    if (round_rows <= 0 || r1 < 2 * round_rows) return r1;  // (rounds would be 1)
    const i64 rounds = std::max<i64>(1, std::min<i64>(max_rounds, (r1 + round_rows / 2) / round_rows));
    // the tallest segments whose plan fits `rounds` full rounds of resident waves
    return balanced_rows_per_chunk(regions, nw, h, k, rounds * resident_waves, min_rows, xwrap);
}

namespace {

// Cut the regions into segments of <= rows_per_chunk rows x <= 62 words and pack them into waves:
// full-width segments get a wave each; narrow ones (same height) are packed first-fit-decreasing.
// `bands` (one region only): its row bands' heights, top to bottom, instead of equal ones.
std::vector<std::vector<Item>> pack_waves(const std::vector<Region>& regions, i64 nw, i64 h, i64 rows_per_chunk,
                                          bool fold, const std::vector<i64>* bands = nullptr) {
    if (rows_per_chunk < 1) rows_per_chunk = 1;
    const int lw = pack_lanes(fold), sw = lw - 2;
    std::map<i64, std::vector<Item>> by_rows;
    for (const Region& rg : regions) {
        i64 rows = rg.r1 - rg.r0, words = rg.c1 - rg.c0;
        if (rows <= 0 || words <= 0) continue;
        // rows may extend into the ghost rows and columns into the ghost words (multi-pass
        // supersteps: at most the 64-row halo and the one-word column halo)
        if (rg.r0 < -128 || rg.r1 > h + 128 || rg.c0 < -1 || rg.c1 > nw + 1) throw Error("plan region outside the tile");
        i64 nch = bands ? (i64)bands->size() : ceil_div(rows, rows_per_chunk);
        i64 base = rows / nch, extra = rows % nch;
        i64 r = rg.r0;
        for (i64 ch = 0; ch < nch; ++ch) {
            i64 nr = bands ? (*bands)[(size_t)ch] : base + (ch < extra ? 1 : 0);
            for (i64 c = rg.c0; c < rg.c1; c += sw) by_rows[nr].push_back({r, nr, c, std::min<i64>(sw, rg.c1 - c)});
            r += nr;
        }
    }
    std::vector<std::vector<Item>> waves;
    for (auto& kv : by_rows) {
        std::vector<Item> narrow;
        for (const Item& it : kv.second) {
            if (it.lanes() == lw)
                waves.push_back({it});
            else
                narrow.push_back(it);
        }
        std::stable_sort(narrow.begin(), narrow.end(),
                         [](const Item& a, const Item& b) { return a.lanes() > b.lanes(); });
        std::vector<std::pair<int, std::vector<Item>>> open;  // used lanes, items
        size_t first_open = 0;  // waves before this index are full (< 3 free lanes)
        for (const Item& it : narrow) {
            bool placed = false;
            for (size_t j = first_open; j < open.size(); ++j) {
                auto& w = open[j];
                if (w.first + it.lanes() <= lw) {
                    w.first += it.lanes();
                    w.second.push_back(it);
                    placed = true;
                    break;
                }
            }
            if (!placed) open.push_back({it.lanes(), {it}});
            while (first_open < open.size() && open[first_open].first > lw - 3) ++first_open;
        }
        for (auto& w : open) waves.push_back(std::move(w.second));
    }
    return waves;
}

}  // namespace

i64 plan_waves(const std::vector<Region>& regions, i64 nw, i64 h, i64 rows_per_chunk, bool fold) {
    return round_up(std::max<i64>(1, (i64)pack_waves(regions, nw, h, rows_per_chunk, fold).size()), kWavesPerBlock);
}

namespace {

// The permutation of whole workgroups that gives XCD x (workgroup b runs on XCD b % xcds) a
// contiguous stretch of the plan order: order[s] = the launch index of plan-order workgroup s.
std::vector<i64> xcd_order(i64 nwg, int xcds) {
    std::vector<i64> order((size_t)nwg);
    for (i64 b = 0; b < nwg; ++b) order[(size_t)b] = b;
    if (xcds > 1)
        std::stable_sort(order.begin(), order.end(), [xcds](i64 a, i64 b) {
            return a % xcds != b % xcds ? a % xcds < b % xcds : a / xcds < b / xcds;
        });
    return order;
}

// Row-band heights of a single-region plan weighted by dispatch class (build_plan age_weights): the
// band count of the equal-height plan, band i's class from the launch index of its first full-width
// segment, heights proportional to the class weights (>= 1 row, summing to the region's rows).
std::vector<i64> age_bands(const Region& rg, i64 rows_per_chunk, int wg_waves, int xcds, const std::vector<double>& w) {
    const i64 rows = rg.r1 - rg.r0, words = rg.c1 - rg.c0;
    const i64 nb = ceil_div(rows, std::max<i64>(1, rows_per_chunk));
    const i64 full = words / kSegWords, narrow = words % kSegWords ? words % kSegWords + 2 : 0;
    if (nb < 2 || full < 1) return {};
    const i64 per_wave = narrow ? kWaveLanes / narrow : 1;  // narrow segments per packed wave
    const i64 nwaves = round_up(nb * full + (narrow ? ceil_div(nb, per_wave) : 0), kWavesPerBlock);
    const i64 nwg = nwaves / std::max(1, wg_waves);
    const std::vector<i64> order = xcd_order(nwg, xcds);
    const i64 C = (i64)w.size();
    std::vector<double> wt((size_t)nb);
    double sum = 0;
    // (the weighted plan orders every wave by its first segment's rows, the packed narrow ones among
    // the full-width ones of their bands: band i starts at wave i x (full + 1 / per_wave))
    const double per_band = (double)full + (narrow ? 1.0 / (double)per_wave : 0.0);
    for (i64 i = 0; i < nb; ++i) {
        const i64 s = std::min(nwg - 1, (i64)((double)i * per_band) / std::max(1, wg_waves));
        const i64 cls = std::min(C - 1, order[(size_t)s] * C / nwg);
        wt[(size_t)i] = std::max(0.05, w[(size_t)cls]);
        sum += wt[(size_t)i];
    }
    std::vector<i64> bands((size_t)nb);
    i64 used = 0;
    double acc = 0;
    for (i64 i = 0; i < nb; ++i) {  // cumulative rounding: every band >= 1 row, the total exact
        acc += wt[(size_t)i] * (double)rows / sum;
        const i64 end = std::min(rows - (nb - 1 - i), std::max(used + 1, (i64)(acc + 0.5)));
        bands[(size_t)i] = end - used;
        used = end;
    }
    bands.back() += rows - used;
    return bands;
}

}  // namespace

std::vector<LaneDesc> build_plan(const std::vector<Region>& regions, i64 nw, i64 h, i64 rows_per_chunk, int k,
                                 bool xwrap, PlanStats* stats, int wg_waves, int xcds, bool fold,
                                 const std::vector<double>* age_weights) {
    std::vector<i64> bands;
    if (age_weights && age_weights->size() > 1 && regions.size() == 1 && !fold)
        bands = age_bands(regions[0], rows_per_chunk, wg_waves < 1 ? 1 : wg_waves, xcds, *age_weights);
    std::vector<std::vector<Item>> packed = pack_waves(regions, nw, h, rows_per_chunk, fold, bands.empty() ? nullptr : &bands);
    const int lw = pack_lanes(fold);
    i64 nwaves = round_up(std::max<i64>(1, (i64)packed.size()), kWavesPerBlock);
    // XCD-aware order.  The full-width segments are sorted (narrow, packed waves stay last), then
    // whole workgroups are permuted so that XCD x — workgroup b is dispatched to XCD b % xcds — runs
    // a contiguous stretch of that order: neighbouring segments, which share halo rows and words,
    // are hits in its own L2.  Row-major: the full-width segments of a row band are consecutive, so an
    // XCD's stretch of the order is a band of whole rows and its stores cover whole rows of HBM.  (The
    // column-major order, round 1's choice for vertical halo reuse in L2, which a band of rows keeps
    // too, left each XCD writing one 496-byte piece of every row: measured 32768^2 K=1 passes 71 -> 61
    // us, K=4 17.5 -> 16.1 us/gen, K=8 11.49 -> 11.20 (two halves on two streams), 16384^2 K=8 4.20 ->
    // 4.11 with row-major, profiles/plan_order_ab.txt.)
    // (Age-weighted plans order the packed narrow waves among the full-width ones, by their first
    // segment: a narrow wave holds segments of its bands' height, so it must land in their dispatch
    // class — placed last, the narrow segments of the tallest bands ran in the youngest class and
    // finished a pass ~30 us after the rest, profiles/stamp_probe.txt.)
    const bool mixed = !bands.empty();
    std::stable_sort(packed.begin(), packed.end(), [lw, mixed](const std::vector<Item>& a, const std::vector<Item>& b) {
        const bool fa = a.size() == 1 && a[0].lanes() == lw, fb = b.size() == 1 && b[0].lanes() == lw;
        if (!mixed) {
            if (fa != fb) return fa;
            if (!fa) return false;
        }
        return a[0].r0 != b[0].r0 ? a[0].r0 < b[0].r0 : a[0].c0 < b[0].c0;
    });
    std::vector<std::vector<Item>> waves((size_t)nwaves);
    if (wg_waves < 1 || nwaves % wg_waves) wg_waves = 1;
    const i64 nwg = nwaves / wg_waves;
    const std::vector<i64> order = xcd_order(nwg, xcds);
    for (i64 s = 0; s < nwg; ++s)
        for (int i = 0; i < wg_waves; ++i) {
            const size_t src = (size_t)(s * wg_waves + i);
            if (src < packed.size()) waves[(size_t)(order[(size_t)s] * wg_waves + i)] = std::move(packed[src]);
        }
    std::vector<LaneDesc> lanes((size_t)(nwaves * kWaveLanes));
    PlanStats st;
    st.waves = nwaves;
    for (size_t wi = 0; wi < (size_t)nwaves; ++wi) {
        LaneDesc* L = &lanes[wi * kWaveLanes];
        if (waves[wi].empty()) {
            for (int l = 0; l < kWaveLanes; ++l) L[l] = {0, 0, 0u, 0};
            continue;
        }
        const std::vector<Item>& w = waves[wi];
        int l = 0;
        i64 nrows = w[0].nrows;
        for (const Item& it : w) {
            for (int j = 0; j < it.lanes(); ++j, ++l) {
                i64 col = it.c0 - 1 + j;
                u32 f = 0;
                if (j >= 1 && j <= it.nwords) {
                    f |= LANE_STORE;
                    st.active_lanes += 1;
                    st.out_words += it.nrows;
                }
                if (xwrap && col == -1) col = nw - 1;
                if (xwrap && col == nw) col = 0;
                // halo lanes of a segment that includes a ghost word (2-D multi-pass) have no
                // word further out: stream the ghost word itself.  Its outer bits are garbage
                // and spread inwards one column per generation, so word 0 / nw-1 stay exact for
                // supersteps of < 64 generations.
                if (col < -1) col = -1;
                if (col > nw) col = nw;
                L[l] = {(i32)it.r0, (i32)col, f, (i32)nrows};
            }
        }
        // idle lanes: stream a valid in-bounds column (the first item's first column), never store
        for (; l < lw; ++l) L[l] = {(i32)w[0].r0, (i32)w[0].c0, 0u, (i32)nrows};
        // folded tile: lanes 32-63 repeat lanes 0-31 (they stream the other half of the same rows)
        for (; l < kWaveLanes; ++l) L[l] = L[l - lw];
        st.lane_rows += (i64)lw * (nrows + 2 * (i64)k);
    }
    if (stats) *stats = st;
    return lanes;
}

std::string validate_plan(const std::vector<LaneDesc>& lanes, i64 nw, i64 h, int R, int k, bool wrap_y) {
    if (lanes.size() % kWaveLanes) return "lane count is not a multiple of 64";
    for (size_t w = 0; w < lanes.size() / kWaveLanes; ++w) {
        const LaneDesc* L = &lanes[w * kWaveLanes];
        for (int l = 0; l < kWaveLanes; ++l) {
            const LaneDesc& d = L[l];
            if (d.nrows != L[0].nrows) return strprintf("wave %zu: nrows differs between lanes", w);
            if (d.nrows <= 0) continue;  // padding wave
            auto bad = [&](const char* what) {
                return strprintf("wave %zu lane %d (row0 %d col %d nrows %d): %s", w, l, d.row0, d.col, d.nrows, what);
            };
            if (d.col < -1 || d.col > nw) return bad("word column outside [-1, nw]");
            if (!wrap_y && (d.row0 - k < -R || (i64)d.row0 + d.nrows + k > h + R))
                return bad("input rows outside the allocated halo rows");
            if (wrap_y && (d.row0 < 0 || (i64)d.row0 + d.nrows > h)) return bad("y-wrapped rows outside the tile");
            if (d.flags & LANE_STORE) {
                if (d.col < -1 || d.col > nw) return bad("store lane outside words [-1, nw]");
                if (d.row0 < -R || (i64)d.row0 + d.nrows > h + R) return bad("store rows outside [-R, h+R)");
            }
        }
    }
    return "";
}

std::vector<int> cheapest_cut(int k, const std::map<int, double>& pass_cost) {
    std::vector<double> best((size_t)std::max(k, 0) + 1, 1e300);
    std::vector<int> pick((size_t)std::max(k, 0) + 1, 0);
    best[0] = 0;
    for (int x = 1; x <= k; ++x)
        for (const auto& dc : pass_cost)
            if (dc.first >= 1 && dc.first <= x && best[(size_t)(x - dc.first)] + dc.second < best[(size_t)x]) {
                best[(size_t)x] = best[(size_t)(x - dc.first)] + dc.second;
                pick[(size_t)x] = dc.first;
            }
    std::vector<int> ps;
    if (k < 1 || pick[(size_t)k] == 0) return ps;
    for (int x = k; x > 0; x -= pick[(size_t)x]) ps.push_back(pick[(size_t)x]);
    std::sort(ps.begin(), ps.end(), std::greater<int>());
    return ps;
}

std::string resident_neighbours(const std::vector<LaneDesc>& lanes, i64 nw, i64 h, int k, bool wrap_y,
                                std::vector<u32>& off, std::vector<u32>& idx) {
    if (lanes.size() % kWaveLanes) return "lane count is not a multiple of 64";
    const size_t nt = lanes.size() / kWaveLanes;
    // owners of every word column: (first row, end row, tile), sorted by row
    std::vector<std::vector<std::tuple<i64, i64, u32>>> own((size_t)nw);
    for (size_t t = 0; t < nt; ++t)
        for (int l = 0; l < kWaveLanes; ++l) {
            const LaneDesc& d = lanes[t * kWaveLanes + l];
            if (d.nrows <= 0) continue;
            if (d.col < 0 || d.col >= nw) return strprintf("tile %zu lane %d: column %d outside [0, nw)", t, l, d.col);
            if (d.flags & LANE_STORE) own[(size_t)d.col].emplace_back(d.row0, (i64)d.row0 + d.nrows, (u32)t);
        }
    i64 lo_row = 0, hi_row = h;  // rows the store lanes cover (every column alike)
    for (i64 c = 0; c < nw; ++c) {
        auto& v = own[(size_t)c];
        std::sort(v.begin(), v.end());
        if (v.empty()) return strprintf("column %lld has no store lane", (long long)c);
        if (c == 0) {
            lo_row = std::get<0>(v.front());
            hi_row = std::get<1>(v.back());
        }
        if (std::get<0>(v.front()) != lo_row || std::get<1>(v.back()) != hi_row)
            return strprintf("column %lld covers other rows than column 0", (long long)c);
        for (size_t i = 1; i < v.size(); ++i)
            if (std::get<0>(v[i]) != std::get<1>(v[i - 1]))
                return strprintf("column %lld: rows not covered exactly once", (long long)c);
    }
    if (wrap_y && (lo_row != 0 || hi_row != h)) return "wrapped plans must cover rows [0, h)";
    off.assign(nt + 1, 0);
    idx.clear();
    for (size_t t = 0; t < nt; ++t) {
        std::set<u32> nb;
        for (int l = 0; l < kWaveLanes; ++l) {
            const LaneDesc& d = lanes[t * kWaveLanes + l];
            if (d.nrows <= 0) continue;
            const auto& v = own[(size_t)d.col];
            // the lane's input rows, as intervals inside [lo_row, hi_row)
            std::vector<std::pair<i64, i64>> iv;
            i64 a = (i64)d.row0 - k, b = (i64)d.row0 + d.nrows + k;
            if (wrap_y) {
                if (b - a >= h) {
                    iv.push_back({0, h});
                } else {
                    a = pmod(a, h);
                    b = a + (b - ((i64)d.row0 - k));
                    if (b <= h) {
                        iv.push_back({a, b});
                    } else {
                        iv.push_back({a, h});
                        iv.push_back({0, b - h});
                    }
                }
            } else {
                // rows beyond the owned range are the rank's ghost rows: read in the first superstep
                // only (from the exchange) and beyond the valid extension later, owned by no tile
                iv.push_back({std::max(a, lo_row), std::min(b, hi_row)});
            }
            for (const auto& q : iv) {
                if (q.second <= q.first) continue;
                auto it = std::upper_bound(v.begin(), v.end(), std::make_tuple(q.first, (i64)1 << 62, (u32)0));
                if (it != v.begin()) --it;
                for (; it != v.end() && std::get<0>(*it) < q.second; ++it)
                    if (std::get<1>(*it) > q.first && std::get<2>(*it) != (u32)t) nb.insert(std::get<2>(*it));
            }
        }
        off[t + 1] = off[t] + (u32)nb.size();
        idx.insert(idx.end(), nb.begin(), nb.end());
    }
    return "";
}

}  // namespace gol
