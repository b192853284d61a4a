#include <chrono>
// gol-mi355x: host-side C++ unit tests (no GPU needed).  Run: build/gol_unit
//
// Covers: CLI parsing, decomposition geometry, pattern placement (survey §2.9), planner coverage,
// the bit-sliced CPU stepper vs a byte-per-cell oracle (any width, incl. N % 64 != 0), temporal
// supersteps vs single generations, dump formatting, and multi-rank engines over ThreadTransport
// (1-D and 2-D, P <= 2 canonical ordering) against the single-rank result.
#include <cstring>
#include <functional>
#include <random>
#include <thread>

#include "gol/bits.hpp"
#include "gol/config.hpp"
#include "gol/cpu.hpp"
#include "gol/engine.hpp"
#include "gol/io.hpp"
#include "gol/pattern.hpp"
#include "gol/plan.hpp"

using namespace gol;

static int g_fail = 0, g_pass = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            if (g_fail < 20) fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                         \
        } else {                                                              \
            ++g_pass;                                                         \
        }                                                                     \
    } while (0)

// ---------- byte oracle ----------
static std::vector<u8> byte_step(const std::vector<u8>& b, i64 H, i64 W) {
    std::vector<u8> o(b.size());
    for (i64 y = 0; y < H; ++y)
        for (i64 x = 0; x < W; ++x) {
            int n = 0;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx)
                    if (dy || dx) n += b[(size_t)(pmod(y + dy, H) * W + pmod(x + dx, W))];
            u8 c = b[(size_t)(y * W + x)];
            o[(size_t)(y * W + x)] = (u8)(n == 3 || (c && n == 2));
        }
    return o;
}

static std::vector<u64> pack(const std::vector<u8>& b, i64 H, i64 W) {
    i64 nw = ceil_div(W, 64);
    std::vector<u64> w((size_t)(H * nw), 0);
    for (i64 y = 0; y < H; ++y)
        for (i64 x = 0; x < W; ++x)
            if (b[(size_t)(y * W + x)]) w[(size_t)(y * nw + x / 64)] |= 1ull << (x % 64);
    return w;
}

static std::vector<u8> random_board(i64 H, i64 W, unsigned seed) {
    std::mt19937 rng(seed);
    std::vector<u8> b((size_t)(H * W));
    for (auto& v : b) v = (u8)(rng() & 1);
    return b;
}

static void test_cli() {
    CliArgs a;
    const char* bad[] = {"gol", "1", "2"};
    CHECK(!parse_cli(3, bad, a));
    const char* ok[] = {"gol", "4", "32", "2", "66000", "1"};
    CHECK(parse_cli(6, ok, a));
    CHECK(a.pattern == 4 && a.world_size == 32 && a.iterations == 2 && a.on_off == 1);
    CHECK(a.threads == (unsigned short)66000);  // ushort truncation like the reference
    CHECK(std::string(kUsage).find("GOL requires 5 arguments") == 0);
}

static void test_geometry() {
    Decomposition d = make_decomposition(32, 4, false, "1d", "");
    CHECK(d.H == 128 && d.W == 32 && d.Px == 1 && d.Py == 4);
    Geometry g = make_geometry(d, 0);
    CHECK(g.nbr[DIR_N] == 3 && g.nbr[DIR_S] == 1 && g.h == 32);
    Decomposition d2 = make_decomposition(256, 8, true, "2d", "4x2");
    CHECK(d2.Px == 4 && d2.Py == 2 && d2.col_starts[1] == 64);
    Geometry g5 = make_geometry(d2, 5);  // cx=1, cy=1
    CHECK(g5.cx == 1 && g5.cy == 1 && g5.nbr[DIR_NW] == 0 && g5.nbr[DIR_SE] == 2 && g5.nbr[DIR_E] == 6);
    Decomposition d3 = make_decomposition(100, 3, true, "1d", "");
    CHECK(d3.row_starts[1] == 34 && d3.row_starts[3] == 100);
    CHECK(clamp_halo_depth(d3, 99) == 33);
}

static void test_patterns() {
    Decomposition d = make_decomposition(140, 2, false, "1d", "");
    PatternSpec p2 = make_pattern(2, d, 0);
    CHECK(p2.cells.size() == 20);
    CHECK(p2.cells[0].first == 139 && p2.cells[0].second == 127 && p2.cells[9].second == 136);
    CHECK(p2.cells[10].first == 279);
    PatternSpec p3 = make_pattern(3, make_decomposition(6, 1, false, "1d", ""), 0);
    CHECK(p3.cells.size() == 2);  // P=1: else-if never sets the lower corners
    PatternSpec p3b = make_pattern(3, make_decomposition(6, 2, false, "1d", ""), 0);
    CHECK(p3b.cells.size() == 4 && p3b.cells[2].first == 11 && p3b.cells[2].second == 0);
    PatternSpec p4 = make_pattern(4, make_decomposition(6, 2, false, "1d", ""), 0);
    CHECK(p4.cells.size() == 3 && p4.cells[2].second == 5);
    bool threw = false;
    try {
        make_pattern(7, d, 0);
    } catch (const ContractError& e) {
        threw = std::string(e.what()) == "Pattern 7 has not been implemented \n" && e.exit_status == 255;
    }
    CHECK(threw);
}

static void test_plan() {
    for (i64 nw : {1, 2, 61, 62, 63, 130, 512}) {
        for (bool xwrap : {false, true}) {
            std::vector<Region> rg = {{0, 7, 0, nw}, {7, 40, 0, nw}};
            PlanStats st;
            auto lanes = build_plan(rg, nw, 40, 9, 2, xwrap, &st);
            std::vector<int> cover((size_t)(40 * nw), 0);
            for (size_t w = 0; w < lanes.size() / 64; ++w) {
                int nrows = lanes[w * 64].nrows;
                for (int l = 0; l < 64; ++l) {
                    const LaneDesc& d = lanes[w * 64 + l];
                    CHECK(d.nrows == nrows);
                    CHECK(d.col >= -1 && d.col <= nw);
                    if (xwrap) CHECK(d.col >= 0 && d.col < nw);
                    if (d.flags & LANE_STORE)
                        for (int r = 0; r < d.nrows; ++r) cover[(size_t)((d.row0 + r) * nw + d.col)]++;
                }
            }
            bool all1 = true;
            for (int c : cover) all1 &= c == 1;
            CHECK(all1);
            CHECK(validate_plan(lanes, nw, 40, 2, 2, false).empty());
        }
    }
    // multi-pass extension: output rows [-e, h+e) with k-deep inputs inside the R-row halo
    for (int R : {8, 32}) {
        for (int k : {1, 4, 8}) {
            const i64 e = R - k, h = 100, nw = 70;
            auto lanes = build_plan({{-e, h + e, 0, nw}}, nw, h, 13, k, true);
            CHECK(validate_plan(lanes, nw, h, R, k, false).empty());
            CHECK(!validate_plan(lanes, nw, h, R - 1, k, false).empty());  // one row too deep
        }
    }
    // folded-tile plans: 32-lane tiles (<= 30 output words + 2 halo lanes), lanes 32-63 repeat lanes
    // 0-31, every output word stored by exactly one lane of the first halves
    for (i64 nw : {1, 29, 30, 31, 128, 130}) {
        for (bool xwrap : {false, true}) {
            const i64 h = 300;
            PlanStats st;
            auto lanes = build_plan({{0, h, 0, nw}}, nw, h, 139, 24, xwrap, &st, 1, 8, true);
            CHECK(validate_plan(lanes, nw, h, 24, 24, false).empty());
            std::vector<int> cover((size_t)(h * nw), 0);
            bool dup = true;
            for (size_t w = 0; w < lanes.size() / 64; ++w) {
                int run = 0;
                for (int l = 0; l < 32; ++l) {
                    const LaneDesc& d = lanes[w * 64 + l];
                    const LaneDesc& e = lanes[w * 64 + 32 + l];
                    dup &= d.row0 == e.row0 && d.col == e.col && d.flags == e.flags && d.nrows == e.nrows;
                    run = (d.flags & LANE_STORE) ? run + 1 : 0;
                    CHECK(run <= 30);
                    if (d.flags & LANE_STORE)
                        for (int r = 0; r < d.nrows; ++r) cover[(size_t)((d.row0 + r) * nw + d.col)]++;
                }
            }
            CHECK(dup);
            bool all1 = true;
            for (int c : cover) all1 &= c == 1;
            CHECK(all1);
            CHECK(st.out_words == h * nw);
        }
    }
    // a corrupted lane is reported
    auto lanes = build_plan({{0, 10, 0, 5}}, 5, 10, 10, 1, false);
    lanes[3].col = 9;
    CHECK(!validate_plan(lanes, 5, 10, 1, 1, false).empty());
}

static void test_cpu_step() {
    for (i64 W : {1, 2, 5, 63, 64, 65, 127, 137, 200}) {
        for (i64 H : {1, 3, 17}) {
            auto b = random_board(H, W, (unsigned)(W * 131 + H));
            Layout L(H, W, 1);
            std::vector<u64> a((size_t)L.words(), 0), c((size_t)L.words(), 0);
            auto pw = pack(b, H, W);
            cpu::insert_words(a.data(), L, pw.data());
            u64* cur = a.data();
            u64* oth = c.data();
            auto ref = b;
            for (int g = 0; g < 4; ++g) {
                cpu::fill_ghost_cols_wrap(cur, L, 0, H);
                cpu::fill_ghost_rows_wrap(cur, L);
                cpu::step_rows(cur, oth, L, 0, H);
                std::swap(cur, oth);
                ref = byte_step(ref, H, W);
            }
            std::vector<u64> out((size_t)(H * L.nw));
            cpu::extract_words(cur, L, out.data());
            CHECK(out == pack(ref, H, W));
        }
    }
}

// Engine over P thread-ranks; returns the global board (H x nw words) of the result.
static std::vector<u64> run_engines(i64 N, int P, bool global, const std::string& decomp, const std::string& grid,
                                    int depth, unsigned pattern, int gens, bool compat, u64* fp_out = nullptr) {
    Decomposition d = make_decomposition(N, P, global, decomp, grid);
    auto group = make_thread_group(P);
    const i64 gw = ceil_div(d.W, 64);
    std::vector<u64> board((size_t)(d.H * gw), 0);
    std::vector<std::thread> th;
    std::vector<u64> fps((size_t)P);
    for (int r = 0; r < P; ++r)
        th.emplace_back([&, r] {
            auto t = std::make_shared<ThreadTransport>(group, r);
            Geometry g = make_geometry(d, r);
            EngineConfig c;
            c.backend = "cpu";
            c.halo_depth = depth;
            c.compat = compat;
            auto e = Engine::create(g, c, t);
            e->init(make_pattern(pattern, d, 77));
            e->run((u64)gens);
            auto w = e->tile_words();
            fps[(size_t)r] = e->fingerprint();
            i64 nw = e->layout().nw;
            for (i64 y = 0; y < g.h; ++y)
                memcpy(&board[(size_t)((g.row0 + y) * gw + g.word0())], &w[(size_t)(y * nw)], (size_t)nw * 8);
        });
    for (auto& x : th) x.join();
    if (fp_out) *fp_out = fps[0];
    return board;
}

static void test_engines() {
    // 1-D and 2-D, P in {1,2,3,4}, depth in {1,3,8}, vs a single-rank depth-1 run of the global board
    for (int P : {1, 2, 3, 4}) {
        for (int depth : {1, 3, 8}) {
            auto ref = run_engines(64 * P, 1, true, "1d", "", 1, 5, 13, false);
            auto got = run_engines(64 * P, P, true, "1d", "", depth, 5, 13, false);
            CHECK(got == ref);
            if (P == 4 || P == 2) {
                auto g2 = run_engines(64 * P, P, true, "2d", P == 4 ? "2x2" : "2x1", depth, 5, 13, false);
                CHECK(g2 == ref);
            }
        }
    }
    // per-rank mode (reference geometry), odd width, vs byte oracle of the (P*N) x N torus
    for (int P : {1, 2, 3}) {
        const i64 N = 37;
        Decomposition d = make_decomposition(N, P, false, "1d", "");
        auto got = run_engines(N, P, false, "1d", "", 4, 5, 9, false);
        std::vector<u8> b((size_t)(d.H * d.W));
        const i64 gw = ceil_div(d.W, 64);
        for (i64 y = 0; y < d.H; ++y)
            for (i64 x = 0; x < d.W; ++x)
                b[(size_t)(y * d.W + x)] = (u8)((random_word(77, y, x / 64, gw) >> (x % 64)) & 1);
        for (int g = 0; g < 9; ++g) b = byte_step(b, d.H, d.W);
        CHECK(got == pack(b, d.H, d.W));
    }
    // deep 2-D supersteps (ghost words recomputed inside a superstep, up to 63 generations)
    {
        auto ref = run_engines(256, 1, true, "1d", "", 1, 5, 70, false);
        CHECK(run_engines(256, 4, true, "2d", "2x2", 63, 5, 70, false) == ref);
        CHECK(run_engines(256, 2, true, "2d", "2x1", 32, 5, 70, false) == ref);
    }
    // fingerprint invariance across decompositions
    u64 f1 = 0, f2 = 0, f3 = 0;
    run_engines(256, 1, true, "1d", "", 8, 5, 20, false, &f1);
    run_engines(256, 4, true, "1d", "", 8, 5, 20, false, &f2);
    run_engines(256, 4, true, "2d", "2x2", 8, 5, 20, false, &f3);
    CHECK(f1 == f2 && f2 == f3 && f1 != 0);
}

static void test_compat() {
    // Quirk model (survey Q3): P=1, pattern 4 blinker across the x-wrap, constant ghost rows =
    // (above = own first row, below = own last row).
    const i64 N = 6;
    auto got = run_engines(N, 1, false, "1d", "", 1, 4, 1, true);
    // emulate: ghost above = row0 (1 1 0 0 0 1), below = row5 (0s)
    std::vector<u8> b((size_t)(N * N), 0);
    b[0] = b[1] = b[5] = 1;
    std::vector<u8> ext((size_t)((N + 2) * N), 0);
    for (i64 x = 0; x < N; ++x) ext[(size_t)x] = b[(size_t)x];                       // above
    for (i64 y = 0; y < N; ++y)
        for (i64 x = 0; x < N; ++x) ext[(size_t)((y + 1) * N + x)] = b[(size_t)(y * N + x)];
    std::vector<u8> o((size_t)(N * N));
    for (i64 y = 0; y < N; ++y)
        for (i64 x = 0; x < N; ++x) {
            int n = 0;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx)
                    if (dy || dx) n += ext[(size_t)((y + 1 + dy) * N + pmod(x + dx, N))];
            u8 c = b[(size_t)(y * N + x)];
            o[(size_t)(y * N + x)] = (u8)(n == 3 || (c && n == 2));
        }
    CHECK(got == pack(o, N, N));
}

static void test_dump() {
    std::vector<u64> w = {0b100011ull};
    std::string s = io::format_rows(w.data(), 1, 6, 1, 0);
    CHECK(s == "Row  0: 1 1 0 0 0 1 \n");
    CHECK(io::dump_header(3) ==
          "######################### FINAL WORLD IN RANK 3 IS ###############################\n");
    CHECK(io::timing_line(0.5, 1234) == "TOTAL DURATION : 0.50000, number of cell updates = 1234\n");
    CHECK(io::dump_filename(2, 8) == "Rank_2_of_8.txt");
    std::vector<u64> w2 = {~0ull, 0x5ull};
    std::string s2 = io::format_rows(w2.data(), 1, 67, 2, 123);
    CHECK(s2.substr(0, 9) == "Row 123: " && s2.size() == 9 + 2 * 67 + 1 && s2.substr(9 + 128, 6) == "1 0 1 ");
}

static void test_bits() {
    CHECK(bitop3_ref(0xF0, 0xCC, 0xAA, kLutXor3) == (0xF0ull ^ 0xCC ^ 0xAA) && kLutOne3 != kLutT34);
    std::vector<u64> row = {0x8000000000000001ull};
    CHECK(wrap64(row.data(), 64, -64) == row[0] && wrap64(row.data(), 64, 1) == ((row[0] >> 1) | (row[0] << 63)));
    std::vector<u64> r5 = {0b10011ull};  // width 5: periodic 1 1 0 0 1
    u64 v = wrap64(r5.data(), 5, 5);
    CHECK((v & 0x3FF) == 0b1001110011ull);
    // split storage: round trip, bit positions, and hsum64 vs a natural-order horizontal sum
    u64 z = 0x9E3779B97F4A7C15ull;
    for (int t = 0; t < 200; ++t) {
        z = mix64(z + (u64)t);
        CHECK(merge_word(split_word(z)) == z && split_word(merge_word(z)) == z);
    }
    for (int c = 0; c < 64; ++c) CHECK(split_word(1ull << c) == (1ull << storage_bit(c)));
    CHECK(split_word(0x2ull) == (1ull << 32) && storage_mask(0, 3) == 0x100000003ull);
    for (int t = 0; t < 100; ++t) {
        const u64 p = mix64(3 * (u64)t + 1), c = mix64(3 * (u64)t + 2), n = mix64(3 * (u64)t + 3);
        u64 s0, s1;
        hsum64(split_word(p), split_word(c), split_word(n), s0, s1);
        const u64 L = (c << 1) | (p >> 63), R = (c >> 1) | (n << 63);
        CHECK(merge_word(s0) == (L ^ c ^ R) && merge_word(s1) == ((L & c) | (L & R) | (c & R)));
    }
    // ghost fill of an unaligned periodic row in split storage (width 70 = 2 words)
    {
        const i64 w = 70;
        std::vector<u8> cells((size_t)w);
        std::vector<u64> nat(2, 0);
        for (i64 x = 0; x < w; ++x) {
            cells[(size_t)x] = (u8)(mix64((u64)x) & 1);
            if (cells[(size_t)x]) nat[(size_t)(x >> 6)] |= 1ull << (x & 63);
        }
        std::vector<u64> row = {0, split_word(nat[0]), split_word(nat[1]), 0};
        wrap_row_ghosts(row.data() + 1, w, 2);
        bool ok = true;
        for (i64 x = -64; x < 128 + 64; ++x) {
            const i64 word = x < 0 ? -1 : x >> 6;
            const u64 bit = (merge_word(row[(size_t)(word + 1)]) >> (x & 63)) & 1;
            ok = ok && bit == cells[(size_t)pmod(x, w)];
        }
        CHECK(ok);
    }
}

static void test_watchdog() {
    std::atomic<int> fired{0};
    {
        Watchdog wd(0.05, [&](const std::string&) { fired++; });
        std::this_thread::sleep_for(std::chrono::milliseconds(150));
        CHECK(fired.load() == 0);  // disarmed: never fires
        wd.arm(true);
        for (int i = 0; i < 10; ++i) {  // kicked in time: no fire
            std::this_thread::sleep_for(std::chrono::milliseconds(10));
            wd.kick("work");
        }
        CHECK(fired.load() == 0);
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
        CHECK(fired.load() >= 1);  // stalled while armed: fires
        wd.arm(false);
    }
}

// Host emulation of step_resident's data flow (resident_kernel.hip): tiles of a plan, bands of B rows
// per wave, edge slots double-buffered by generation parity (inactive bands leave theirs stale),
// trapezoid skips, supersteps publishing store lanes' rows into alternating boards and reloading the
// rest, on split-format words with the device's lane semantics (lanes -1 / 64 read 0).  Checked against
// the byte oracle; every word a tile reloads must be owned by itself or one of its neighbours.
static std::string emulate_resident(const std::vector<LaneDesc>& lanes, i64 nw, i64 h, int NW, int Bb, int G, int S,
                                    int K, std::vector<u64>& A, std::vector<u64>& Bd) {
    const size_t nt = lanes.size() / 64;
    std::vector<u32> off, idx;
    const std::string bad = resident_neighbours(lanes, nw, h, K, true, off, idx);
    if (!bad.empty()) return bad;
    std::vector<int> owner((size_t)(h * nw), -1);
    for (size_t t = 0; t < nt; ++t)
        for (int l = 0; l < 64; ++l) {
            const LaneDesc& d = lanes[t * 64 + l];
            if (d.nrows > 0 && (d.flags & LANE_STORE))
                for (int r = 0; r < d.nrows; ++r) owner[(size_t)((d.row0 + r) * nw + d.col)] = (int)t;
        }
    const int E = NW * Bb;
    auto word = [&](std::vector<u64>& buf, const LaneDesc& d, int e) -> u64& {
        return buf[(size_t)(pmod((i64)d.row0 - K + e, h) * nw + d.col)];
    };
    // state[t][l][e], slots[t][par][band][first/last][l]
    std::vector<std::vector<std::vector<u64>>> st(nt, std::vector<std::vector<u64>>(64, std::vector<u64>((size_t)E, 0)));
    std::vector<u64> slots(nt * 2 * (size_t)NW * 2 * 64, 0);
    auto slot = [&](size_t t, int par, int b, int fl, int l) -> u64& {
        return slots[(((t * 2 + (size_t)par) * (size_t)NW + (size_t)b) * 2 + (size_t)fl) * 64 + (size_t)l];
    };
    for (size_t t = 0; t < nt; ++t) {
        const int nrows = lanes[t * 64].nrows;
        if (nrows <= 0) continue;
        if (nrows + 2 * K > E) return "tile taller than NW x B";
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < nrows + 2 * K; ++e) st[t][l][(size_t)e] = word(A, lanes[t * 64 + l], e);
    }
    for (int s = 1; s <= S; ++s) {
        const int ks = G / S + (s <= G % S ? 1 : 0);
        for (int g = 1; g <= ks; ++g) {
            const int par = g & 1;
            for (size_t t = 0; t < nt; ++t) {
                const int T = lanes[t * 64].nrows + 2 * K;
                if (T <= 2 * K) continue;
                for (int w = 0; w < NW; ++w) {
                    const int b0 = w * Bb;
                    if (!(b0 + Bb > g - 1 && b0 < T - g + 1)) continue;
                    for (int l = 0; l < 64; ++l) {
                        slot(t, par, w, 0, l) = st[t][l][(size_t)b0];
                        slot(t, par, w, 1, l) = st[t][l][(size_t)(b0 + Bb - 1)];
                    }
                }
                std::vector<std::vector<u64>> nx = st[t];
                for (int w = 0; w < NW; ++w) {
                    const int b0 = w * Bb;
                    if (!(b0 + Bb > g - 1 && b0 < T - g + 1)) continue;
                    // rows -1 .. B of the band for all lanes
                    auto row = [&](int i, int l) -> u64 {
                        if (l < 0 || l > 63) return 0;
                        if (i < 0) return w > 0 ? slot(t, par, w - 1, 1, l) : 0;
                        if (i >= Bb) return w < NW - 1 ? slot(t, par, w + 1, 0, l) : 0;
                        return st[t][l][(size_t)(b0 + i)];
                    };
                    for (int i = 0; i < Bb; ++i)
                        for (int l = 0; l < 64; ++l) {
                            u64 a0, a1, b0s, b1, c0, c1;
                            hsum64(row(i - 1, l - 1), row(i - 1, l), row(i - 1, l + 1), a0, a1);
                            hsum64(row(i, l - 1), row(i, l), row(i, l + 1), b0s, b1);
                            hsum64(row(i + 1, l - 1), row(i + 1, l), row(i + 1, l + 1), c0, c1);
                            nx[l][(size_t)(b0 + i)] = rule64(a0, a1, b0s, b1, c0, c1, row(i, l));
                        }
                }
                st[t] = nx;
            }
        }
        std::vector<u64>& X = ((S - s) & 1) ? A : Bd;
        for (size_t t = 0; t < nt; ++t) {
            const int nrows = lanes[t * 64].nrows;
            for (int l = 0; l < 64 && nrows > 0; ++l) {
                const LaneDesc& d = lanes[t * 64 + l];
                if (d.flags & LANE_STORE)
                    for (int e = K; e < K + nrows; ++e) word(X, d, e) = st[t][l][(size_t)e];
            }
        }
        if (s == S) break;
        for (size_t t = 0; t < nt; ++t) {
            const int nrows = lanes[t * 64].nrows;
            for (int l = 0; l < 64 && nrows > 0; ++l) {
                const LaneDesc& d = lanes[t * 64 + l];
                for (int e = 0; e < nrows + 2 * K; ++e) {
                    if ((d.flags & LANE_STORE) && e >= K && e < K + nrows) continue;
                    const int o = owner[(size_t)(pmod((i64)d.row0 - K + e, h) * nw + d.col)];
                    bool known = o == (int)t;
                    for (u32 j = off[t]; j < off[t + 1] && !known; ++j) known = (int)idx[j] == o;
                    if (!known) return strprintf("tile %zu reads a word of tile %d, not a neighbour", t, o);
                    st[t][l][(size_t)e] = word(X, d, e);
                }
            }
        }
    }
    return "";
}

static void test_resident() {
    struct Case {
        i64 h, nw, rows;
        int K, NW, B, G;
    };
    for (const Case& c : std::vector<Case>{{96, 2, 24, 4, 8, 5, 13},
                                           {96, 2, 24, 4, 8, 5, 12},
                                           {80, 1, 10, 3, 4, 4, 9},
                                           {128, 3, 32, 8, 8, 6, 40},
                                           {64, 2, 64, 6, 8, 10, 17},
                                           {70, 70, 20, 5, 8, 4, 31}}) {
        const i64 W = c.nw * 64;
        auto b = random_board(c.h, W, (unsigned)(c.h * 7 + c.nw + c.G));
        std::vector<u8> ref = b;
        for (int g = 0; g < c.G; ++g) ref = byte_step(ref, c.h, W);
        auto lanes = build_plan({{0, c.h, 0, c.nw}}, c.nw, c.h, c.rows, c.K, true, nullptr, 1, 8);
        CHECK(validate_plan(lanes, c.nw, c.h, 0, c.K, true).empty());
        int S = (c.G + c.K - 1) / c.K;
        S += (S % 2 == 0);
        const int kmax = (c.G + S - 1) / S;
        std::vector<u64> A = pack(b, c.h, W), Bd(A.size(), 0);
        for (auto& x : A) x = split_word(x);
        const std::string err = emulate_resident(lanes, c.nw, c.h, c.NW, c.B, c.G, S, kmax, A, Bd);
        if (!err.empty()) fprintf(stderr, "resident emulation: %s\n", err.c_str());
        CHECK(err.empty());
        std::vector<u64> want = pack(ref, c.h, W);
        bool same = true;
        for (size_t i = 0; i < want.size(); ++i) same &= merge_word(Bd[i]) == want[i];
        CHECK(same);
    }
    // a plan with a hole in one column is refused
    auto lanes = build_plan({{0, 40, 0, 3}}, 3, 40, 10, 2, true, nullptr, 1, 8);
    for (auto& d : lanes)
        if (d.col == 1 && (d.flags & LANE_STORE) && d.row0 == 10) d.flags = 0;
    std::vector<u32> off, idx;
    CHECK(!resident_neighbours(lanes, 3, 40, 2, true, off, idx).empty());
}

// Multi-round segment heights for big regions (plan.hpp round_balanced_rows): small regions keep the
// one-round height; big ones get a whole number of full rounds with segments near round_rows.
static void test_plan_rounds() {
    const i64 resident = 3 * 4 * 256;  // 3 waves per SIMD on 256 CUs
    {
        const i64 h = 32768, nw = 512;
        std::vector<Region> rg = {{0, h, 0, nw}};
        const i64 r1 = balanced_rows_per_chunk(rg, nw, h, 8, resident, 16, true);
        CHECK(round_balanced_rows(rg, nw, h, 8, resident, 16, true, 360) == r1);  // one round: ~97 rows
    }
    {
        const i64 h = 65536, nw = 1024;  // one round is ~365 rows: stays one round
        std::vector<Region> rg = {{0, h, 0, nw}};
        const i64 r1 = balanced_rows_per_chunk(rg, nw, h, 8, resident, 16, true);
        CHECK(round_balanced_rows(rg, nw, h, 8, resident, 16, true, 360) == r1);
    }
    {
        const i64 h = 131072, nw = 2048;  // one round is ~1425 rows: four rounds of ~360
        std::vector<Region> rg = {{0, h, 0, nw}};
        const i64 r1 = balanced_rows_per_chunk(rg, nw, h, 8, resident, 16, true);
        const i64 r4 = round_balanced_rows(rg, nw, h, 8, resident, 16, true, 360);
        CHECK(r1 > 1300 && r4 < r1);
        CHECK(r4 >= 330 && r4 <= 400);
        CHECK(plan_waves(rg, nw, h, r4) <= 4 * resident && plan_waves(rg, nw, h, r4) > 3 * resident);
        CHECK(round_balanced_rows(rg, nw, h, 8, resident, 16, true, 0) == r1);  // disabled
        // at most max_rounds rounds
        const i64 r2 = round_balanced_rows(rg, nw, h, 8, resident, 16, true, 90, 2);
        CHECK(plan_waves(rg, nw, h, r2) <= 2 * resident && plan_waves(rg, nw, h, r2) > resident);
        // the plan still covers every output word exactly once
        PlanStats st;
        std::vector<LaneDesc> lanes = build_plan(rg, nw, h, r4, 8, true, &st, 4, 8);
        CHECK(validate_plan(lanes, nw, h, 8, 8, true).empty());
        CHECK(st.out_words == h * nw);
    }
    {
        // BASELINE config 5's 2^20 x 2^20 tile: the row search of a 512-workgroup plan from 1-row
        // segments up must not pack the candidate plans it can reject by counting (it took minutes)
        const i64 h = 1 << 20, nw = 1 << 14;
        std::vector<Region> rg = {{0, h, 0, nw}};
        const auto t0 = std::chrono::steady_clock::now();
        const i64 r = balanced_rows_per_chunk(rg, nw, h, 24, 512, 1, true);
        const i64 r32 = round_balanced_rows(rg, nw, h, 8, resident, 16, true, 360);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CHECK(s < 10.0);
        CHECK(r > 500000 && plan_waves(rg, nw, h, r) <= 512);
        CHECK(plan_waves(rg, nw, h, r32) <= 32 * resident && plan_waves(rg, nw, h, r32) > 31 * resident);
    }
}

// Age-weighted plans (build_plan age_weights): the plan still covers every output word exactly once,
// fits the same waves, and the first-dispatched third of the grid gets the tallest segments.
// A band with ghost rows above (or below) it as a tile-kernel plan (one tile per 62-word column; the
// shape of the sub-tile overlap's band, docs/PERFORMANCE.md §11): every output word once, inside the halo.
static void test_band_tile_plan() {
    for (const auto& c : std::vector<std::tuple<i64, i64, int, i64>>{{16384, 512, 12, 8}, {16384, 512, 8, 0}, {4096, 100, 12, 8}}) {
        const i64 h = std::get<0>(c), nw = std::get<1>(c), e = std::get<3>(c);
        const int k = std::get<2>(c);
        for (int s = 0; s < 2; ++s) {
            const std::vector<Region> rg = {{s == 0 ? -e : h - k, s == 0 ? k : h + e, 0, nw}};
            const i64 band = rg[0].r1 - rg[0].r0;
            PlanStats st;
            const std::vector<LaneDesc> lanes = build_plan(rg, nw, h, band, k, true, &st, 1, 8);
            CHECK(validate_plan(lanes, nw, h, 128, k, false).empty());
            CHECK(st.out_words == band * nw);
            const i64 tiles = (i64)lanes.size() / kWaveLanes;
            CHECK(tiles >= (nw + kSegWords - 1) / kSegWords && tiles <= (nw + kSegWords - 1) / kSegWords + 4);
            for (i64 t = 0; t < tiles; ++t) CHECK(lanes[(size_t)(t * kWaveLanes)].nrows == 0 || lanes[(size_t)(t * kWaveLanes)].nrows == band);
        }
    }
}

static void test_plan_age_weights() {
    const std::vector<double> w = {1.6, 1.15, 0.75};
    for (const auto& c : std::vector<std::pair<i64, i64>>{{32768, 512}, {16384, 256}, {8192, 512}, {4000, 100}}) {
        const i64 h = c.first, nw = c.second;
        std::vector<Region> rg = {{0, h, 0, nw}};
        const i64 resident = 3 * 4 * 256;
        const i64 rows = balanced_rows_per_chunk(rg, nw, h, 8, resident, 16, true);
        PlanStats s0, s1;
        const std::vector<LaneDesc> eq = build_plan(rg, nw, h, rows, 8, true, &s0, 4, 8);
        const std::vector<LaneDesc> aw = build_plan(rg, nw, h, rows, 8, true, &s1, 4, 8, false, &w);
        CHECK(validate_plan(aw, nw, h, 8, 8, true).empty());
        CHECK(s1.out_words == h * nw);
        const i64 waves = (i64)aw.size() / kWaveLanes, nwg = waves / 4;
        CHECK(waves <= (i64)eq.size() / kWaveLanes + 8);
        // every output word exactly once
        std::vector<int> cover((size_t)(h * nw), 0);
        for (i64 wv = 0; wv < waves; ++wv)
            for (int l = 0; l < kWaveLanes; ++l) {
                const LaneDesc& d = aw[(size_t)(wv * kWaveLanes + l)];
                if (!(d.flags & LANE_STORE)) continue;
                for (i64 r = d.row0; r < d.row0 + d.nrows; ++r) ++cover[(size_t)(r * nw + d.col)];
            }
        bool once = true;
        for (int v : cover) once = once && v == 1;
        CHECK(once);
        // mean full-segment height by dispatch third: decreasing, in about the weights' ratios
        double sum[3] = {0, 0, 0}, n[3] = {0, 0, 0};
        for (i64 wv = 0; wv < waves; ++wv) {
            const LaneDesc& d = aw[(size_t)(wv * kWaveLanes)];
            if (d.nrows <= 0 || !(aw[(size_t)(wv * kWaveLanes + 62)].flags & LANE_STORE)) continue;  // full segments
            const int cls = (int)std::min<i64>(2, (wv / 4) * 3 / std::max<i64>(1, nwg));
            sum[cls] += d.nrows;
            n[cls] += 1;
        }
        if (n[0] > 0 && n[1] > 0 && n[2] > 0) {
            const double m0 = sum[0] / n[0], m1 = sum[1] / n[1], m2 = sum[2] / n[2];
            CHECK(m0 > m1 && m1 > m2);
            CHECK(std::fabs(m0 / m2 - w[0] / w[2]) < 0.35 * w[0] / w[2]);
        }
    }
}

// cheapest_cut: the pass cut of a superstep from measured per-depth pass costs (plan.hpp).
static void test_cheapest_cut() {
    // one tile, 32768^2-like costs: shallow passes cost nearly as much as deep ones
    std::map<int, double> c = {{4, 74}, {6, 78}, {7, 80}, {8, 83}, {12, 122}};
    CHECK((cheapest_cut(20, c) == std::vector<int>{12, 8}));
    CHECK((cheapest_cut(16, c) == std::vector<int>{8, 8}));
    CHECK((cheapest_cut(8, c) == std::vector<int>{8}));
    // a step_pipe depth of 20 cheaper than any mix of shallower passes (config 3's strip)
    std::map<int, double> s = {{6, 15.2}, {7, 20.0}, {8, 21.5}, {16, 38.0}, {20, 46.0}};
    CHECK((cheapest_cut(20, s) == std::vector<int>{20}));
    CHECK((cheapest_cut(27, s) == std::vector<int>{20, 7}));
    // the sum of the cut is always k when depth 1 exists; empty when no depth sums to k
    std::map<int, double> d = {{1, 10}, {5, 20}};
    for (int k = 1; k <= 40; ++k) {
        const std::vector<int> v = cheapest_cut(k, d);
        int sum = 0;
        for (int x : v) sum += x;
        CHECK(sum == k && std::is_sorted(v.rbegin(), v.rend()));
    }
    CHECK(cheapest_cut(3, {{2, 1.0}}).empty());
    CHECK(cheapest_cut(0, d).empty());
}

int main() {
    test_cheapest_cut();
    test_band_tile_plan();
    test_plan_age_weights();
    test_watchdog();
    test_plan_rounds();
    test_cli();
    test_geometry();
    test_patterns();
    test_plan();
    test_resident();
    test_bits();
    test_cpu_step();
    test_dump();
    test_engines();
    test_compat();
    printf("gol_unit: %d checks passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
