// gol-mi355x: decomposition + layout implementation.  See geometry.hpp.
#include "gol/geometry.hpp"

#include <algorithm>
#include <cmath>

namespace gol {

const char* dir_name(Dir d) {
    static const char* n[NUM_DIRS] = {"N", "S", "W", "E", "NW", "NE", "SW", "SE"};
    return n[d];
}

static std::vector<i64> even_split(i64 total, int parts, i64 unit) {
    // Split `total` into `parts` contiguous pieces in units of `unit` (the last piece absorbs the
    // remainder that is not a whole unit).  Starts are multiples of `unit`.
    std::vector<i64> s(parts + 1);
    i64 units = total / unit;
    i64 base = units / parts, extra = units % parts;
    i64 pos = 0;
    for (int i = 0; i < parts; ++i) {
        s[i] = pos * unit;
        pos += base + (i < extra ? 1 : 0);
    }
    s[parts] = total;
    return s;
}

std::string Decomposition::describe() const {
    return strprintf("%s %lldx%lld board, P=%d, grid %dx%d (%s)", per_rank ? "per-rank" : "global",
                     (long long)H, (long long)W, P, Px, Py, two_d() ? "2d" : "1d");
}

static void choose_grid(int P, i64 H, i64 W, int& Px, int& Py) {
    // Pick Px*Py == P minimising the halo perimeter per tile (sum of tile height and width),
    // subject to tile widths being >= 64 cells.
    double best = 1e300;
    Px = 1;
    Py = P;
    for (int px = 1; px <= P; ++px) {
        if (P % px) continue;
        int py = P / px;
        if (px > 1 && W / 64 < px) continue;
        if (py > H) continue;
        double th = (double)H / py, tw = (double)W / px;
        // Column halos cost a word per row and a pack/unpack; weigh them a bit higher.
        double cost = tw + (px > 1 ? 1.5 : 0.0) * th;
        if (cost < best) {
            best = cost;
            Px = px;
            Py = py;
        }
    }
}

Decomposition make_decomposition(i64 N, int P, bool global_mode, const std::string& decomp,
                                 const std::string& grid, i64 width) {
    if (P < 1) throw Error("number of ranks must be >= 1");
    if (N < 1) throw Error(strprintf("world size must be >= 1 (got %lld)", (long long)N));
    if (width < 0) throw Error(strprintf("board width must be >= 1 (got %lld)", (long long)width));
    Decomposition d;
    d.P = P;
    d.per_rank = !global_mode;
    d.W = width > 0 ? width : N;
    d.H = global_mode ? N : N * (i64)P;
    if (global_mode && d.H < P) throw Error("global board has fewer rows than ranks");

    int Px = 1, Py = P;
    std::string dm = decomp.empty() ? "1d" : decomp;
    if (!grid.empty() && grid != "auto") {
        int a = 0, b = 0;
        if (sscanf(grid.c_str(), "%dx%d", &a, &b) != 2 || a < 1 || b < 1 || a * b != P)
            throw Error(strprintf("GOL_GRID=%s does not describe %d ranks (expected PxxPy)", grid.c_str(), P));
        Px = a;
        Py = b;
    } else if (dm == "2d" || dm == "auto") {
        choose_grid(P, d.H, d.W, Px, Py);
        if (dm == "2d" && Px == 1 && P > 1) {
            // force a genuinely 2-D grid when asked for and possible
            for (int px = 2; px <= P; ++px)
                if (P % px == 0 && d.W / 64 >= px) {
                    Px = px;
                    Py = P / px;
                    break;
                }
        }
    } else if (dm != "1d") {
        throw Error("GOL_DECOMP must be 1d, 2d or auto (got " + dm + ")");
    }
    if (Px > 1 && (d.W % 64) != 0) {
        // Column halos are whole 64-cell words: a 2-D split needs W % 64 == 0.  Fall back to strips.
        fprintf(stderr, "[gol] 2-D decomposition needs a width divisible by 64 (W=%lld); using 1-D strips\n",
                (long long)d.W);
        Px = 1;
        Py = P;
    }
    if (Px > 1 && d.W / 64 < Px) throw Error("2-D grid has more column ranks than 64-cell words");
    if (Py > d.H) throw Error("grid has more row ranks than board rows");
    d.Px = Px;
    d.Py = Py;
    d.want_2d = Px > 1 || (dm == "2d" && (d.W % 64) == 0);
    d.row_starts = even_split(d.H, Py, 1);
    d.col_starts = (Px > 1) ? even_split(d.W, Px, 64) : std::vector<i64>{0, d.W};
    if (d.per_rank) {
        d.strip_starts.resize(P + 1);
        for (int s = 0; s <= P; ++s) d.strip_starts[s] = N * (i64)s;
    } else {
        d.strip_starts = even_split(d.H, P, 1);
    }
    return d;
}

Geometry make_geometry(const Decomposition& dec, int rank) {
    if (rank < 0 || rank >= dec.P) throw Error("rank out of range");
    Geometry g;
    g.dec = dec;
    g.rank = rank;
    g.cx = rank % dec.Px;
    g.cy = rank / dec.Px;
    g.row0 = dec.row_starts[g.cy];
    g.h = dec.row_starts[g.cy + 1] - g.row0;
    g.col0 = dec.col_starts[g.cx];
    g.w = dec.col_starts[g.cx + 1] - g.col0;
    for (int d = 0; d < NUM_DIRS; ++d)
        g.nbr[d] = dec.rank_of(g.cx + dir_dx((Dir)d), g.cy + dir_dy((Dir)d));
    return g;
}

Layout::Layout(i64 h_, i64 w_, int R_) : h(h_), w(w_), R(R_) {
    if (h < 1 || w < 1) throw Error("tile must have at least one row and one column");
    if (R < 1) throw Error("halo depth must be >= 1");
    nw = ceil_div(w, 64);
    pitch = round_up(nw + 2, 2);  // (128-byte aligned rows, 528 words at 32768^2, measured 1-8% slower)
}

int clamp_halo_depth(const Decomposition& dec, int requested) {
    i64 min_h = dec.H;
    for (int i = 0; i < dec.Py; ++i) min_h = std::min(min_h, dec.row_starts[i + 1] - dec.row_starts[i]);
    i64 r = std::max(1, requested);
    // the column halo is one 64-cell word: in 2-D a superstep may not exceed 63 generations; 1-D
    // strips have no column halo (128: deep supersteps for the two-sub-tile mode)
    r = std::min<i64>(r, dec.Px > 1 ? 63 : 128);
    r = std::min<i64>(r, min_h);
    return (int)std::max<i64>(1, r);
}

}  // namespace gol
