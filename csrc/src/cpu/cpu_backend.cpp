// gol-mi355x: CPU stepper and host-side board helpers (see cpu.hpp).
#include <algorithm>
#include <cstring>

#include "gol/bits.hpp"
#include "gol/cpu.hpp"

namespace gol {
namespace cpu {

void step_rows(const u64* src, u64* dst, const Layout& L, i64 r_lo, i64 r_hi) {
    const i64 n = L.nw + 2;  // words -1 .. nw
#pragma omp parallel for schedule(static) if ((r_hi - r_lo) * n > 16384)
    for (i64 r = r_lo; r < r_hi; ++r) {
        const u64* up = src + L.index(r - 1, -1);
        const u64* mid = src + L.index(r, -1);
        const u64* dn = src + L.index(r + 1, -1);
        u64* out = dst + L.index(r, -1);
        for (i64 j = 0; j < n; ++j) {
            u64 pu = j ? up[j - 1] : 0, nu = j + 1 < n ? up[j + 1] : 0;
            u64 pm = j ? mid[j - 1] : 0, nm = j + 1 < n ? mid[j + 1] : 0;
            u64 pd = j ? dn[j - 1] : 0, nd = j + 1 < n ? dn[j + 1] : 0;
            u64 a0, a1, b0, b1, c0, c1;
            hsum64(pu, up[j], nu, a0, a1);
            hsum64(pm, mid[j], nm, b0, b1);
            hsum64(pd, dn[j], nd, c0, c1);
            out[j] = rule64(a0, a1, b0, b1, c0, c1, mid[j]);
        }
    }
}

u64* superstep(u64* a, u64* b, const Layout& L, int k) {
    if (k < 1 || k > L.R) throw Error(strprintf("superstep depth %d outside 1..%d", k, L.R));
    u64* src = a;
    u64* dst = b;
    for (int g = 0; g < k; ++g) {
        i64 ext = k - 1 - g;
        step_rows(src, dst, L, -ext, L.h + ext);
        std::swap(src, dst);
    }
    return src;
}

void fill_ghost_cols_wrap(u64* buf, const Layout& L, i64 r_lo, i64 r_hi) {
    for (i64 r = r_lo; r < r_hi; ++r) wrap_row_ghosts(buf + L.index(r, 0), L.w, L.nw);
}

void fill_ghost_rows_wrap(u64* buf, const Layout& L) {
    for (i64 g = 1; g <= L.R; ++g) {
        i64 top = -g, bot = L.h - 1 + g;
        std::memcpy(buf + L.index(top, -1), buf + L.index(pmod(top, L.h), -1), (size_t)L.pitch * 8);
        std::memcpy(buf + L.index(bot, -1), buf + L.index(pmod(bot, L.h), -1), (size_t)L.pitch * 8);
    }
}

void init_tile(u64* buf, const Layout& L, const Geometry& g, const PatternSpec& p) {
    std::memset(buf, 0, (size_t)L.bytes());
    const i64 gwords = g.global_words(), gw0 = g.word0();
#pragma omp parallel for schedule(static) if (L.h * L.nw > 65536)
    for (i64 r = 0; r < L.h; ++r) {
        u64* row = buf + L.index(r, 0);
        for (i64 c = 0; c < L.nw; ++c) {
            u64 v = 0;
            if (p.fill == Fill::Ones)
                v = ~0ull;
            else if (p.fill == Fill::Random)
                v = random_word(p.seed, g.row0 + r, gw0 + c, gwords);
            row[c] = split_word(v & L.mask(c));
        }
    }
    for (const auto& rc : p.cells) {
        i64 r = rc.first - g.row0, c = rc.second - g.col0;
        if (r < 0 || r >= L.h || c < 0 || c >= L.w) continue;
        buf[L.index(r, c >> 6)] |= 1ull << storage_bit(c);
    }
}

// Board storage is split-format (bits.hpp); dense words are natural order.
void extract_words(const u64* buf, const Layout& L, u64* dense) {
    for (i64 r = 0; r < L.h; ++r) {
        const u64* row = buf + L.index(r, 0);
        for (i64 c = 0; c < L.nw; ++c) dense[r * L.nw + c] = merge_word(row[c]) & L.mask(c);
    }
}

void insert_words(u64* buf, const Layout& L, const u64* dense) {
    for (i64 r = 0; r < L.h; ++r) {
        u64* row = buf + L.index(r, 0);
        for (i64 c = 0; c < L.nw; ++c) row[c] = split_word(dense[r * L.nw + c] & L.mask(c));
    }
}

u64 population(const u64* buf, const Layout& L) {
    u64 n = 0;
    for (i64 r = 0; r < L.h; ++r) {
        const u64* row = buf + L.index(r, 0);
        for (i64 c = 0; c < L.nw; ++c) n += (u64)__builtin_popcountll(row[c] & storage_mask(c, L.w));
    }
    return n;
}

// Defined on natural-order words, so it does not depend on the storage format.
u64 fingerprint(const u64* buf, const Layout& L, i64 grow0, i64 gword0, i64 gwords) {
    u64 s = 0;
    for (i64 r = 0; r < L.h; ++r) {
        const u64* row = buf + L.index(r, 0);
        for (i64 c = 0; c < L.nw; ++c)
            s += fingerprint_word((u64)(grow0 + r) * (u64)gwords + (u64)(gword0 + c), merge_word(row[c]) & L.mask(c));
    }
    return s;
}

}  // namespace cpu
}  // namespace gol
