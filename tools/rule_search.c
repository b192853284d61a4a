// Exhaustive search for the B3/S23 rule as a circuit of 3-input boolean gates (v_bitop3_b32).
//
// After the vertical adder tree of the bit-sliced counter (bits.hpp) the rule is a function of five
// bit-planes: x0 = parity of the 3 row-sums' low bits, cy = their majority, u0 / u1 = parity /
// majority of the high bits (T = x0 + 2*(cy + u0 + 2*u1)), and alive.  The textbook evaluation takes
// 4 gates.  This tool enumerates every circuit of 2 and 3 gates (any 3 of the available signals,
// any of the 256 LUTs), with the don't-care "alive with T = 0" (T counts the centre cell), and prints
// the circuits found.  It also checks whether "exactly two of five inputs" (the same condition after
// folding x0 in) fits in 3 gates.
//
// Pair mode (round 6, stencil_device.hpp PAIR): two vertically adjacent output rows share two input rows,
// so their vertical sum P = a + b (0..6: planes p0, p1, p2, 4 gates) can be computed once per pair and each
// output finished from (p0, p1, p2, c0, c1, alive), c the third row's 2-bit sum.  pair_search() shows that
// no 3-gate finish exists and lists 4-gate finishes of the shape F(G(u, v, w), s, t) (the last two gates
// decomposed: the target must be a function of the 5 signals, and each of its 4 cofactors in (s, t) one of
// 0, 1, G, ~G), then checks the kept circuit on every (a, b, c, alive).
//
//   gcc -O2 -o /tmp/rule_search tools/rule_search.c && /tmp/rule_search
#include <stdint.h>
#include <stdio.h>

typedef uint32_t T;  // truth table over 5 inputs (32 rows)

static T gate(int lut, T a, T b, T c) {
    T g = 0;
    for (int m = 0; m < 8; m++)
        if (lut >> m & 1) g |= ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c);
    return g;
}

// Is `target` (on the rows in `care`) a function of the three signals?  Returns the LUT or -1.
static int fits(T a, T b, T c, T target, T care) {
    int tbl[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
    for (int i = 0; i < 32; i++) {
        if (!(care >> i & 1)) continue;
        int m = ((a >> i & 1) << 2) | ((b >> i & 1) << 1) | (c >> i & 1), t = target >> i & 1;
        if (tbl[m] < 0)
            tbl[m] = t;
        else if (tbl[m] != t)
            return -1;
    }
    int lut = 0;
    for (int m = 0; m < 8; m++)
        if (tbl[m] == 1) lut |= 1 << m;
    return lut;
}

// Circuits of `ngates` (2 or 3) gates; the last gate's LUT is solved for, earlier ones enumerated.
static long search(const char* what, const char* const* names, T target, T care, int ngates, int show) {
    T sig[8];
    for (int v = 0; v < 5; v++) {
        sig[v] = 0;
        for (int i = 0; i < 32; i++)
            if (i >> v & 1) sig[v] |= 1u << i;
    }
    long found = 0;
    for (int a = 0; a < 5; a++)
        for (int b = a + 1; b < 5; b++)
            for (int c = b + 1; c < 5; c++)
                for (int l1 = 0; l1 < 256; l1++) {
                    sig[5] = gate(l1, sig[a], sig[b], sig[c]);
                    if (ngates == 2) {
                        for (int p = 0; p < 6; p++)
                            for (int q = p + 1; q < 6; q++)
                                for (int r = q + 1; r < 6; r++)
                                    if (fits(sig[p], sig[q], sig[r], target, care) >= 0) found++;
                        continue;
                    }
                    for (int d = 0; d < 6; d++)
                        for (int e = d + 1; e < 6; e++)
                            for (int f = e + 1; f < 6; f++)
                                for (int l2 = 0; l2 < 256; l2++) {
                                    sig[6] = gate(l2, sig[d], sig[e], sig[f]);
                                    for (int p = 0; p < 7; p++)
                                        for (int q = p + 1; q < 7; q++)
                                            for (int r = q + 1; r < 7; r++) {
                                                const int l3 = fits(sig[p], sig[q], sig[r], target, care);
                                                if (l3 < 0) continue;
                                                if (found++ < show) {
                                                    const char* nm[8] = {names[0], names[1], names[2], names[3], names[4],
                                                                         "g1", "g2", ""};
                                                    printf("  g1 = lut%02X(%s,%s,%s)  g2 = lut%02X(%s,%s,%s)  out = lut%02X(%s,%s,%s)\n",
                                                           l1, nm[a], nm[b], nm[c], l2, nm[d], nm[e], nm[f], l3, nm[p],
                                                           nm[q], nm[r]);
                                                }
                                            }
                                }
                }
    printf("%s: %ld circuits of %d gates\n", what, found, ngates);
    return found;
}

typedef uint64_t T6;  // truth table over (p0, p1, p2, c0, c1, alive): 64 rows
static T6 gate6(int lut, T6 a, T6 b, T6 c) {
    T6 g = 0;
    for (int m = 0; m < 8; m++)
        if (lut >> m & 1) g |= ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c);
    return g;
}
static int fits6(T6 a, T6 b, T6 c, T6 tgt, T6 care) {
    int lut = 0;
    for (int m = 0; m < 8; m++) {
        T6 mk = ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c) & care, on = mk & tgt;
        if (on && on != mk) return -1;
        if (on) lut |= 1 << m;
    }
    return lut;
}
static void pair_search(void) {
    T6 sig[8], tgt = 0, care = 0;
    for (int v = 0; v < 6; v++) {
        sig[v] = 0;
        for (int i = 0; i < 64; i++)
            if (i >> v & 1) sig[v] |= 1ull << i;
    }
    for (int i = 0; i < 64; i++) {
        const int P = (i & 1) + 2 * (i >> 1 & 1) + 4 * (i >> 2 & 1), c = (i >> 3 & 1) + 2 * (i >> 4 & 1), x = i >> 5 & 1;
        if (P == 7 || (x && P + c == 0)) continue;  // P <= 6; alive => T >= 1
        care |= 1ull << i;
        if (P + c == 3 || (x && P + c == 4)) tgt |= 1ull << i;
    }
    long n3 = 0;  // 3 gates: g1, g2 enumerated, the last solved for
    for (int a = 0; a < 6; a++) for (int b = a + 1; b < 6; b++) for (int c = b + 1; c < 6; c++)
        for (int l1 = 0; l1 < 256; l1++) {
            sig[6] = gate6(l1, sig[a], sig[b], sig[c]);
            for (int d = 0; d < 7; d++) for (int e = d + 1; e < 7; e++) for (int f = e + 1; f < 7; f++)
                for (int l2 = 0; l2 < 256; l2++) {
                    sig[7] = gate6(l2, sig[d], sig[e], sig[f]);
                    for (int p = 0; p < 8; p++) for (int q = p + 1; q < 8; q++) for (int r = q + 1; r < 8; r++)
                        if (fits6(sig[p], sig[q], sig[r], tgt, care) >= 0) n3++;
                }
        }
    printf("pair finish: %ld circuits of 3 gates\n", n3);
    // the kept 4-gate finish, checked on every (a, b, c, alive) with the pair sum's own 4 gates
    int err = 0;
    for (int A = 0; A < 4; A++) for (int B = 0; B < 4; B++) for (int C = 0; C < 4; C++) for (int x = 0; x < 2; x++) {
        const int a0 = A & 1, a1 = A >> 1, b0 = B & 1, b1 = B >> 1, c0 = C & 1, c1 = C >> 1, t = a0 & b0;
        const int p0 = a0 ^ b0, p1 = a1 ^ b1 ^ t, p2 = (a1 & b1) | (a1 & t) | (b1 & t), Tt = A + B + C;
        if (x && Tt == 0) continue;
        const int g1 = 0x43 >> (p0 << 2 | c0 << 1 | x) & 1, g3 = 0x25 >> (p1 << 2 | p2 << 1 | c1) & 1;
        const int g2 = 0x27 >> (p2 << 2 | x << 1 | g1) & 1, out = 0x42 >> (g3 << 2 | g1 << 1 | g2) & 1;
        if (out != (Tt == 3 || (x && Tt == 4))) err++;
    }
    printf("pair finish g1=f43(p0,c0,x) g3=f25(p1,p2,c1) g2=f27(p2,x,g1) next=f42(g3,g1,g2): %d errors\n", err);
}

int main(void) {
    // rule over (x0, cy, u0, u1, alive); bit v of the row index is input v
    static const char* const rn[5] = {"x0", "cy", "u0", "u1", "alive"};
    T rule = 0, rcare = 0;
    for (int i = 0; i < 32; i++) {
        const int x0 = i & 1, cy = i >> 1 & 1, u0 = i >> 2 & 1, u1 = i >> 3 & 1, al = i >> 4 & 1;
        const int t = x0 + 2 * (cy + u0 + 2 * u1);
        if (!(al && t == 0)) rcare |= 1u << i;  // alive => T >= 1
        if (t == 3 || (al && t == 4)) rule |= 1u << i;
    }
    search("B3/S23 rule", rn, rule, rcare, 2, 0);
    search("B3/S23 rule", rn, rule, rcare, 3, 4);
    // exactly two of five inputs
    static const char* const en[5] = {"a", "b", "c", "d", "e"};
    T two = 0;
    for (int i = 0; i < 32; i++)
        if (__builtin_popcount(i) == 2) two |= 1u << i;
    search("exactly-2-of-5", en, two, 0xFFFFFFFFu, 3, 2);
    pair_search();
    return 0;
}
