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
    return 0;
}
