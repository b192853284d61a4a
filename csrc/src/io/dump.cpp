// gol-mi355x: dump + report formatting (see io.hpp).
#include <algorithm>
#include <cstring>
#include <vector>

#include "gol/io.hpp"

namespace gol {
namespace io {

const char* const kBanner = "This is the Game of Life running in parallel on a GPU on multiple ranks.\n";

std::string dump_filename(int rank, int nranks) { return strprintf("Rank_%d_of_%d.txt", rank, nranks); }

std::string dump_header(int rank) {
    return strprintf("######################### FINAL WORLD IN RANK %d IS ###############################\n", rank);
}

void write_header(FILE* fp, int rank) {
    std::string h = dump_header(rank);
    fwrite(h.data(), 1, h.size(), fp);
}

namespace {

struct ByteTable {
    char t[256][16];
    ByteTable() {
        for (int v = 0; v < 256; ++v)
            for (int b = 0; b < 8; ++b) {
                t[v][2 * b] = ((v >> b) & 1) ? '1' : '0';
                t[v][2 * b + 1] = ' ';
            }
    }
};
const ByteTable& table() {
    static ByteTable tb;
    return tb;
}

// Append one formatted row to `out` (which has room: 16 + 2*w + 2 bytes).
size_t format_row(char* out, const u64* row, i64 w, i64 label) {
    size_t n = (size_t)snprintf(out, 32, "Row %2lld: ", (long long)label);
    const ByteTable& tb = table();
    i64 full_bytes = w / 8;
    for (i64 b = 0; b < full_bytes; ++b) {
        unsigned v = (unsigned)((row[b >> 3] >> ((b & 7) * 8)) & 0xFF);
        memcpy(out + n, tb.t[v], 16);
        n += 16;
    }
    for (i64 c = full_bytes * 8; c < w; ++c) {
        out[n++] = ((row[c >> 6] >> (c & 63)) & 1) ? '1' : '0';
        out[n++] = ' ';
    }
    out[n++] = '\n';
    return n;
}

}  // namespace

void write_rows(FILE* fp, const u64* dense, i64 rows, i64 w, i64 nw, i64 label0) {
    // Batch several rows per fwrite (~4 MiB).
    const size_t row_cap = (size_t)(32 + 2 * w + 1);
    const i64 batch = std::max<i64>(1, (i64)((4u << 20) / row_cap));
    std::vector<char> buf(row_cap * (size_t)batch);
    for (i64 r0 = 0; r0 < rows; r0 += batch) {
        i64 r1 = std::min(rows, r0 + batch);
        size_t n = 0;
        for (i64 r = r0; r < r1; ++r) n += format_row(buf.data() + n, dense + r * nw, w, label0 + r);
        fwrite(buf.data(), 1, n, fp);
    }
}

std::string format_rows(const u64* dense, i64 rows, i64 w, i64 nw, i64 label0) {
    std::string s;
    std::vector<char> buf((size_t)(32 + 2 * w + 1));
    for (i64 r = 0; r < rows; ++r) {
        size_t n = format_row(buf.data(), dense + r * nw, w, label0 + r);
        s.append(buf.data(), n);
    }
    return s;
}

std::string timing_line(double duration, long count) {
    return strprintf("TOTAL DURATION : %.5lf, number of cell updates = %ld\n", duration, count);
}

}  // namespace io
}  // namespace gol
