// gol-mi355x: reference-compatible output — the stdout report lines and the per-rank board dump.
//
// Byte-for-byte the reference's formats:
//   stdout (rank 0):  "TOTAL DURATION : %.5lf, number of cell updates = %ld\n"   gol-main.c:124
//                     "This is the Game of Life running in parallel on a GPU on multiple ranks.\n"
//                                                                                 gol-main.c:132
//   Rank_<r>_of_<P>.txt (gol-main.c:66), header gol-main.c:136, rows gol-main.c:17-28:
//     "######################### FINAL WORLD IN RANK <r> IS ###############################\n"
//     "Row %2d: " then "%u " per cell, then "\n", one line per row, label = first global row + i.
// The dump formatter works straight from the bit-packed words with a byte->16-char table instead of
// one fprintf per cell (gol-main.c:24), so multi-GiB dumps are I/O bound, not printf bound.
#pragma once

#include <cstdio>
#include <string>

#include "gol/common.hpp"

namespace gol {
namespace io {

std::string dump_filename(int rank, int nranks);
std::string dump_header(int rank);
void write_header(FILE* fp, int rank);
// `dense`: rows x nw packed words (bit b of word c = column 64c+b), valid width w.
void write_rows(FILE* fp, const u64* dense, i64 rows, i64 w, i64 nw, i64 label0);
std::string format_rows(const u64* dense, i64 rows, i64 w, i64 nw, i64 label0);

std::string timing_line(double duration, long count);
extern const char* const kBanner;

}  // namespace io
}  // namespace gol
