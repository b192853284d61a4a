// gol-mi355x: benchmark helpers.
#pragma once

#include "gol/common.hpp"

namespace gol {
namespace bench {

// Reference-class yardstick on one GPU: N x N byte-per-cell torus, one thread per cell, global
// loads only, one launch per generation, optionally a device sync per generation (as the reference
// does, gol-with-cuda.cu:277) — but no device printf.  Returns seconds for `gens` generations and
// the final population in *pop.
double naive_byte_run(i64 N, int gens, int threads, bool sync_each, u64 seed, u64* pop);

}  // namespace bench
}  // namespace gol
