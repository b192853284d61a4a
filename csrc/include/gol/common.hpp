// gol-mi355x: common types, error handling and environment helpers.
//
// The reference keeps all state in C globals shared across two translation units
// (/root/reference/gol-main.c:11-13, gol-with-cuda.cu:9-30) and reports errors with
// printf + exit(-1).  Here state lives in typed objects (Geometry, Layout, Engine) and
// errors travel as gol::Error exceptions until the CLI converts them into the reference's
// exact message + exit status (see cli/main.cpp).
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace gol {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i32 = int32_t;
using i64 = int64_t;

// Generic framework error.
struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// An error that must be reported to the user with an exact, reference-compatible message and
// process exit status (e.g. "Pattern %u has not been implemented \n" -> 255).
struct ContractError : Error {
    int exit_status;
    ContractError(const std::string& msg, int status) : Error(msg), exit_status(status) {}
};

std::string strprintf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

std::string env_str(const char* name, const std::string& dflt = "");
long long env_int(const char* name, long long dflt);
bool env_flag(const char* name, bool dflt);

inline i64 ceil_div(i64 a, i64 b) { return (a + b - 1) / b; }
inline i64 round_up(i64 a, i64 b) { return ceil_div(a, b) * b; }
// Mathematical modulo (result in [0, m)).
inline i64 pmod(i64 a, i64 m) {
    i64 r = a % m;
    return r < 0 ? r + m : r;
}

// splitmix64 finaliser: the counter-based hash used for decomposition-invariant random init
// (pattern 5) and for the board fingerprint.  Identical on host and device.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline u64 mix64(u64 z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Random word for global word coordinates (grow, gword) of a board whose rows have `gwords`
// 64-bit words.  Bit b of the word is the cell at column 64*gword + b.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline u64 random_word(u64 seed, i64 grow, i64 gword, i64 gwords) {
    return mix64(seed * 0xD1B54A32D192ED03ull ^ mix64((u64)grow * (u64)gwords + (u64)gword));
}

// Mask of the valid bits of word `c` of a row of width `w` cells.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline u64 word_mask(i64 c, i64 w) {
    i64 rem = w - 64 * c;
    if (rem >= 64) return ~0ull;
    if (rem <= 0) return 0ull;
    return (1ull << rem) - 1ull;
}

}  // namespace gol
