// gol-mi355x: the byte-per-cell yardstick run (see bench.hpp).  Written from scratch as a
// measurement baseline of the reference's algorithm class; not used by the engine.
#include <hip/hip_runtime.h>

#include <chrono>
#include <vector>

#include "gol/bench.hpp"
#include "gol/hip_kernels.hpp"

namespace gol {
namespace bench {

namespace {
void check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Error(strprintf("%s: %s", what, hipGetErrorString(e)));
}
}  // namespace

double naive_byte_run(i64 N, int gens, int threads, bool sync_each, u64 seed, u64* pop) {
    const size_t n = (size_t)(N * N);
    std::vector<u8> host(n);
    const i64 gw = ceil_div(N, 64);
    for (i64 r = 0; r < N; ++r)
        for (i64 c = 0; c < N; ++c) host[(size_t)(r * N + c)] = (u8)((random_word(seed, r, c >> 6, gw) >> (c & 63)) & 1);
    u8 *a = nullptr, *b = nullptr;
    check(hipMalloc(&a, n), "hipMalloc");
    check(hipMalloc(&b, n), "hipMalloc");
    check(hipMemcpy(a, host.data(), n, hipMemcpyHostToDevice), "hipMemcpy");
    hipStream_t s;
    check(hipStreamCreate(&s), "hipStreamCreate");
    check(hipDeviceSynchronize(), "sync");
    auto t0 = std::chrono::steady_clock::now();
    for (int g = 0; g < gens; ++g) {
        // single rank torus: the ghost rows are the tile's own last / first rows
        hipk::launch_naive_byte_step(a, b, N, N, a + (N - 1) * N, a, threads, s);
        if (sync_each) check(hipStreamSynchronize(s), "sync");
        std::swap(a, b);
    }
    check(hipStreamSynchronize(s), "sync");
    auto t1 = std::chrono::steady_clock::now();
    check(hipGetLastError(), "naive kernel");
    if (pop) {
        check(hipMemcpy(host.data(), a, n, hipMemcpyDeviceToHost), "hipMemcpy");
        u64 p = 0;
        for (u8 v : host) p += v;
        *pop = p;
    }
    hipStreamDestroy(s);
    hipFree(a);
    hipFree(b);
    return std::chrono::duration<double>(t1 - t0).count();
}

}  // namespace bench
}  // namespace gol
