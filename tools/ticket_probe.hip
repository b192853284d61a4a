// ticket_probe: what a persistent grid's shared work counter costs on MI355X (flow kernel design input).
//
//   mode 0  every wave draws tickets (one agent-scope atomic add per draw, lane 0 adds 1) until N
//   mode 1  the same, each draw followed by 4 agent-scope loads of another word of the same 128-B line
//           (the flow kernel's fault polling next to its ticket counter)
//   mode 2  the same loads from a word 256 B away
//   mode 3  draws of 4 tickets at once (a wave takes 4 consecutive tickets per atomic)
//   mode 4  one counter per XCD (HW_REG_XCC_ID), N / 8 tickets each
//   mode 5  the "done" count only: one atomic per wave, then exit
//   mode 6  one atomic per 256-thread workgroup (after a barrier), then exit
//   mode 7  an empty kernel of the same grid
//
// Usage: ticket_probe [N] [blocks_per_cu]; prints us per launch (median of 20) and ns per ticket.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__device__ __forceinline__ unsigned draw(unsigned* c, int lane, unsigned n) {
    return __builtin_amdgcn_readfirstlane(
        __hip_atomic_fetch_add(c, lane == 0 ? n : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__global__ __launch_bounds__(256) void probe(unsigned* ctr, unsigned N, int mode, unsigned* sink) {
    const int lane = threadIdx.x & 63;
    unsigned acc = 0;
    if (mode == 7) {
        acc = lane;
    } else if (mode == 5) {
        acc += draw(ctr, lane, 1);
    } else if (mode == 6) {
        __syncthreads();
        if (threadIdx.x < 64) acc += draw(ctr, lane, 1);
    } else if (mode == 4) {
        unsigned xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        unsigned* c = ctr + 64 * xcc;  // 256 B apart
        for (;;) {
            const unsigned t = draw(c, lane, 1);
            if (t >= N / 8) break;
            acc += t;
        }
    } else {
        const unsigned step = mode == 3 ? 4u : 1u;
        for (;;) {
            const unsigned t = draw(ctr, lane, step);
            if (t >= N) break;
            acc += t;
            if (mode == 1 || mode == 2) {
                const unsigned* w = mode == 1 ? ctr + 4 : ctr + 64;
                for (int i = 0; i < 4; ++i)
                    acc += __builtin_amdgcn_readfirstlane(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            }
        }
    }
    if (acc == 0xFFFFFFFFu) sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const unsigned N = argc > 1 ? (unsigned)atoi(argv[1]) : 10000u;
    const int bpc = argc > 2 ? atoi(argv[2]) : 3;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int blocks = bpc * prop.multiProcessorCount;
    unsigned *ctr = nullptr, *sink = nullptr;
    CK(hipMalloc(&ctr, 4096));
    CK(hipMalloc(&sink, 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("ticket_probe: N %u, %d blocks (%d waves)\n", N, blocks, blocks * 4);
    const char* names[] = {"draws", "draws+4 loads same line", "draws+4 loads other line", "draws of 4", "per-XCD counters",
                           "one atomic per wave", "one atomic per workgroup", "empty kernel"};
    for (int mode = 0; mode < 8; ++mode) {
        std::vector<float> ts;
        for (int r = 0; r < 21; ++r) {
            CK(hipMemset(ctr, 0, 4096));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, ctr, N, mode, sink);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) ts.push_back(ms * 1e3f);
        }
        std::sort(ts.begin(), ts.end());
        const float med = ts[ts.size() / 2];
        const double n_atomics = mode == 5 ? blocks * 4.0 : mode == 6 ? blocks : mode == 3 ? N / 4.0 + blocks * 4 : N + blocks * 4.0;
        printf("mode %d %-28s min %8.2f med %8.2f us  (%6.2f ns per atomic)\n", mode, names[mode], ts[0], med,
               med * 1e3 / n_atomics);
    }
    return 0;
}
