// Micro-benchmarks for the instructions of the temporal kernel's dependency chain (gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o build/microbench
// Prints cycles per instruction (s_memtime) for dependent chains and for independent streams.
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP16(x) x x x x x x x x x x x x x x x x

template <int MODE>
__global__ void chain(unsigned* out, unsigned long long* cyc, int iters) {
    unsigned a = threadIdx.x * 2654435761u, b = a ^ 0x1234567u, c = a + 99u, d = a * 7u, e = a ^ 0xFFu, f = a + 3u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {  // dependent v_bitop3
            asm volatile(REP16("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n") : "+v"(a) : "v"(b), "v"(c));
        } else if (MODE == 1) {  // dependent dpp wave_shr (+2 wait states required by the ISA)
            asm volatile(REP16("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n") : "+v"(a));
        } else if (MODE == 2) {  // dependent dpp row_shr
            asm volatile(REP16("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n") : "+v"(a));
        } else if (MODE == 3) {  // dependent alignbit
            asm volatile(REP16("v_alignbit_b32 %0, %0, %1, 31\n") : "+v"(a) : "v"(b));
        } else if (MODE == 4) {  // 6 independent bitop3 streams
            asm volatile(REP16("v_bitop3_b32 %0, %0, %6, %6 bitop3:0x96\n v_bitop3_b32 %1, %1, %6, %6 bitop3:0x96\n"
                               "v_bitop3_b32 %2, %2, %6, %6 bitop3:0x96\n v_bitop3_b32 %3, %3, %6, %6 bitop3:0x96\n"
                               "v_bitop3_b32 %4, %4, %6, %6 bitop3:0x96\n v_bitop3_b32 %5, %5, %6, %6 bitop3:0x96\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f)
                         : "v"(a ^ 0x5a5a5a5au));
        } else if (MODE == 6) {  // 4 independent bitop3 streams, all operands in VGPR bank 0
            asm volatile(REP16("v_bitop3_b32 v40, v40, v44, v48 bitop3:0x96\n v_bitop3_b32 v52, v52, v56, v60 bitop3:0x96\n"
                               "v_bitop3_b32 v64, v64, v68, v72 bitop3:0x96\n v_bitop3_b32 v76, v76, v80, v84 bitop3:0x96\n")
                         ::: "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68", "v72", "v76", "v80", "v84");
        } else if (MODE == 7) {  // 4 independent bitop3 streams, operands in banks 0,1,2
            asm volatile(REP16("v_bitop3_b32 v40, v40, v41, v42 bitop3:0x96\n v_bitop3_b32 v52, v52, v53, v54 bitop3:0x96\n"
                               "v_bitop3_b32 v64, v64, v65, v66 bitop3:0x96\n v_bitop3_b32 v76, v76, v77, v78 bitop3:0x96\n")
                         ::: "v40", "v41", "v42", "v52", "v53", "v54", "v64", "v65", "v66", "v76", "v77", "v78");
        } else if (MODE == 5) {  // 6 independent dpp wave_shr streams
            asm volatile(REP16("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                               "v_mov_b32_dpp %1, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                               "v_mov_b32_dpp %2, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                               "v_mov_b32_dpp %3, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                               "v_mov_b32_dpp %4, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                               "v_mov_b32_dpp %5, %5 wave_shr:1 row_mask:0xf bank_mask:0xf\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f));
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE>
double run(int blocks, int threads, int iters, int per_iter) {
    unsigned* out;
    unsigned long long* cyc;
    hipMalloc(&out, sizeof(unsigned) * blocks * threads);
    hipMalloc(&cyc, 8);
    hipLaunchKernelGGL(chain<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    hipFree(out);
    hipFree(cyc);
    return (double)c / ((double)iters * per_iter);
}

int main() {
    const int it = 2000;
    const char* names[] = {"dep bitop3", "dep dpp wave_shr (+s_nop1)", "dep dpp row_shr (+s_nop1)", "dep alignbit",
                           "6x indep bitop3", "6x indep dpp wave_shr", "4x indep bitop3 same bank", "4x indep bitop3 3 banks"};
    const int per[] = {16, 16, 16, 16, 96, 96, 64, 64};
    for (int waves : {1, 2, 4}) {
        // one workgroup of `waves` x 4 waves -> `waves` waves per SIMD on one CU
        int threads = 256 * waves;
        double r[8] = {run<0>(1, threads, it, per[0]), run<1>(1, threads, it, per[1]), run<2>(1, threads, it, per[2]),
                       run<3>(1, threads, it, per[3]), run<4>(1, threads, it, per[4]), run<5>(1, threads, it, per[5]),
                       run<6>(1, threads, it, per[6]), run<7>(1, threads, it, per[7])};
        for (int m = 0; m < 8; ++m)
            printf("waves/SIMD=%d  %-28s %.2f cycles per instruction (wave 0 view)\n", waves, names[m], r[m]);
    }
    return 0;
}
