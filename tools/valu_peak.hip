// Chip-wide VALU throughput of the temporal kernel's instruction kinds on gfx950 (event-timed,
// full grid).  Reports wave-instructions per SIMD per nanosecond and per cycle at the given clock.
// hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o build/valu_peak
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(x) x x x x x x x x

template <int MODE>
__global__ __launch_bounds__(256) void peak(unsigned* out, int iters) {
    unsigned a = threadIdx.x * 2654435761u, b = a ^ 0x1234567u, c = a + 99u, d = a * 7u, e = a ^ 0xFFu, f = a + 3u,
             g = a ^ 0x5a5a5a5au;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            asm volatile(REP8("v_bitop3_b32 %0, %0, %6, %1 bitop3:0x96\n v_bitop3_b32 %1, %1, %6, %2 bitop3:0x96\n"
                              "v_bitop3_b32 %2, %2, %6, %3 bitop3:0x96\n v_bitop3_b32 %3, %3, %6, %4 bitop3:0x96\n"
                              "v_bitop3_b32 %4, %4, %6, %5 bitop3:0x96\n v_bitop3_b32 %5, %5, %6, %0 bitop3:0x96\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f)
                         : "v"(g));
        } else if (MODE == 1) {
            asm volatile(REP8("v_alignbit_b32 %0, %0, %6, 31\n v_alignbit_b32 %1, %1, %6, 31\n"
                              "v_alignbit_b32 %2, %2, %6, 31\n v_alignbit_b32 %3, %3, %6, 31\n"
                              "v_alignbit_b32 %4, %4, %6, 31\n v_alignbit_b32 %5, %5, %6, 31\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f)
                         : "v"(g));
        } else if (MODE == 2) {
            asm volatile(REP8("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                              "v_mov_b32_dpp %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                              "v_mov_b32_dpp %2, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                              "v_mov_b32_dpp %3, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                              "v_mov_b32_dpp %4, %5 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                              "v_mov_b32_dpp %5, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f));
        } else if (MODE == 3) {  // v_xor_b32 (VOP2) for comparison
            asm volatile(REP8("v_xor_b32 %0, %0, %6\n v_xor_b32 %1, %1, %6\n v_xor_b32 %2, %2, %6\n"
                              "v_xor_b32 %3, %3, %6\n v_xor_b32 %4, %4, %6\n v_xor_b32 %5, %5, %6\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f)
                         : "v"(g));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f;
}

template <int MODE>
void run(const char* name, int blocks_per_cu, int cus, double ghz) {
    const int iters = 4000, blocks = cus * blocks_per_cu;
    unsigned* out;
    (void)hipMalloc(&out, sizeof(unsigned) * blocks * 256);
    hipLaunchKernelGGL(peak<MODE>, dim3(blocks), dim3(256), 0, 0, out, 10);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(peak<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winstr = (double)blocks * 4 * iters * 48;  // wave-instructions
    const double per_simd_ns = winstr / (cus * 4.0) / (ms * 1e6);
    printf("%-10s waves/SIMD=%d  %.3f wave-instr/SIMD/ns  = %.3f per cycle @%.2f GHz\n", name, blocks_per_cu, per_simd_ns,
           per_simd_ns / ghz, ghz);
    (void)hipFree(out);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double ghz = p.clockRate / 1e6;
    printf("CUs=%d clock=%.2f GHz\n", cus, ghz);
    for (int w : {1, 2, 4, 8}) {
        run<0>("bitop3", w, cus, ghz);
        run<1>("alignbit", w, cus, ghz);
        run<2>("dpp", w, cus, ghz);
        run<3>("v_xor", w, cus, ghz);
    }
    return 0;
}
