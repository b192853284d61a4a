// Why does v_bitop3_b32 issue slower than v_xor_b32 (tools/valu_peak.hip: 0.73 vs 0.92 wave-instr
// per SIMD per ns)?  Candidates: the 8-byte VOP3 encoding, or VGPR bank conflicts between its three
// sources (bank = register index mod 4).  Fixed registers (v40..v63), 12 independent destinations
// per round, every CU busy.
// hipcc --offload-arch=gfx950 -O3 tools/valu_bank.hip -o build/valu_bank
#include <hip/hip_runtime.h>

#include <cstdio>

#define R4(x) x x x x
#define CLOB                                                                                                     \
    "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
        "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"

// 12 destinations v52..v63 (each its own chain), sources from v40..v51 (read-only)
#define XOR_E32 "v_xor_b32 v52, v40, v52\n v_xor_b32 v53, v41, v53\n v_xor_b32 v54, v42, v54\n v_xor_b32 v55, v43, v55\n" \
                "v_xor_b32 v56, v40, v56\n v_xor_b32 v57, v41, v57\n v_xor_b32 v58, v42, v58\n v_xor_b32 v59, v43, v59\n" \
                "v_xor_b32 v60, v40, v60\n v_xor_b32 v61, v41, v61\n v_xor_b32 v62, v42, v62\n v_xor_b32 v63, v43, v63\n"
#define XOR_E64 "v_xor_b32_e64 v52, v40, v52\n v_xor_b32_e64 v53, v41, v53\n v_xor_b32_e64 v54, v42, v54\n v_xor_b32_e64 v55, v43, v55\n" \
                "v_xor_b32_e64 v56, v40, v56\n v_xor_b32_e64 v57, v41, v57\n v_xor_b32_e64 v58, v42, v58\n v_xor_b32_e64 v59, v43, v59\n" \
                "v_xor_b32_e64 v60, v40, v60\n v_xor_b32_e64 v61, v41, v61\n v_xor_b32_e64 v62, v42, v62\n v_xor_b32_e64 v63, v43, v63\n"
// three sources in three different banks: dst(bank d), srcs from banks d+1, d+2 (v41.. / v42..)
#define B3_DIFF "v_bitop3_b32 v52, v52, v41, v42 bitop3:0x96\n v_bitop3_b32 v53, v53, v42, v43 bitop3:0x96\n" \
                "v_bitop3_b32 v54, v54, v43, v40 bitop3:0x96\n v_bitop3_b32 v55, v55, v40, v41 bitop3:0x96\n" \
                "v_bitop3_b32 v56, v56, v41, v42 bitop3:0x96\n v_bitop3_b32 v57, v57, v42, v43 bitop3:0x96\n" \
                "v_bitop3_b32 v58, v58, v43, v40 bitop3:0x96\n v_bitop3_b32 v59, v59, v40, v41 bitop3:0x96\n" \
                "v_bitop3_b32 v60, v60, v41, v42 bitop3:0x96\n v_bitop3_b32 v61, v61, v42, v43 bitop3:0x96\n" \
                "v_bitop3_b32 v62, v62, v43, v40 bitop3:0x96\n v_bitop3_b32 v63, v63, v40, v41 bitop3:0x96\n"
// three sources in the same bank as the destination (v52 bank 0 with v40, v44)
#define B3_SAME "v_bitop3_b32 v52, v52, v40, v44 bitop3:0x96\n v_bitop3_b32 v53, v53, v41, v45 bitop3:0x96\n" \
                "v_bitop3_b32 v54, v54, v42, v46 bitop3:0x96\n v_bitop3_b32 v55, v55, v43, v47 bitop3:0x96\n" \
                "v_bitop3_b32 v56, v56, v44, v48 bitop3:0x96\n v_bitop3_b32 v57, v57, v45, v49 bitop3:0x96\n" \
                "v_bitop3_b32 v58, v58, v46, v50 bitop3:0x96\n v_bitop3_b32 v59, v59, v47, v51 bitop3:0x96\n" \
                "v_bitop3_b32 v60, v60, v48, v40 bitop3:0x96\n v_bitop3_b32 v61, v61, v49, v41 bitop3:0x96\n" \
                "v_bitop3_b32 v62, v62, v50, v42 bitop3:0x96\n v_bitop3_b32 v63, v63, v51, v43 bitop3:0x96\n"
// two sources only (the third is an inline constant): bitop3 with 2 VGPR reads
#define B3_TWO  "v_bitop3_b32 v52, v52, v41, 0 bitop3:0x96\n v_bitop3_b32 v53, v53, v42, 0 bitop3:0x96\n" \
                "v_bitop3_b32 v54, v54, v43, 0 bitop3:0x96\n v_bitop3_b32 v55, v55, v40, 0 bitop3:0x96\n" \
                "v_bitop3_b32 v56, v56, v41, 0 bitop3:0x96\n v_bitop3_b32 v57, v57, v42, 0 bitop3:0x96\n" \
                "v_bitop3_b32 v58, v58, v43, 0 bitop3:0x96\n v_bitop3_b32 v59, v59, v40, 0 bitop3:0x96\n" \
                "v_bitop3_b32 v60, v60, v41, 0 bitop3:0x96\n v_bitop3_b32 v61, v61, v42, 0 bitop3:0x96\n" \
                "v_bitop3_b32 v62, v62, v43, 0 bitop3:0x96\n v_bitop3_b32 v63, v63, v40, 0 bitop3:0x96\n"
// v_add3_u32 (VOP3, 3 sources, different banks) for comparison
#define XOR3    "v_add3_u32 v52, v52, v41, v42\n v_add3_u32 v53, v53, v42, v43\n v_add3_u32 v54, v54, v43, v40\n" \
                "v_add3_u32 v55, v55, v40, v41\n v_add3_u32 v56, v56, v41, v42\n v_add3_u32 v57, v57, v42, v43\n" \
                "v_add3_u32 v58, v58, v43, v40\n v_add3_u32 v59, v59, v40, v41\n v_add3_u32 v60, v60, v41, v42\n" \
                "v_add3_u32 v61, v61, v42, v43\n v_add3_u32 v62, v62, v43, v40\n v_add3_u32 v63, v63, v40, v41\n"

template <int MODE>
__global__ __launch_bounds__(256) void peak(unsigned* out, int iters) {
    unsigned seed = threadIdx.x * 2654435761u;
    asm volatile(
        "v_mov_b32 v40, %0\n v_add_u32 v41, 1, v40\n v_add_u32 v42, 2, v40\n v_add_u32 v43, 3, v40\n"
        "v_add_u32 v44, 4, v40\n v_add_u32 v45, 5, v40\n v_add_u32 v46, 6, v40\n v_add_u32 v47, 7, v40\n"
        "v_add_u32 v48, 8, v40\n v_add_u32 v49, 9, v40\n v_add_u32 v50, 10, v40\n v_add_u32 v51, 11, v40\n"
        "v_mov_b32 v52, v40\n v_mov_b32 v53, v41\n v_mov_b32 v54, v42\n v_mov_b32 v55, v43\n v_mov_b32 v56, v44\n"
        "v_mov_b32 v57, v45\n v_mov_b32 v58, v46\n v_mov_b32 v59, v47\n v_mov_b32 v60, v48\n v_mov_b32 v61, v49\n"
        "v_mov_b32 v62, v50\n v_mov_b32 v63, v51\n" ::"v"(seed)
        : CLOB);
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) asm volatile(R4(XOR_E32) ::: CLOB);
        if (MODE == 1) asm volatile(R4(XOR_E64) ::: CLOB);
        if (MODE == 2) asm volatile(R4(B3_DIFF) ::: CLOB);
        if (MODE == 3) asm volatile(R4(B3_SAME) ::: CLOB);
        if (MODE == 4) asm volatile(R4(B3_TWO) ::: CLOB);
        if (MODE == 5) asm volatile(R4(XOR3) ::: CLOB);
    }
    unsigned r;
    asm volatile("v_bitop3_b32 %0, v52, v53, v54 bitop3:0x96\n v_bitop3_b32 %0, %0, v55, v56 bitop3:0x96\n"
                 "v_bitop3_b32 %0, %0, v57, v58 bitop3:0x96\n v_bitop3_b32 %0, %0, v59, v60 bitop3:0x96\n"
                 "v_bitop3_b32 %0, %0, v61, v62 bitop3:0x96\n v_xor_b32 %0, %0, v63\n"
                 : "=v"(r)::CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE>
void run(const char* name, int blocks_per_cu, int cus) {
    const int iters = 4000, blocks = cus * blocks_per_cu;
    unsigned* out;
    (void)hipMalloc(&out, sizeof(unsigned) * blocks * 256);
    hipLaunchKernelGGL(peak<MODE>, dim3(blocks), dim3(256), 0, 0, out, 10);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(peak<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double winstr = (double)blocks * 4 * iters * 48;  // wave-instructions
    printf("%-9s waves/SIMD=%d  %.3f wave-instr/SIMD/ns\n", name, blocks_per_cu, winstr / (cus * 4.0) / (best * 1e6));
    (void)hipFree(out);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("CUs=%d max clock=%.2f GHz\n", cus, p.clockRate / 1e6);
    for (int w : {1, 2, 3, 4, 8}) {
        run<0>("xor_e32", w, cus);
        run<1>("xor_e64", w, cus);
        run<2>("b3_diff", w, cus);
        run<3>("b3_same", w, cus);
        run<4>("b3_two", w, cus);
        run<5>("add3", w, cus);
    }
    return 0;
}
