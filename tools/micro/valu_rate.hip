// Throughput of single VALU instruction kinds on gfx950 at full occupancy (8 waves/SIMD,
// every CU busy): 16 independent chains of one instruction per lane, in an unrolled loop.
// Prints wave-instructions per cycle per SIMD relative to v_add_f32 (analysis only; used
// to price the fast walk's integer/bit work against its float work).
// build: hipcc -O3 --offload-arch=gfx950 tools/micro/valu_rate.hip -o build/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS(OP)                                                                                \
    for (int it = 0; it < iters; ++it) {                                                          \
        _Pragma("unroll") for (int c = 0; c < 16; ++c) { OP; }                                    \
    }

template <int K>
__global__ void __launch_bounds__(256) kern(float* out, int iters, float seed) {
    float f[16];
    unsigned u[16];
    for (int c = 0; c < 16; ++c) {
        f[c] = seed + threadIdx.x * 0.001f + c;
        u[c] = threadIdx.x * 2654435761u + c;
    }
    float g = seed * 0.5f;
    unsigned s = (unsigned)seed | 1u;
    if (K == 0) CHAINS(asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 1) CHAINS(asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 2) CHAINS(asm volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 3) CHAINS(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 4) CHAINS(asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 5) CHAINS(asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(u[c])))
    if (K == 6) CHAINS(asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 7) CHAINS(asm volatile("v_bfe_u32 %0, %0, 3, 5" : "+v"(u[c])))
    if (K == 8) CHAINS(asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(u[c]) : "v"(s)))
    if (K == 9) CHAINS(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(s)))
    if (K == 10) CHAINS(asm volatile("v_ffbh_u32 %0, %0" : "+v"(u[c])))
    if (K == 11) CHAINS(asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 12) CHAINS(asm volatile("v_mov_b32 %0, %0" : "+v"(u[c])))
    if (K == 13) CHAINS(asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(double*)&f[c & ~1]) : "v"(*(double*)&f[0])))
    if (K == 14) CHAINS(asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(f[c]), "v"(g) : "vcc"))
    if (K == 15) CHAINS(asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 16) CHAINS(asm volatile("v_sub_f32 %0, %0, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 17) CHAINS(asm volatile("v_min_f32 %0, %0, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 18) CHAINS(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 19) CHAINS(asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 20) CHAINS(asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0xc8" : "+v"(u[c]) : "v"(s)))
    if (K == 21) CHAINS(asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(unsigned long long*)&u[c & ~1])))
    if (K == 22) CHAINS(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 23) CHAINS(asm volatile("v_sqrt_f32 %0, %0" : "+v"(f[c])))
    if (K == 24) CHAINS(asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(f[c]) : "v"(u[c])))
    if (K == 25) {  // cndmask on a mask that v_cmp wrote once before the loop
        asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(f[0]), "v"(g) : "vcc");
        CHAINS(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(s)))
    }
    if (K == 26) {  // e64 form, mask in an SGPR pair
        unsigned long long m = 0x5555555555555555ull;
        asm volatile("" : "+s"(m));
        CHAINS(asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[c]) : "v"(s), "s"(m)))
    }
    if (K == 27)  // v_cmp writing an SGPR pair + cndmask reading it: the compiler's select idiom
        CHAINS(asm volatile("v_cmp_lt_f32_e64 s[60:61], %1, %2\n\ts_nop 1\n\tv_cndmask_b32_e64 %0, %0, %3, s[60:61]"
                            : "+v"(u[c]) : "v"(f[c]), "v"(g), "v"(s) : "s60", "s61"))
    if (K == 28) CHAINS(asm volatile("v_max_f32 %0, %0, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 29) CHAINS(asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 30) CHAINS(asm volatile("v_or_b32 %0, %0, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 31) CHAINS(asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(u[c])))
    if (K == 32) CHAINS(asm volatile("v_sub_u32 %0, %0, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 33) CHAINS(asm volatile("v_cmp_lt_u32 vcc, %0, %1" : : "v"(u[c]), "v"(s) : "vcc"))
    if (K == 34) CHAINS(asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(f[c]) : "v"(g)))
    if (K == 35) CHAINS(asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(u[c]) : "v"(s)))
    if (K == 37)
        CHAINS(asm volatile("v_cmp_lt_f32 vcc, %1, %2\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %3, vcc"
                            : "+v"(u[c]) : "v"(f[c]), "v"(g), "v"(s) : "vcc"))
    if (K == 38) {
        asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(f[0]), "v"(g) : "vcc");
        CHAINS(asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(s)))
    }
    if (K == 39) {  // e32 cndmask, vcc written by s_mov (SALU) before the loop
        asm volatile("s_mov_b64 vcc, -1" : : : "vcc");
        CHAINS(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(s)))
    }
    if (K == 40) CHAINS(asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(u[c]) : "v"(s) : "vcc"))
    if (K == 41) CHAINS(asm volatile("v_max_f32 %0, %0, %1" : "+v"(f[c]) : "s"(g)))
    if (K == 42) CHAINS(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "s"(g)))
    if (K == 36) CHAINS(asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "s"(g)))
    float acc = 0.0f;
    for (int c = 0; c < 16; ++c) acc += f[c] + (float)u[c];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static const char* names[] = {"v_add_f32", "v_mul_f32", "v_max3_f32", "v_fma_f32", "v_add_u32", "v_lshlrev_b32",
                              "v_and_b32", "v_bfe_u32", "v_alignbit_b32", "v_cndmask_b32", "v_ffbh_u32",
                              "v_lshl_add_u32", "v_mov_b32", "v_pk_add_f32", "v_cmp_lt_f32", "v_mul_u32_u24",
                              "v_sub_f32", "v_min_f32", "v_xor_b32", "v_add3_u32", "v_bitop3_b32",
                              "v_lshlrev_b64", "v_mul_lo_u32", "v_sqrt_f32", "v_cvt_f32_u32", "cndmask(vcc set)",
                              "cndmask_e64 sgpr", "cmp+nop1+cndmask", "v_max_f32", "v_med3_f32", "v_or_b32",
                              "v_lshrrev_b32", "v_sub_u32", "v_cmp_lt_u32", "v_fmac_f32", "v_and_or_b32",
                              "v_add_f32 sgpr", "cmp vcc+nop+cndmask32", "cndmask_e64 vcc",
                              "cndmask32 vcc=s_mov", "v_add_co_u32", "v_max_f32 sgpr", "v_fma_f32 sgpr"};
typedef void (*KF)(float*, int, float);
static KF kfs[] = {kern<0>, kern<1>, kern<2>, kern<3>, kern<4>, kern<5>, kern<6>, kern<7>, kern<8>,
                   kern<9>, kern<10>, kern<11>, kern<12>, kern<13>, kern<14>, kern<15>, kern<16>,
                   kern<17>, kern<18>, kern<19>, kern<20>, kern<21>, kern<22>, kern<23>, kern<24>,
                   kern<25>, kern<26>, kern<27>, kern<28>, kern<29>, kern<30>, kern<31>, kern<32>, kern<33>,
                   kern<34>, kern<35>, kern<36>, kern<37>, kern<38>, kern<39>, kern<40>, kern<41>, kern<42>};

int main() {
    const int blocks = 256 * 8 * 4, iters = 2000;  // 8 WGs of 4 waves per CU = 8 waves/SIMD, x4 rounds
    float* out;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    double base = 0.0;
    for (int k = 0; k < 43; ++k) {
        hipLaunchKernelGGL(kfs[k], dim3(blocks), dim3(256), 0, 0, out, 10, 1.0f);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(kfs[k], dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double winst = (double)blocks * 4 * iters * 16;  // wave-instructions
        const double per_simd_ns = ms * 1e6 / (winst / 1024.0);  // ns per wave-instruction per SIMD
        if (k == 0) base = per_simd_ns;
        printf("%-16s %8.3f ms  %.3f ns/wave-instr/SIMD  (%.2fx v_add_f32)\n", names[k], ms, per_simd_ns,
               per_simd_ns / base);
    }
    return 0;
}
