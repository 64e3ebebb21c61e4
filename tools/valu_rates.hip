// Issue rate of the VALU instructions BLAKE2b is made of, on one gfx950 GPU: each lane runs
// 8 independent chains of one instruction (inline asm blocks of 8, so compiler hazards land
// once per block), enough waves to fill every SIMD. Prints cycles per wave instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O2 tools/valu_rates.hip -o bin/valu_rates && bin/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

constexpr int ITERS = 2048;

#define OP8(fmt)                                                                              \
    asm volatile(fmt(0) fmt(1) fmt(2) fmt(3) fmt(4) fmt(5) fmt(6) fmt(7)                    \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),  \
                   "+v"(a[6]), "+v"(a[7])                                                    \
                 : "v"(k)                                                                    \
                 : "vcc")

#define F_XOR(i) "v_xor_b32 %" #i ", %" #i ", %8\n\t"
#define F_ALIGN(i) "v_alignbit_b32 %" #i ", %" #i ", %8, 7\n\t"
#define F_ADD(i) "v_add_u32 %" #i ", %" #i ", %8\n\t"
#define F_SDWA(i) "v_xor_b32_sdwa %" #i ", %" #i ", %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n\t"
#define F_PERM(i) "v_perm_b32 %" #i ", %" #i ", %8, %8\n\t"
#define F_LSHR(i) "v_lshrrev_b32 %" #i ", 7, %" #i "\n\t"
#define F_MULLO(i) "v_mul_lo_u32 %" #i ", %" #i ", %8\n\t"
#define F_MULHI(i) "v_mul_hi_u32 %" #i ", %" #i ", %8\n\t"
#define F_MAD24(i) "v_mad_u32_u24 %" #i ", %" #i ", %8, %8\n\t"
#define F_MULHI24(i) "v_mul_hi_u32_u24 %" #i ", %" #i ", %8\n\t"
#define F_XOR3(i) "v_lshl_or_b32 %" #i ", %" #i ", 3, %8\n\t"

template <int OP> __global__ void bench(unsigned* out, unsigned seed) {
    unsigned a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
    unsigned k = seed ^ threadIdx.x;
    unsigned long long b[4];
    for (int i = 0; i < 4; ++i) b[i] = ((unsigned long long)a[2 * i] << 32) | a[2 * i + 1];
    unsigned long long kk = ((unsigned long long)k << 32) | k;
    for (int it = 0; it < ITERS; ++it) {
        if constexpr (OP == 0) OP8(F_XOR);
        if constexpr (OP == 1) OP8(F_ALIGN);
        if constexpr (OP == 2) OP8(F_ADD);
        if constexpr (OP == 5) OP8(F_SDWA);
        if constexpr (OP == 6) OP8(F_PERM);
        if constexpr (OP == 7) OP8(F_LSHR);
        if constexpr (OP == 8) OP8(F_XOR3);
        if constexpr (OP == 9) OP8(F_MULLO);
        if constexpr (OP == 10) OP8(F_MULHI);
        if constexpr (OP == 11) OP8(F_MAD24);
        if constexpr (OP == 12) OP8(F_MULHI24);
        if constexpr (OP == 13) { // 8 x v_mad_u64_u32 on 4 chains
            asm volatile(
                "v_mad_u64_u32 %0, vcc, %5, %4, %0\n\tv_mad_u64_u32 %1, vcc, %5, %4, %1\n\t"
                "v_mad_u64_u32 %2, vcc, %5, %4, %2\n\tv_mad_u64_u32 %3, vcc, %5, %4, %3\n\t"
                "v_mad_u64_u32 %0, vcc, %5, %4, %0\n\tv_mad_u64_u32 %1, vcc, %5, %4, %1\n\t"
                "v_mad_u64_u32 %2, vcc, %5, %4, %2\n\tv_mad_u64_u32 %3, vcc, %5, %4, %3\n\t"
                : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])
                : "v"(k), "v"(k ^ 5u)
                : "vcc");
        }
        if constexpr (OP == 14) { // 8 x v_fma_f64 on 4 chains
            double* d = reinterpret_cast<double*>(b);
            const double kd = (double)k;
            asm volatile(
                "v_fma_f64 %0, %0, %4, %4\n\tv_fma_f64 %1, %1, %4, %4\n\t"
                "v_fma_f64 %2, %2, %4, %4\n\tv_fma_f64 %3, %3, %4, %4\n\t"
                "v_fma_f64 %0, %0, %4, %4\n\tv_fma_f64 %1, %1, %4, %4\n\t"
                "v_fma_f64 %2, %2, %4, %4\n\tv_fma_f64 %3, %3, %4, %4\n\t"
                : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3])
                : "v"(kd));
        }
        if constexpr (OP == 3) { // 8 x v_lshl_add_u64 (64-bit add) on 4 chains, twice
            asm volatile(
                "v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\t"
                "v_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4\n\t"
                "v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\t"
                "v_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4\n\t"
                : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])
                : "v"(kk));
        }
        if constexpr (OP == 4) { // 4 x (v_add_co + v_addc) = 8 instructions, 4 64-bit adds
            unsigned* p = a;
            asm volatile(
                "v_add_co_u32 %0, vcc, %0, %8\n\tv_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
                "v_add_co_u32 %2, vcc, %2, %8\n\tv_addc_co_u32 %3, vcc, %3, %8, vcc\n\t"
                "v_add_co_u32 %4, vcc, %4, %8\n\tv_addc_co_u32 %5, vcc, %5, %8, vcc\n\t"
                "v_add_co_u32 %6, vcc, %6, %8\n\tv_addc_co_u32 %7, vcc, %7, %8, vcc\n\t"
                : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]), "+v"(p[7])
                : "v"(k)
                : "vcc");
        }
    }
    unsigned r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    for (int i = 0; i < 4; ++i) r ^= (unsigned)b[i] ^ (unsigned)(b[i] >> 32);
    if (r == 0x12345678u) out[blockIdx.x] = r;
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    const double clk_hz = prop.clockRate * 1e3;
    unsigned* out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"v_xor_b32",    "v_alignbit_b32", "v_add_u32",     "v_lshl_add_u64", "v_add_co+v_addc (pair)",
                           "v_xor_b32_sdwa", "v_perm_b32",   "v_lshrrev_b32", "v_lshl_or_b32",
                           "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24", "v_mul_hi_u32_u24",
                           "v_mad_u64_u32", "v_fma_f64"};
    void (*ks[])(unsigned*, unsigned) = {bench<0>, bench<1>, bench<2>, bench<3>, bench<4>,
                                         bench<5>, bench<6>, bench<7>, bench<8>, bench<9>,
                                         bench<10>, bench<11>, bench<12>, bench<13>, bench<14>};
    for (int waves_per_simd = 1; waves_per_simd <= 8; waves_per_simd *= 2) {
        const int blocks = ncu * 4 * waves_per_simd, threads = 64;
        for (int op = 0; op < 15; ++op) {
            auto k = ks[op];
            hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1u);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 3u);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            // instructions per wave: ITERS * 8; waves per SIMD: waves_per_simd
            const double insts = (double)ITERS * 8 * waves_per_simd;
            const double cyc = ms * 1e-3 * clk_hz;
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"cycles_per_wave_inst\": %.2f}\n",
                   names[op], waves_per_simd, ms, cyc / insts);
        }
    }
    return 0;
}
