// Latency and throughput of secp256k1 field multiplication variants on one gfx950 GPU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fe_lat.hip -o bin/fe_lat && bin/fe_lat
// Each lane runs a chain of ITERS dependent products x = x * y (or x = x^2). "lone" launches one
// wave (the latency a small ECDSA batch sees), "full" 16 waves per CU (throughput). Variants:
//   fe8   the verify kernel's 8 x 32-bit Comba product (v_mad_u64_u32 + VCC carry word)
//   fe10  10 x 26-bit limbs, 64-bit column sums without carries, reduction by partial carries
// Primitive rows time dependent chains of one instruction in one wave (cycles via s_memtime).
// Results are checked: both variants must agree on every lane's final canonical value.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                        \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

constexpr int ITERS = 4096;

// ------------------------------------------------------------------ 8 x 32 (verify kernel copy)
struct fe8 {
    uint32_t v[8];
};
__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t ci, uint32_t* co) {
    return __builtin_addc(a, b, ci, co);
}
__device__ __forceinline__ void fe8_fold(fe8& r, uint64_t c) {
    while (c) {
        uint32_t co;
        const uint64_t lo = c * 977u;
        const uint64_t mid = (lo >> 32) + (uint32_t)c;
        r.v[0] = addc(r.v[0], (uint32_t)lo, 0, &co);
        r.v[1] = addc(r.v[1], (uint32_t)mid, co, &co);
        r.v[2] = addc(r.v[2], (uint32_t)(mid >> 32) + (uint32_t)(c >> 32), co, &co);
#pragma unroll
        for (int i = 3; i < 8; i++) r.v[i] = addc(r.v[i], 0, co, &co);
        c = co;
    }
}
__device__ __forceinline__ void fe8_mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(c2)
        : "v"(a), "v"(b)
        : "vcc");
}
__device__ __forceinline__ void fe8_reduce512(fe8& r, const uint32_t (&t)[16]) {
    uint32_t u[8], c = 0;
    u[0] = t[0];
#pragma unroll
    for (int i = 1; i < 8; i++) u[i] = addc(t[i], t[7 + i], c, &c);
    const uint64_t u8 = (uint64_t)t[15] + c;
    uint32_t cc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t p = (uint64_t)t[8 + i] * 977u + cc;
        uint32_t co;
        r.v[i] = addc(u[i], (uint32_t)p, 0, &co);
        cc = (uint32_t)(p >> 32) + co;
    }
    fe8_fold(r, u8 + cc);
}
__device__ __forceinline__ void fe8_mul(fe8& r, const fe8& a, const fe8& b) {
    uint32_t t[16];
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 0; k < 15; k++) {
#pragma unroll
        for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) fe8_mac(acc, c2, a.v[i], b.v[k - i]);
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)c2 << 32);
        c2 = 0;
    }
    t[15] = (uint32_t)acc;
    fe8_reduce512(r, t);
}
__device__ __forceinline__ void fe8_sqr(fe8& r, const fe8& a) {
    uint32_t t[16];
    t[0] = 0;
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 1; k < 14; k++) {
#pragma unroll
        for (int i = (k > 7 ? k - 7 : 0); 2 * i < k; i++) fe8_mac(acc, c2, a.v[i], a.v[k - i]);
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)c2 << 32);
        c2 = 0;
    }
    t[14] = (uint32_t)acc;
    t[15] = t[14] >> 31;
#pragma unroll
    for (int i = 14; i > 0; i--) t[i] = __builtin_amdgcn_alignbit(t[i], t[i - 1], 31);
    t[0] = 0;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t sq = (uint64_t)a.v[i] * a.v[i];
        t[2 * i] = addc(t[2 * i], (uint32_t)sq, c, &c);
        t[2 * i + 1] = addc(t[2 * i + 1], (uint32_t)(sq >> 32), c, &c);
    }
    fe8_reduce512(r, t);
}
__device__ __noinline__ fe8 fe8_mul_v(fe8 a, fe8 b) {
    fe8 r;
    fe8_mul(r, a, b);
    return r;
}
__device__ __noinline__ fe8 fe8_sqr_v(fe8 a) {
    fe8 r;
    fe8_sqr(r, a);
    return r;
}

// ------------------------------------------------------------------ 10 x 26
// value = sum n[i] 2^(26 i). Products take limbs below 2^27.3 (every column sum then stays
// below 2^58, so each column's carry word t >> 26 fits 32 bits) and return limbs below 2^26.1.
struct fe10 {
    uint32_t n[10];
};
constexpr uint32_t M26 = 0x3FFFFFFu;
constexpr uint32_t R0 = 0x3D10u; // 2^260 = 2^36 + 0x3D10 (mod p): weight 2^260 -> 0x3D10 at limb 0, 2^10 at limb 1

__device__ __forceinline__ uint32_t lo26(uint64_t t) { return (uint32_t)t & M26; }
__device__ __forceinline__ uint32_t hi26(uint64_t t) { return __builtin_amdgcn_alignbit((uint32_t)(t >> 32), (uint32_t)t, 26); }

// t[0..18] column sums -> r (limbs < 2^26.1)
__device__ __forceinline__ void fe10_reduce(fe10& r, uint64_t (&t)[19]) {
    // high columns 10..18 as 26-bit limbs plus the carry of the column below (one partial carry)
    uint32_t u[10]; // weight 2^(26 (10 + i))
    u[0] = lo26(t[10]);
#pragma unroll
    for (int k = 11; k < 19; k++) u[k - 10] = lo26(t[k]) + hi26(t[k - 1]);
    u[9] = hi26(t[18]);
    // fold: weight 2^(260 + 26 i) -> 0x3D10 at column i, 2^10 at column i + 1
#pragma unroll
    for (int i = 0; i < 9; i++) {
        t[i] += (uint64_t)u[i] * R0;
        t[i + 1] += (uint64_t)u[i] << 10;
    }
    t[9] += (uint64_t)u[9] * R0;
    // u[9] << 10 lands on column 10 again: 2^10 u9 -> 0x3D10 * 2^10 u9 at 0, 2^20 u9 at 1
    t[0] += ((uint64_t)u[9] << 10) * R0;
    t[1] += (uint64_t)u[9] << 20;
    // partial carry pass 1 (every limb at once): limbs < 2^32.
    uint32_t w[10];
    w[0] = lo26(t[0]);
#pragma unroll
    for (int k = 1; k < 10; k++) w[k] = lo26(t[k]) + hi26(t[k - 1]);
    const uint32_t h9 = hi26(t[9]); // weight 2^260
    uint64_t w0 = (uint64_t)w[0] + (uint64_t)h9 * R0;
    uint64_t w1 = (uint64_t)w[1] + ((uint64_t)h9 << 10);
    // pass 2: limbs < 2^26 + 2^20
    r.n[0] = lo26(w0);
    r.n[1] = lo26(w1) + hi26(w0);
    r.n[2] = (w[2] & M26) + (uint32_t)(w1 >> 26);
#pragma unroll
    for (int k = 3; k < 10; k++) r.n[k] = (w[k] & M26) + (w[k - 1] >> 26);
    const uint32_t c9 = w[9] >> 26;
    r.n[0] += c9 * R0;
    r.n[1] += c9 << 10;
}
__device__ __forceinline__ void fe10_mul(fe10& r, const fe10& a, const fe10& b) {
    uint64_t t[19];
#pragma unroll
    for (int k = 0; k < 19; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++)
#pragma unroll
        for (int j = 0; j < 10; j++) t[i + j] += (uint64_t)a.n[i] * b.n[j];
    fe10_reduce(r, t);
}
__device__ __forceinline__ void fe10_sqr(fe10& r, const fe10& a) {
    uint64_t t[19];
    uint32_t d[10];
#pragma unroll
    for (int i = 0; i < 10; i++) d[i] = a.n[i] << 1;
#pragma unroll
    for (int k = 0; k < 19; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        t[2 * i] += (uint64_t)a.n[i] * a.n[i];
#pragma unroll
        for (int j = i + 1; j < 10; j++) t[i + j] += (uint64_t)a.n[i] * d[j];
    }
    fe10_reduce(r, t);
}

// ------------------------------------------------------------------ conversions (not timed)
__device__ void fe8_canon(fe8& a) { // < 2^256 -> < p
    const uint32_t P[8] = {0xFFFFFC2F, 0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF};
    uint32_t t[8];
    uint64_t br = 0;
    for (int i = 0; i < 8; i++) {
        const uint64_t d = (uint64_t)a.v[i] - P[i] - br;
        t[i] = (uint32_t)d;
        br = (d >> 63) & 1;
    }
    if (!br)
        for (int i = 0; i < 8; i++) a.v[i] = t[i];
}
__device__ fe8 fe10_to8(const fe10& a) {
    // exact integer sum n_i 2^(26 i) (< 2^261), folded back below 2^256, then canonical
    uint32_t w[9] = {0};
    for (int i = 0; i < 10; i++) {
        const int bit = 26 * i, q = bit / 32, s = bit % 32;
        uint64_t add = (uint64_t)a.n[i] << s;
        uint64_t c = 0;
        for (int k = q; k < 9; k++) {
            c += (uint64_t)w[k] + (k == q ? (uint32_t)add : k == q + 1 ? (uint32_t)(add >> 32) : 0u);
            w[k] = (uint32_t)c;
            c >>= 32;
        }
    }
    fe8 r;
    for (int i = 0; i < 8; i++) r.v[i] = w[i];
    fe8_fold(r, w[8]);
    fe8_canon(r);
    return r;
}
__device__ fe10 fe8_to10(const fe8& a) {
    fe10 r;
    for (int i = 0; i < 10; i++) {
        const int bit = 26 * i, q = bit / 32, s = bit % 32;
        uint64_t x = a.v[q];
        if (q + 1 < 8) x |= (uint64_t)a.v[q + 1] << 32;
        r.n[i] = (uint32_t)(x >> s) & M26;
    }
    return r;
}

// ------------------------------------------------------------------ kernels
// MODE 0: fe8 mul chain, 1: fe8 sqr chain, 2: fe10 mul chain, 3: fe10 sqr chain
template <int MODE>
__global__ __launch_bounds__(64) void chain(const uint32_t* in, uint32_t* out, unsigned long long* cyc, int iters) {
    const int g = blockIdx.x * 64 + threadIdx.x;
    fe8 x, y;
    for (int i = 0; i < 8; i++) {
        x.v[i] = in[(g % 4096) * 16 + i];
        y.v[i] = in[(g % 4096) * 16 + 8 + i];
    }
    fe8_canon(x);
    fe8_canon(y);
    const unsigned long long t0 = __builtin_readcyclecounter();
    if constexpr (MODE == 0) {
        for (int it = 0; it < iters; it++) x = fe8_mul_v(x, y);
    } else if constexpr (MODE == 1) {
        for (int it = 0; it < iters; it++) x = fe8_sqr_v(x);
    } else {
        fe10 a = fe8_to10(x), b = fe8_to10(y);
        const unsigned long long t1 = __builtin_readcyclecounter();
        for (int it = 0; it < iters; it++) {
            if constexpr (MODE == 2) fe10_mul(a, a, b);
            else fe10_sqr(a, a);
        }
        const unsigned long long t2 = __builtin_readcyclecounter();
        x = fe10_to8(a);
        if (threadIdx.x == 0) cyc[blockIdx.x] = t2 - t1;
        for (int i = 0; i < 8; i++) out[g * 8 + i] = x.v[i];
        return;
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    fe8_canon(x);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    for (int i = 0; i < 8; i++) out[g * 8 + i] = x.v[i];
}

// primitive dependent chains, 16 instructions per block
#define R16(s) s s s s s s s s s s s s s s s s
template <int P>
__global__ __launch_bounds__(64) void prim(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
    uint64_t a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7;
    uint32_t x = (uint32_t)a, k = seed ^ 0x1234567u;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 256; it++) {
        if constexpr (P == 0) asm volatile(R16("v_mad_u64_u32 %0, vcc, %1, %1, %0\n\t") : "+v"(a) : "v"(k) : "vcc");
        if constexpr (P == 1)
            asm volatile(R16("v_mad_u64_u32 %0, vcc, %4, %4, %0\n\tv_mad_u64_u32 %1, vcc, %4, %4, %1\n\t"
                             "v_mad_u64_u32 %2, vcc, %4, %4, %2\n\tv_mad_u64_u32 %3, vcc, %4, %4, %3\n\t")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
                         : "v"(k)
                         : "vcc");
        if constexpr (P == 2) asm volatile(R16("v_add_u32 %0, %0, %1\n\t") : "+v"(x) : "v"(k));
        if constexpr (P == 3) asm volatile(R16("v_alignbit_b32 %0, %0, %1, 7\n\t") : "+v"(x) : "v"(k));
        if constexpr (P == 4) asm volatile(R16("v_lshl_add_u64 %0, %0, 0, %1\n\t") : "+v"(a) : "v"(b));
        if constexpr (P == 5) asm volatile(R16("v_add_co_u32 %0, vcc, %0, %1\n\ts_nop 1\n\t") : "+v"(x) : "v"(k) : "vcc");
        if constexpr (P == 6) asm volatile(R16("v_mul_lo_u32 %0, %0, %1\n\t") : "+v"(x) : "v"(k));
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    out[threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d) ^ x;
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    const int nfull = ncu * 16; // waves
    std::vector<uint32_t> h(4096 * 16);
    uint64_t s = 88172645463325252ull;
    for (auto& w : h) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        w = (uint32_t)s;
    }
    uint32_t *din, *dout;
    unsigned long long* dcyc;
    CK(hipMalloc(&din, h.size() * 4));
    CK(hipMalloc(&dout, (size_t)nfull * 64 * 8 * 4));
    CK(hipMalloc(&dcyc, (size_t)nfull * 8));
    CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* pn[] = {"v_mad_u64_u32 dep", "v_mad_u64_u32 4 chains", "v_add_u32 dep", "v_alignbit_b32 dep",
                        "v_lshl_add_u64 dep", "v_add_co_u32 + s_nop 1 dep", "v_mul_lo_u32 dep"};
    void (*pk[])(uint32_t*, unsigned long long*, uint32_t) = {prim<0>, prim<1>, prim<2>, prim<3>, prim<4>, prim<5>, prim<6>};
    for (int p = 0; p < 7; p++) {
        hipLaunchKernelGGL(pk[p], dim3(1), dim3(64), 0, 0, dout, dcyc, 1u);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(pk[p], dim3(1), dim3(64), 0, 0, dout, dcyc, 3u);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        unsigned long long c = 0;
        CK(hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost));
        const int ninst = 256 * 16 * (p == 1 ? 4 : 1);
        printf("{\"prim\": \"%s\", \"memtime_per_inst\": %.2f}\n", pn[p], (double)c / ninst);
    }
    const char* mn[] = {"fe8_mul", "fe8_sqr", "fe10_mul", "fe10_sqr"};
    void (*mk[])(const uint32_t*, uint32_t*, unsigned long long*, int) = {chain<0>, chain<1>, chain<2>, chain<3>};
    std::vector<uint32_t> ref[2], got(64 * 8);
    for (int m = 0; m < 4; m++) {
        for (int full = 0; full < 2; full++) {
            const int blocks = full ? nfull : 1;
            hipLaunchKernelGGL(mk[m], dim3(blocks), dim3(64), 0, 0, din, dout, dcyc, 16);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(mk[m], dim3(blocks), dim3(64), 0, 0, din, dout, dcyc, ITERS);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            unsigned long long c = 0;
            CK(hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost));
            const double ops = (double)blocks * 64 * ITERS;
            printf("{\"op\": \"%s\", \"waves\": %d, \"ms\": %.3f, \"ns_per_op_lane0\": %.1f, \"memtime_per_op_wave0\": %.1f, "
                   "\"Gop_per_s\": %.2f}\n",
                   mn[m], blocks, ms, ms * 1e6 / ITERS, (double)c / ITERS, ops / (ms * 1e-3) / 1e9);
            if (!full) {
                CK(hipMemcpy(got.data(), dout, 64 * 8 * 4, hipMemcpyDeviceToHost));
                if (m < 2) {
                    ref[m] = got;
                } else if (memcmp(ref[m - 2].data(), got.data(), got.size() * 4) != 0) {
                    printf("MISMATCH %s vs %s\n", mn[m], mn[m - 2]);
                    return 2;
                }
            }
        }
    }
    printf("fe10 results match fe8 on all 64 lanes\n");
    return 0;
}
