// secp256k1 field arithmetic in 10 x 26-bit limbs for the latency-bound ECDSA path (gfx950).
//
// Why a second representation next to the 8 x 32-bit one of the throughput kernel
// (secp256k1.hip fe_mul_impl): a 26-bit limb product fits a 64-bit column sum without carries,
// so a multiplication is 100 independent-per-column v_mad_u64_u32 followed by a reduction of
// partial carries that every limb does at once. Additions, negations and small multiples are
// limb-wise 32-bit adds with no carry chain at all. The 8 x 32 product is one serial chain of
// multiply-adds whose every carry read costs two wait states on gfx950 (s_nop 1); with one wave
// per SIMD (small batches) nothing hides that. Same role as the reference's 10x26 field
// (src/secp256k1/src/field_10x26_impl.h), with a reduction shaped for ILP instead of a serial
// carry accumulator.
//
// Magnitudes (m): every limb is at most m * 2^26 (the top limb, 22 bits when canonical, at most
// m * 2^22 + 2^7). Products and f10_norm return m <= 1.032 ("M1"). A product's inputs must
// satisfy m_a * m_b <= 6.3: its column sums then stay below 2^58, so each column's carry word
// (t >> 26) fits 32 bits. f10_neg(a, c) is c * p - a and needs c >= m_a + 0.001 limb-wise.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace bcp {
namespace gpu {
namespace f10 {

struct fe {
    uint32_t n[10];
};

constexpr uint32_t M26 = 0x3FFFFFFu;
constexpr uint32_t M22 = 0x3FFFFFu;
// p = 2^256 - 2^32 - 977 in 26-bit limbs
constexpr uint32_t P0 = 0x3FFFC2Fu, P1 = 0x3FFFFBFu, PM = 0x3FFFFFFu, P9 = 0x3FFFFFu;
constexpr uint32_t R260 = 0x3D10u; // 2^260 = 2^36 + 0x3D10 (mod p): weight 2^260 -> 0x3D10 at limb 0, 2^10 at limb 1

__device__ __forceinline__ uint32_t lo26(uint64_t t) { return (uint32_t)t & M26; }
// bits 26..57 of t (t < 2^58)
__device__ __forceinline__ uint32_t hi26(uint64_t t) {
    return __builtin_amdgcn_alignbit((uint32_t)(t >> 32), (uint32_t)t, 26);
}

__device__ __forceinline__ void set_int(fe& r, uint32_t v) {
#pragma unroll
    for (int i = 0; i < 10; i++) r.n[i] = i == 0 ? v : 0u;
}

// t[0..18] column sums (each < 2^58) -> r, M1
__device__ __forceinline__ void reduce(fe& r, uint64_t (&t)[19]) {
    // columns 10..18 as 26-bit digits plus the carry word of the column below: weight 2^(260 + 26 i)
    uint32_t u[10];
    u[0] = lo26(t[10]);
#pragma unroll
    for (int k = 11; k < 19; k++) u[k - 10] = lo26(t[k]) + hi26(t[k - 1]);
    u[9] = hi26(t[18]);
    // fold: 2^(260 + 26 i) -> 0x3D10 at column i, 2^10 at column i + 1
#pragma unroll
    for (int i = 0; i < 9; i++) {
        t[i] += (uint64_t)u[i] * R260;
        t[i + 1] += (uint64_t)u[i] << 10;
    }
    t[9] += (uint64_t)u[9] * R260;
    t[0] += ((uint64_t)u[9] << 10) * R260; // u9 << 10 sits at column 10 again
    t[1] += (uint64_t)u[9] << 20;
    // partial carry, every column at once: w < 2^32 (w0, w1 64-bit after the top carry)
    uint32_t w[10];
    w[0] = lo26(t[0]);
#pragma unroll
    for (int k = 1; k < 10; k++) w[k] = lo26(t[k]) + hi26(t[k - 1]);
    const uint32_t h9 = hi26(t[9]); // weight 2^260
    const uint64_t w0 = (uint64_t)w[0] + (uint64_t)h9 * R260;
    const uint64_t w1 = (uint64_t)w[1] + ((uint64_t)h9 << 10);
    // second partial carry; the top limb keeps 22 bits (2^256 = 2^32 + 977: 977 at limb 0, 64 at limb 1)
    const uint32_t c9 = w[9] >> 22;
    r.n[0] = lo26(w0) + c9 * 977u;
    r.n[1] = lo26(w1) + hi26(w0) + (c9 << 6);
    r.n[2] = (w[2] & M26) + (uint32_t)(w1 >> 26);
#pragma unroll
    for (int k = 3; k < 9; k++) r.n[k] = (w[k] & M26) + (w[k - 1] >> 26);
    r.n[9] = (w[9] & M22) + (w[8] >> 26);
}

__device__ __forceinline__ void mul(fe& r, const fe& a, const fe& b) {
    uint64_t t[19];
#pragma unroll
    for (int k = 0; k < 19; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++)
#pragma unroll
        for (int j = 0; j < 10; j++) t[i + j] += (uint64_t)a.n[i] * b.n[j];
    reduce(r, t);
}

__device__ __forceinline__ void sqr(fe& r, const fe& a) {
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
    reduce(r, t);
}

// one partial carry over every limb (limbs < 2^32 in, M1 out)
__device__ __forceinline__ void norm(fe& r) {
    uint32_t h[10];
#pragma unroll
    for (int k = 0; k < 9; k++) h[k] = r.n[k] >> 26;
    h[9] = r.n[9] >> 22;
    r.n[0] = (r.n[0] & M26) + h[9] * 977u;
    r.n[1] = (r.n[1] & M26) + h[0] + (h[9] << 6);
#pragma unroll
    for (int k = 2; k < 9; k++) r.n[k] = (r.n[k] & M26) + h[k - 1];
    r.n[9] = (r.n[9] & M22) + h[8];
}

__device__ __forceinline__ void add(fe& r, const fe& a, const fe& b) {
#pragma unroll
    for (int k = 0; k < 10; k++) r.n[k] = a.n[k] + b.n[k];
}
// r = c * p - a (c >= magnitude of a)
__device__ __forceinline__ void neg(fe& r, const fe& a, uint32_t c) {
    r.n[0] = c * P0 - a.n[0];
    r.n[1] = c * P1 - a.n[1];
#pragma unroll
    for (int k = 2; k < 9; k++) r.n[k] = c * PM - a.n[k];
    r.n[9] = c * P9 - a.n[9];
}
// r = a + c * p - b (c >= magnitude of b)
__device__ __forceinline__ void sub(fe& r, const fe& a, const fe& b, uint32_t c) {
    r.n[0] = a.n[0] + (c * P0 - b.n[0]);
    r.n[1] = a.n[1] + (c * P1 - b.n[1]);
#pragma unroll
    for (int k = 2; k < 9; k++) r.n[k] = a.n[k] + (c * PM - b.n[k]);
    r.n[9] = a.n[9] + (c * P9 - b.n[9]);
}
__device__ __forceinline__ void mul_int(fe& r, const fe& a, uint32_t m) {
#pragma unroll
    for (int k = 0; k < 10; k++) r.n[k] = a.n[k] * m;
}

// Canonical value (< p) of an M1 value, as digits with the top one at most 22 bits.
__device__ __forceinline__ void normalize(fe& r) {
    norm(r);
    // exact carry propagation (serial), then one conditional subtraction of p
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        const uint32_t v = r.n[k] + c;
        r.n[k] = v & M26;
        c = v >> 26;
    }
    r.n[9] += c;
    // value < 2^256 + 2^241: >= p iff the top carries or every digit equals p's
    uint32_t top = r.n[9] >> 22;
    uint32_t all = r.n[2] & r.n[3] & r.n[4] & r.n[5] & r.n[6] & r.n[7] & r.n[8];
    const bool ge = top != 0 || (r.n[9] == P9 && all == M26 && (r.n[1] + 64u + ((r.n[0] + 977u) >> 26)) > M26);
    if (ge) { // subtract p = add 2^32 + 977 and drop 2^256
        c = 977u;
        uint32_t v = r.n[0] + c;
        r.n[0] = v & M26;
        c = (v >> 26) + 64u;
#pragma unroll
        for (int k = 1; k < 9; k++) {
            v = r.n[k] + c;
            r.n[k] = v & M26;
            c = v >> 26;
        }
        r.n[9] = (r.n[9] + c) & M22;
    }
}

// a == 0 (mod p) for an M1 value (< 2p, so 0 or p). The lowest digit of the value is exactly
// n0 mod 2^26: anything but 0 or p's digit rules zero out without carrying.
__device__ __forceinline__ bool maybe_zero(const fe& a) {
    const uint32_t d0 = a.n[0] & M26;
    return d0 == 0u || d0 == P0;
}
__device__ __forceinline__ bool is_zero(const fe& a) {
    if (!maybe_zero(a)) return false;
    fe t = a;
    normalize(t);
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 10; k++) o |= t.n[k];
    return o == 0;
}

// from 8 little-endian 32-bit words (any value < 2^256)
__device__ __forceinline__ void from_words(fe& r, const uint32_t (&w)[8]) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const int bit = 26 * i, q = bit / 32, s = bit % 32;
        const uint32_t lo = w[q];
        const uint32_t hi = q + 1 < 8 ? w[q + 1] : 0u;
        r.n[i] = (s == 0 ? lo : __builtin_amdgcn_alignbit(hi, lo, s)) & (i == 9 ? M22 : M26);
    }
}
// canonical value to 8 little-endian words
__device__ __forceinline__ void to_words(uint32_t (&w)[8], const fe& a) {
#pragma unroll
    for (int q = 0; q < 8; q++) w[q] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const int bit = 26 * i, q = bit / 32, s = bit % 32;
        w[q] |= a.n[i] << s;
        if (s > 6 && q + 1 < 8) w[q + 1] |= a.n[i] >> (32 - s);
    }
}

// ------------------------------------------------------------------ points (Jacobian, a = 0)
// Formulas hold on every curve y^2 = x^3 + b, so they also run on an isomorphic curve whose
// points are (x z^2, y z^3) of the original ones (the "global z" table below).
// Invariant between operations: x, y M1; z magnitude <= 2.07.
struct gej {
    fe x, y, z;
    bool inf;
};

// dbl-2009-l: 2M + 5S
__device__ __forceinline__ void dbl(gej& r, const gej& p) {
    if (p.inf) {
        r.inf = true;
        return;
    }
    fe A, B, C, D, E, F, t;
    sqr(A, p.x);
    sqr(B, p.y);
    sqr(C, B);
    add(t, p.x, B); // 2.07
    sqr(t, t);
    sub(t, t, A, 2);
    sub(t, t, C, 2); // 5.03
    mul_int(D, t, 2);
    norm(D);
    mul_int(E, A, 3);
    norm(E);
    sqr(F, E);
    fe D2;
    mul_int(D2, D, 2);        // 2.07
    sub(r.x, F, D2, 3);        // 4.04
    norm(r.x);
    sub(t, D, r.x, 2);         // 3.04
    mul(t, E, t);
    fe C8;
    mul_int(C8, C, 8);         // 8.26
    sub(r.y, t, C8, 9);        // 10.04
    norm(r.y);
    mul(t, p.y, p.z);
    mul_int(r.z, t, 2);        // 2.07
    r.inf = false;
}

// the doubling branch of the additions (a == b): rare, kept out of line
__device__ __noinline__ gej dbl_rare(gej a) {
    norm(a.x);
    norm(a.y);
    gej r;
    dbl(r, a);
    return r;
}

// madd-2007-bl with z3 = 2 z1 h: a + (bx, by) affine (bx M1, by magnitude <= 2). ratio (if
// given) receives z3 / z1 = 2h, magnitude 2.07 (the table build needs it).
__device__ __forceinline__ void add_ge(gej& r, const gej& a, const fe& bx, const fe& by, fe* ratio = nullptr) {
    if (a.inf) {
        r.x = bx;
        r.y = by;
        norm(r.y);
        set_int(r.z, 1);
        r.inf = false;
        return;
    }
    fe z1z1, u2, s2, h, hh, i, j, rr, v, t;
    sqr(z1z1, a.z);
    mul(u2, bx, z1z1);
    mul(t, a.z, z1z1);
    mul(s2, by, t);
    sub(h, u2, a.x, 2);
    norm(h);
    sub(rr, s2, a.y, 2);
    mul_int(rr, rr, 2); // 6.07
    norm(rr);
    if (is_zero(h)) {
        if (is_zero(rr)) {
            r = dbl_rare(a);
        } else {
            r.inf = true;
        }
        return;
    }
    if (ratio) mul_int(*ratio, h, 2);
    sqr(hh, h);
    mul_int(i, hh, 4); // 4.13
    mul(j, h, i);
    mul(v, a.x, i);
    fe x3;
    sqr(x3, rr);
    sub(x3, x3, j, 2);
    fe v2;
    mul_int(v2, v, 2);
    sub(x3, x3, v2, 3); // 6.04
    norm(x3);
    sub(t, v, x3, 2);
    mul(t, rr, t);
    fe yj;
    mul(yj, a.y, j);
    mul_int(yj, yj, 2);
    sub(r.y, t, yj, 3);
    norm(r.y);
    mul(t, a.z, h);
    mul_int(r.z, t, 2);
    r.x = x3;
    r.inf = false;
}

// add-2007-bl, general Jacobian + Jacobian (inputs: x, y M1 or up to 2.07; z <= 2.07)
__device__ __forceinline__ void add_gej(gej& r, const gej& a, const gej& b) {
    if (a.inf) {
        r = b;
        return;
    }
    if (b.inf) {
        r = a;
        return;
    }
    fe z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
    sqr(z1z1, a.z);
    sqr(z2z2, b.z);
    mul(u1, a.x, z2z2);
    mul(u2, b.x, z1z1);
    mul(t, b.z, z2z2);
    mul(s1, a.y, t);
    mul(t, a.z, z1z1);
    mul(s2, b.y, t);
    sub(h, u2, u1, 2);
    norm(h);
    sub(rr, s2, s1, 2);
    mul_int(rr, rr, 2);
    norm(rr);
    if (is_zero(h)) {
        if (is_zero(rr)) {
            r = dbl_rare(a);
        } else {
            r.inf = true;
        }
        return;
    }
    mul_int(t, h, 2);
    sqr(i, t);
    mul(j, h, i);
    mul(v, u1, i);
    fe x3;
    sqr(x3, rr);
    sub(x3, x3, j, 2);
    fe v2;
    mul_int(v2, v, 2);
    sub(x3, x3, v2, 3);
    norm(x3);
    sub(t, v, x3, 2);
    mul(t, rr, t);
    fe sj;
    mul(sj, s1, j);
    mul_int(sj, sj, 2);
    sub(r.y, t, sj, 3);
    norm(r.y);
    mul(t, a.z, b.z);
    mul(t, t, h);
    mul_int(r.z, t, 2);
    r.x = x3;
    r.inf = false;
}

// r = a^((p+1)/4); true iff r^2 == a (a M1)
__device__ __forceinline__ void sqr_n(fe& r, const fe& a, int n) {
    sqr(r, a);
    for (int i = 1; i < n; i++) sqr(r, r);
}
__device__ __noinline__ bool sqrt_var(fe& r, fe a) {
    fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t1;
    sqr(x2, a);
    mul(x2, x2, a);
    sqr(x3, x2);
    mul(x3, x3, a);
    sqr_n(x6, x3, 3);
    mul(x6, x6, x3);
    sqr_n(x9, x6, 3);
    mul(x9, x9, x3);
    sqr_n(x11, x9, 2);
    mul(x11, x11, x2);
    sqr_n(x22, x11, 11);
    mul(x22, x22, x11);
    sqr_n(x44, x22, 22);
    mul(x44, x44, x22);
    sqr_n(x88, x44, 44);
    mul(x88, x88, x44);
    sqr_n(x176, x88, 88);
    mul(x176, x176, x88);
    sqr_n(x220, x176, 44);
    mul(x220, x220, x44);
    sqr_n(x223, x220, 3);
    mul(x223, x223, x3);
    sqr_n(t1, x223, 23);
    mul(t1, t1, x22);
    sqr_n(t1, t1, 6);
    mul(t1, t1, x2);
    sqr_n(r, t1, 2);
    fe chk;
    sqr(chk, r);
    sub(chk, chk, a, 2);
    norm(chk);
    return is_zero(chk);
}

} // namespace f10
} // namespace gpu
} // namespace bcp
