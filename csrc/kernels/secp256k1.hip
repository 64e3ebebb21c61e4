// Batched secp256k1 ECDSA verification on CDNA4 (gfx950).
//
// Replaces the CCheckQueue fan-out of CPubKey::Verify (reference src/pubkey.cpp:170-193,
// src/validation.cpp:1740 scriptcheckqueue) for block validation.
//
// Work split (see csrc/node/sigverify.cpp):
//   host  : lax-DER parse and low-S normalisation only (copies r, s, z, pubkey)
//   device: ecdsa_prep_kernel  - r,s range checks, s^-1 mod n (Montgomery CIOS,
//                                Fermat exponent n-2), u1 = z/s, u2 = r/s, width-4 wNAF
//                                recoding of u2, r+n precompute
//           ecdsa_verify_kernel - pubkey decompression (sqrt chain), R = u1*G + u2*Q,
//                                check x(R) == r (mod n) without any field inversion:
//                                X == r*Z^2  or  X == (r+n)*Z^2 when r+n < p.
//
// Field arithmetic: 8 x 32-bit limbs (one VGPR each), schoolbook products through
// 32x32+64 -> 64 multiply-adds, reduction by 2^256 = 2^32 + 977 (mod p).
// u1*G: fixed-base comb over 32 byte-windows, table[i][j] = j*256^i*G (affine,
// 512 KiB in global memory, L2/MALL resident) -> 32 mixed additions, no doublings.
// u2*Q: width-4 wNAF with 4 odd multiples of Q held in LDS (96 B each per lane).
// One lane per signature, 128-lane workgroups (2 waves) -> 48 KiB LDS per WG.
#include <hip/hip_runtime.h>

#include "kernels/gpu_api.h"
#include "kernels/hip_util.h"
#include "kernels/der_lax.h"
#include "kernels/modinv.h"
#include "kernels/fe10.h"
#include "secp256k1/secp256k1.h"

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <vector>

namespace bcp {
namespace gpu {

namespace {

struct fe {
    uint32_t v[8];
};

__device__ __constant__ uint32_t P_LIMBS[8] = {0xFFFFFC2F, 0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFF,
                                               0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF};

__device__ __forceinline__ void fe_set(fe& r, const fe& a) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = a.v[i];
}

// Field elements are kept LAZILY reduced: any value in [0, 2^256) stands for itself mod p.
// Additions, subtractions and products fold the excess over 2^256 back in as
// 2^256 = 2^32 + 977 (mod p) instead of comparing against p, and only fe_normalize (used by
// every comparison and parity test) brings a value below p — a value below 2^256 < 2p needs at
// most one subtraction of p.

// r = a - p if a >= p (a < 2p)
__device__ __forceinline__ void fe_cond_sub_p(fe& a, uint32_t carry_in) {
    uint32_t t[8];
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t d = (uint64_t)a.v[i] - P_LIMBS[i] - borrow;
        t[i] = (uint32_t)d;
        borrow = (d >> 63) & 1;
    }
    // take t if carry_in (value >= 2^256) or no borrow (a >= p)
    const bool take = carry_in || !borrow;
#pragma unroll
    for (int i = 0; i < 8; i++) a.v[i] = take ? t[i] : a.v[i];
}
__device__ __forceinline__ void fe_normalize(fe& a) { fe_cond_sub_p(a, 0); }

// 32-bit add / subtract with carry (v_add_co / v_addc, v_sub_co / v_subb chains)
__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t ci, uint32_t* co) {
    return __builtin_addc(a, b, ci, co);
}
__device__ __forceinline__ uint32_t subb(uint32_t a, uint32_t b, uint32_t bi, uint32_t* bo) {
    return __builtin_subc(a, b, bi, bo);
}

// r += c * 2^256 (mod p) for c < 2^40, as r += c * (2^32 + 977); repeats while the sum carries
// out of 2^256 again (only for r within (2^32 + 977) c of 2^256).
__device__ __forceinline__ void fe_fold(fe& r, uint64_t c) {
    while (c) {
        uint32_t co;
        const uint64_t lo = c * 977u;                          // < 2^50
        const uint64_t mid = (lo >> 32) + (uint32_t)c;         // limb 1 (< 2^33)
        r.v[0] = addc(r.v[0], (uint32_t)lo, 0, &co);
        r.v[1] = addc(r.v[1], (uint32_t)mid, co, &co);
        r.v[2] = addc(r.v[2], (uint32_t)(mid >> 32) + (uint32_t)(c >> 32), co, &co);
#pragma unroll
        for (int i = 3; i < 8; i++) r.v[i] = addc(r.v[i], 0, co, &co);
        c = co;
    }
}
// r -= b * 2^256 (mod p), as r -= b * (2^32 + 977), while the difference borrows below 0
__device__ __forceinline__ void fe_unfold(fe& r, uint32_t b) {
    while (b) {
        uint32_t bo;
        r.v[0] = subb(r.v[0], 977u * b, 0, &bo);
        r.v[1] = subb(r.v[1], b, bo, &bo);
#pragma unroll
        for (int i = 2; i < 8; i++) r.v[i] = subb(r.v[i], 0, bo, &bo);
        b = bo;
    }
}

__device__ __forceinline__ void fe_add(fe& r, const fe& a, const fe& b) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = addc(a.v[i], b.v[i], c, &c);
    fe_fold(r, c);
}

__device__ __forceinline__ void fe_sub(fe& r, const fe& a, const fe& b) {
    uint32_t bo = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = subb(a.v[i], b.v[i], bo, &bo);
    fe_unfold(r, bo); // a - b + 2^256 was computed: take 2^256 = 2^32 + 977 back out
}

__device__ __forceinline__ void fe_mul_small(fe& r, const fe& a, uint32_t m) {
    // r = a*m mod p for small m (2, 3, 4, 8)
    uint32_t hi = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t p = (uint64_t)a.v[i] * m + hi;
        r.v[i] = (uint32_t)p;
        hi = (uint32_t)(p >> 32);
    }
    fe_fold(r, hi);
}

// One product-scanning step: {acc} += a*b, c2 += the carry out of the 64-bit accumulator
// (v_mad_u64_u32 writes its carry to VCC, which v_addc folds into the column's third word; a
// VALU carry-in read needs two wait states after the VALU write of VCC on gfx950).
__device__ __forceinline__ void fe_mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(c2)
        : "v"(a), "v"(b)
        : "vcc");
}

// 512-bit value t reduced to r < 2^256 (r = t mod p, lazily): r = lo + hi * (2^32 + 977)
__device__ __forceinline__ void fe_reduce512(fe& r, const uint32_t (&t)[16]) {
    uint32_t u[8], c = 0; // u = lo + (hi << 32), u8 its top word (33 bits)
    u[0] = t[0];
#pragma unroll
    for (int i = 1; i < 8; i++) u[i] = addc(t[i], t[7 + i], c, &c);
    const uint64_t u8 = (uint64_t)t[15] + c;
    uint32_t cc = 0; // + hi * 977, carried limb by limb (every partial < 2^43)
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t p = (uint64_t)t[8 + i] * 977u + cc;
        uint32_t co;
        r.v[i] = addc(u[i], (uint32_t)p, 0, &co);
        cc = (uint32_t)(p >> 32) + co;
    }
    fe_fold(r, u8 + cc); // value = r + (u8 + cc) * 2^256, u8 + cc < 2^34
}

// Product scanning (Comba): column k of a*b accumulates every a_i*b_j with i + j = k in a
// 3-word accumulator; 64 v_mad_u64_u32 + 64 v_addc, no zero-extended 64-bit adds.
__device__ __forceinline__ void fe_mul_impl(fe& r, const fe& a, const fe& b) {
    uint32_t t[16];
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 0; k < 15; k++) {
#pragma unroll
        for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) fe_mac(acc, c2, a.v[i], b.v[k - i]);
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)c2 << 32);
        c2 = 0;
    }
    t[15] = (uint32_t)acc;
    fe_reduce512(r, t);
}

// Squaring: the 28 cross products a_i*a_j (i<j) once by product scanning, doubled with a 1-bit
// shift, plus the 8 diagonal squares — 36 multiplies instead of 64.
__device__ __forceinline__ void fe_sqr_impl(fe& r, const fe& a) {
    uint32_t t[16];
    t[0] = 0;
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 1; k < 14; k++) {
#pragma unroll
        for (int i = (k > 7 ? k - 7 : 0); 2 * i < k; i++) fe_mac(acc, c2, a.v[i], a.v[k - i]);
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)c2 << 32);
        c2 = 0;
    }
    t[14] = (uint32_t)acc;
    t[15] = t[14] >> 31;
#pragma unroll
    for (int i = 14; i > 0; i--) t[i] = __builtin_amdgcn_alignbit(t[i], t[i - 1], 31); // (t[i] << 1) | (t[i-1] >> 31)
    t[0] = 0;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t sq = (uint64_t)a.v[i] * a.v[i];
        t[2 * i] = addc(t[2 * i], (uint32_t)sq, c, &c);
        t[2 * i + 1] = addc(t[2 * i + 1], (uint32_t)(sq >> 32), c, &c);
    }
    fe_reduce512(r, t);
}

// Out-of-line multiply and square, arguments and result in VGPRs (by value: a by-reference
// argument of a non-inlined function would go through scratch). Inlining every field operation
// made the verify kernel ~460 KB of straight-line code: with one wave per SIMD the instruction
// cache, not the multipliers, set its speed.
__device__ __noinline__ fe fe_mul_v(fe a, fe b) {
    fe r;
    fe_mul_impl(r, a, b);
    return r;
}
__device__ __noinline__ fe fe_sqr_v(fe a) {
    fe r;
    fe_sqr_impl(r, a);
    return r;
}
__device__ __forceinline__ void fe_mul(fe& r, const fe& a, const fe& b) { r = fe_mul_v(a, b); }
__device__ __forceinline__ void fe_sqr(fe& r, const fe& a) { r = fe_sqr_v(a); }

__device__ __forceinline__ void fe_sqr_n(fe& r, const fe& a, int n) {
    fe_sqr(r, a);
    for (int i = 1; i < n; i++) fe_sqr(r, r);
}

// comparisons see canonical values (a lazily reduced p reads as 0)
__device__ __forceinline__ bool fe_is_zero(const fe& in) {
    fe a = in;
    fe_normalize(a);
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) o |= a.v[i];
    return o == 0;
}

__device__ __forceinline__ bool fe_eq(const fe& ain, const fe& bin) {
    fe a = ain, b = bin;
    fe_normalize(a);
    fe_normalize(b);
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i];
    return o == 0;
}

// x223 = a^(2^223 - 1), with x2 = a^3 and x22 = a^(2^22 - 1) on the way (libsecp256k1 chain).
__device__ void fe_chain223(fe& x223, fe& x22, fe& x2, const fe& a) {
    fe x3, x6, x9, x11, x44, x88, x176, x220;
    fe_sqr(x2, a);
    fe_mul(x2, x2, a);
    fe_sqr(x3, x2);
    fe_mul(x3, x3, a);
    fe_sqr_n(x6, x3, 3);
    fe_mul(x6, x6, x3);
    fe_sqr_n(x9, x6, 3);
    fe_mul(x9, x9, x3);
    fe_sqr_n(x11, x9, 2);
    fe_mul(x11, x11, x2);
    fe_sqr_n(x22, x11, 11);
    fe_mul(x22, x22, x11);
    fe_sqr_n(x44, x22, 22);
    fe_mul(x44, x44, x22);
    fe_sqr_n(x88, x44, 44);
    fe_mul(x88, x88, x44);
    fe_sqr_n(x176, x88, 88);
    fe_mul(x176, x176, x88);
    fe_sqr_n(x220, x176, 44);
    fe_mul(x220, x220, x44);
    fe_sqr_n(x223, x220, 3);
    fe_mul(x223, x223, x3);
}

// r = a^(p-2) = 1/a (a != 0): the p-2 blocks of ones are 223, 22, 1, 2, 1 bits long.
__device__ void fe_inv(fe& r, const fe& a) {
    fe x223, x22, x2, t1;
    fe_chain223(x223, x22, x2, a);
    fe_sqr_n(t1, x223, 23);
    fe_mul(t1, t1, x22);
    fe_sqr_n(t1, t1, 5);
    fe_mul(t1, t1, a);
    fe_sqr_n(t1, t1, 3);
    fe_mul(t1, t1, x2);
    fe_sqr_n(t1, t1, 2);
    fe_mul(r, t1, a);
}

// r = a^((p+1)/4); returns whether r^2 == a (libsecp256k1 addition chain).
__device__ __forceinline__ bool fe_sqrt(fe& r, const fe& a) {
    fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t1;
    fe_sqr(x2, a);
    fe_mul(x2, x2, a);
    fe_sqr(x3, x2);
    fe_mul(x3, x3, a);
    fe_sqr_n(x6, x3, 3);
    fe_mul(x6, x6, x3);
    fe_sqr_n(x9, x6, 3);
    fe_mul(x9, x9, x3);
    fe_sqr_n(x11, x9, 2);
    fe_mul(x11, x11, x2);
    fe_sqr_n(x22, x11, 11);
    fe_mul(x22, x22, x11);
    fe_sqr_n(x44, x22, 22);
    fe_mul(x44, x44, x22);
    fe_sqr_n(x88, x44, 44);
    fe_mul(x88, x88, x44);
    fe_sqr_n(x176, x88, 88);
    fe_mul(x176, x176, x88);
    fe_sqr_n(x220, x176, 44);
    fe_mul(x220, x220, x44);
    fe_sqr_n(x223, x220, 3);
    fe_mul(x223, x223, x3);
    fe_sqr_n(t1, x223, 23);
    fe_mul(t1, t1, x22);
    fe_sqr_n(t1, t1, 6);
    fe_mul(t1, t1, x2);
    fe_sqr_n(r, t1, 2);
    fe chk;
    fe_sqr(chk, r);
    return fe_eq(chk, a);
}

struct gej {
    fe x, y, z;
    bool inf;
};

// dbl-2009-l (a = 0): 2M + 5S
__device__ __forceinline__ void gej_double(gej& r, const gej& p) {
    if (p.inf) {
        r.inf = true;
        return;
    }
    fe A, B, C, D, E, F, t;
    fe_sqr(A, p.x);
    fe_sqr(B, p.y);
    fe_sqr(C, B);
    fe_add(t, p.x, B);
    fe_sqr(t, t);
    fe_sub(t, t, A);
    fe_sub(t, t, C);
    fe_mul_small(D, t, 2);
    fe_mul_small(E, A, 3);
    fe_sqr(F, E);
    fe z3;
    fe_mul(z3, p.y, p.z);
    fe_mul_small(r.z, z3, 2);
    fe_mul_small(t, D, 2);
    fe_sub(r.x, F, t);
    fe_sub(t, D, r.x);
    fe_mul(t, E, t);
    fe C8;
    fe_mul_small(C8, C, 8);
    fe_sub(r.y, t, C8);
    r.inf = false;
}

// add-2007-bl, general Jacobian + Jacobian
__device__ __forceinline__ void gej_add(gej& r, const gej& a, const gej& b) {
    if (a.inf) {
        r = b;
        return;
    }
    if (b.inf) {
        r = a;
        return;
    }
    fe z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
    fe_sqr(z1z1, a.z);
    fe_sqr(z2z2, b.z);
    fe_mul(u1, a.x, z2z2);
    fe_mul(u2, b.x, z1z1);
    fe_mul(s1, a.y, b.z);
    fe_mul(s1, s1, z2z2);
    fe_mul(s2, b.y, a.z);
    fe_mul(s2, s2, z1z1);
    fe_sub(h, u2, u1);
    fe_sub(rr, s2, s1);
    if (fe_is_zero(h)) {
        if (fe_is_zero(rr)) {
            gej_double(r, a);
        } else {
            r.inf = true;
        }
        return;
    }
    fe_mul_small(i, h, 2);
    fe_sqr(i, i);
    fe_mul(j, h, i);
    fe_mul_small(rr, rr, 2);
    fe_mul(v, u1, i);
    fe x3, y3, z3;
    fe_sqr(x3, rr);
    fe_sub(x3, x3, j);
    fe_mul_small(t, v, 2);
    fe_sub(x3, x3, t);
    fe_sub(t, v, x3);
    fe_mul(y3, rr, t);
    fe_mul(t, s1, j);
    fe_mul_small(t, t, 2);
    fe_sub(y3, y3, t);
    fe_add(t, a.z, b.z);
    fe_sqr(t, t);
    fe_sub(t, t, z1z1);
    fe_sub(t, t, z2z2);
    fe_mul(z3, t, h);
    r.x = x3;
    r.y = y3;
    r.z = z3;
    r.inf = false;
}

// madd-2007-bl, Jacobian + affine
__device__ __forceinline__ void gej_add_ge(gej& r, const gej& a, const fe& bx, const fe& by) {
    if (a.inf) {
        r.x = bx;
        r.y = by;
#pragma unroll
        for (int k = 0; k < 8; k++) r.z.v[k] = k == 0 ? 1u : 0u;
        r.inf = false;
        return;
    }
    fe z1z1, u2, s2, h, hh, i, j, rr, v, t;
    fe_sqr(z1z1, a.z);
    fe_mul(u2, bx, z1z1);
    fe_mul(s2, by, a.z);
    fe_mul(s2, s2, z1z1);
    fe_sub(h, u2, a.x);
    fe_sub(rr, s2, a.y);
    if (fe_is_zero(h)) {
        if (fe_is_zero(rr)) {
            gej_double(r, a);
        } else {
            r.inf = true;
        }
        return;
    }
    fe_sqr(hh, h);
    fe_mul_small(i, hh, 4);
    fe_mul(j, h, i);
    fe_mul_small(rr, rr, 2);
    fe_mul(v, a.x, i);
    fe x3, y3, z3;
    fe_sqr(x3, rr);
    fe_sub(x3, x3, j);
    fe_mul_small(t, v, 2);
    fe_sub(x3, x3, t);
    fe_sub(t, v, x3);
    fe_mul(y3, rr, t);
    fe_mul(t, a.y, j);
    fe_mul_small(t, t, 2);
    fe_sub(y3, y3, t);
    fe_add(t, a.z, h);
    fe_sqr(t, t);
    fe_sub(t, t, z1z1);
    fe_sub(z3, t, hh);
    r.x = x3;
    r.y = y3;
    r.z = z3;
    r.inf = false;
}

__device__ __forceinline__ void load_be32(fe& r, const unsigned char* b) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const unsigned char* q = b + 28 - 4 * i;
        r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
}

__device__ __forceinline__ bool fe_lt_p(const fe& a) {
    // a < p  <=>  a - p borrows
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t d = (uint64_t)a.v[i] - P_LIMBS[i] - borrow;
        borrow = (d >> 63) & 1;
    }
    return borrow != 0;
}

constexpr int WG = 128;
#ifndef BCP_ECDSA_AFFINE_TABLE // 1: the Q multiples are made affine (one batched inversion), LDS holds
#define BCP_ECDSA_AFFINE_TABLE 1 //    X and Y only and every table addition is a mixed one
#endif
#ifndef BCP_ECDSA_BINGCD // 1: s^-1 mod n by the binary extended Euclid (modinv.h), 0: Fermat power
#define BCP_ECDSA_BINGCD 1
#endif
#ifndef BCP_ECDSA_REGULAR // 1: regular window-3 recoding of the GLV halves (uniform additions)
#define BCP_ECDSA_REGULAR 1
#endif
#ifndef BCP_ECDSA_FUSED_MAX // default of EcdsaFusedMax(): batches up to this size run the fused latency kernel
#define BCP_ECDSA_FUSED_MAX 16384 // one workgroup per CU at most (profiles/ecdsa_r5.md)
#endif
#ifndef BCP_ECDSA_SPLIT_KERNEL // verify kernel after the prep kernel: 0 = 8 x 32 (ecdsa_verify_kernel), 1 = 10 x 26
                               // (one lane per signature for whole rounds, a half-lane tail), 2 / 3 = only
                               // the one-lane / the half-lane 10 x 26 kernel (tests)
#define BCP_ECDSA_SPLIT_KERNEL 1
#endif
constexpr int WNAF_W = 4;              // odd multiples 1,3,5,7
constexpr int NPRE = 1 << (WNAF_W - 2); // 4

constexpr int GLV_DIGITS = 132; // width-4 wNAF digits of a <= 129-bit GLV half (|k1|,|k2| < 2^129)

struct Job {
    unsigned char u1[32];   // big-endian scalar for the G comb
    unsigned char r[32];    // big-endian r
    unsigned char rn[32];   // big-endian r + n (valid when rplusn_ok)
    unsigned char pub[33];  // compressed key
    unsigned char rplusn_ok;
    // u2 = k1 + k2*lambda (mod n), |k1|, |k2| < 2^129 (GLV): width-4 wNAF of |k1| and |k2|,
    // 2 signed nibbles per byte, digit b at wnaf[i][b>>1]; neg[i]: k_i < 0
    unsigned char wnaf[2][GLV_DIGITS / 2];
    unsigned char nwnaf[2]; // digits of each half
    unsigned char neg[2];
    unsigned char scalar_ok; // set by the prep kernel: r, s in [1, n-1]
    unsigned char pad[5];    // regular recoding: pad[0], pad[1] = half 0 / 1 was even (encoded as k + 1)
};
// Host-filled input to the prep kernel (u1 <- z, rn <- s before prep).
static_assert(sizeof(Job) == 272, "job layout");

__device__ __forceinline__ int wnaf_digit(const Job& J, int h, int b) {
    if (b >= J.nwnaf[h]) return 0;
    const int byte = J.wnaf[h][b >> 1];
    const int nib = (b & 1) ? (byte >> 4) : (byte & 15);
    return nib >= 8 ? nib - 16 : nib;
}


// ---------------------------------------------------------------- scalars mod n
__device__ __constant__ uint32_t N_LIMBS[8] = {0xD0364141, 0xBFD25E8C, 0xAF48A03B, 0xBAAEDCE6,
                                               0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF};
__device__ __constant__ uint32_t N_R2[8] = {0x67D7D140, 0x896CF214, 0x0E7CF878, 0x741496C2,
                                            0x5BCD07C6, 0xE697F5E4, 0x81C69BC5, 0x9D671CD5};
__device__ __constant__ uint32_t N_ONE_M[8] = {0x2FC9BEBF, 0x402DA173, 0x50B75FC4, 0x45512319, 1, 0, 0, 0};
__device__ __constant__ uint32_t N_MINUS_2[8] = {0xD036413F, 0xBFD25E8C, 0xAF48A03B, 0xBAAEDCE6,
                                                 0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF};
constexpr uint32_t N_INV32 = 0x5588B13F; // -n^-1 mod 2^32

// GLV endomorphism (secp256k1 has a cube root of unity lambda mod n with lambda*(x, y) =
// (beta*x, y)): u2 = k1 + k2*lambda with ~128-bit k1, k2 halves the doublings of u2*Q.
// Lattice basis (a1,b1), (a2,b2) of {(a,b): a + b*lambda = 0 mod n}; c1 = round(b2*k/n),
// c2 = round(-b1*k/n) through g1 = round(2^384*b2/n), g2 = round(2^384*(-b1)/n);
// k1 = k - c1*a1 - c2*a2, k2 = -c1*b1 - c2*b2 (exact integers, |k1|,|k2| < 2^129).
// Derived and range-checked over 2e5 random scalars with Python integers.
__device__ __constant__ uint32_t GLV_G1[8] = {0x45DBB031, 0xE893209A, 0x71E8CA7F, 0x3DAA8A14,
                                              0x9284EB15, 0xE86C90E4, 0xA7D46BCD, 0x3086D221};
__device__ __constant__ uint32_t GLV_G2[8] = {0x8AC47F71, 0x1571B4AE, 0x9DF506C6, 0x221208AC,
                                              0x0ABFE4C4, 0x6F547FA9, 0x010E8828, 0xE4437ED6};
__device__ __constant__ uint32_t GLV_A1[4] = {0x9284EB15, 0xE86C90E4, 0xA7D46BCD, 0x3086D221};
__device__ __constant__ uint32_t GLV_B1N[4] = {0x0ABFE4C3, 0x6F547FA9, 0x010E8828, 0xE4437ED6}; // -b1
__device__ __constant__ uint32_t GLV_A2[5] = {0x9D44CFD8, 0x57C1108D, 0xA8E2F3F6, 0x14CA50F7, 0x00000001};
__device__ __constant__ uint32_t GLV_B2[4] = {0x9284EB15, 0xE86C90E4, 0xA7D46BCD, 0x3086D221};
__device__ __constant__ uint32_t GLV_BETA[8] = {0x719501EE, 0xC1396C28, 0x12F58995, 0x9CF04975,
                                                0xAC3434E9, 0x6E64479E, 0x657C0710, 0x7AE96A2B};

// r[0 .. NA+NB) = a[0 .. NA) * b[0 .. NB) (plain integers, 32-bit limbs, little-endian)
template <int NA, int NB>
__device__ __forceinline__ void mul_wide(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#pragma unroll
    for (int i = 0; i < NA + NB; i++) r[i] = 0;
#pragma unroll
    for (int i = 0; i < NA; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < NB; j++) {
            c += (uint64_t)r[i + j] + (uint64_t)a[i] * b[j];
            r[i + j] = (uint32_t)c;
            c >>= 32;
        }
        r[i + NB] = (uint32_t)c;
    }
}
// round(k * g / 2^384) for 256-bit k and g: the top 128 bits of the product plus the rounding bit
__device__ __forceinline__ void mul_shift384(uint32_t (&c)[4], const fe& k, const uint32_t* g) {
    uint32_t t[16];
    mul_wide<8, 8>(t, k.v, g);
    uint64_t carry = t[11] >> 31; // bit 383
#pragma unroll
    for (int i = 0; i < 4; i++) {
        carry += t[12 + i];
        c[i] = (uint32_t)carry;
        carry >>= 32;
    }
}
// width-4 wNAF of a magnitude m (<= 5 limbs, < 2^130), LSB first into J-style nibble bytes
__device__ __forceinline__ int wnaf4(unsigned char* out, const uint32_t (&m)[5]) {
    uint32_t k[6];
#pragma unroll
    for (int i = 0; i < 5; i++) k[i] = m[i];
    k[5] = 0;
    int len = 0;
    unsigned char cur = 0;
    for (int b = 0; b < GLV_DIGITS; b++) {
        int d = 0;
        if (k[0] & 1) {
            d = (int)(k[0] & 15);
            if (d >= 8) d -= 16;
            const uint32_t addend = (uint32_t)(-d);
            const uint32_t ext = d > 0 ? 0xFFFFFFFFu : 0u;
            uint64_t c = 0;
#pragma unroll
            for (int i = 0; i < 6; i++) {
                c += (uint64_t)k[i] + (i == 0 ? addend : ext);
                k[i] = (uint32_t)c;
                c >>= 32;
            }
            len = b + 1;
        }
        const unsigned char nib = (unsigned char)(d & 15);
        if (b & 1) {
            out[b >> 1] = cur | (unsigned char)(nib << 4);
            cur = 0;
        } else {
            cur = nib;
        }
#pragma unroll
        for (int i = 0; i < 5; i++) k[i] = (k[i] >> 1) | (k[i + 1] << 31);
        k[5] >>= 1;
    }
    return len;
}
// Regular signed-digit recoding with window 3 (BCP_ECDSA_REGULAR): an odd magnitude m < 2^130
// becomes exactly REG_DIGITS digits, every one odd in [-7, 7] (never zero), m = sum d_i 8^i:
// d = (m mod 16) - 8, m = (m - d) / 8 for the low digits, the remaining 1..7 on top. Every lane
// then adds at the same positions, so a wave runs 2 x 44 point additions instead of one at
// almost every bit (a width-4 wNAF digit is nonzero somewhere among 64 lanes at nearly every
// position, and the divergent branch costs the whole wave).
constexpr int REG_DIGITS = 44;
__device__ __forceinline__ void regw3(unsigned char* out, const uint32_t (&m)[5]) {
    uint32_t k[5];
#pragma unroll
    for (int i = 0; i < 5; i++) k[i] = m[i];
    unsigned char cur = 0;
    for (int b = 0; b < REG_DIGITS; b++) {
        int d;
        if (b == REG_DIGITS - 1) {
            d = (int)k[0]; // 1..7
        } else {
            d = (int)(k[0] & 15) - 8;
            // k -= d (k - d = 8 mod 16), then k >>= 3
            const uint32_t addend = (uint32_t)(-d), ext = d > 0 ? 0xFFFFFFFFu : 0u;
            uint64_t c = 0;
#pragma unroll
            for (int i = 0; i < 5; i++) {
                c += (uint64_t)k[i] + (i == 0 ? addend : ext);
                k[i] = (uint32_t)c;
                c >>= 32;
            }
#pragma unroll
            for (int i = 0; i < 4; i++) k[i] = (k[i] >> 3) | (k[i + 1] << 29);
            k[4] >>= 3;
        }
        const unsigned char nib = (unsigned char)(d & 15);
        if (b & 1) {
            out[b >> 1] = cur | (unsigned char)(nib << 4);
            cur = 0;
        } else {
            cur = nib;
        }
    }
}

// Regular recoding with window 4 for the 10 x 26 kernels: an odd magnitude m < 2^130 becomes
// REG4_DIGITS odd digits in [-15, 15], m = sum d_i 16^i (d = (m mod 32) - 16, m = (m - d) / 16;
// the top digit is what remains, 1..3). Each digit is stored as a nibble: bit 3 = sign,
// bits 0-2 = |d| >> 1 (the index of the odd multiple |d| Q).
constexpr int REG4_DIGITS = 33;
constexpr int NPRE4 = 8; // odd multiples Q .. 15Q
__device__ __forceinline__ void regw4(unsigned char* out, const uint32_t (&m)[5]) {
    uint32_t k[5];
#pragma unroll
    for (int i = 0; i < 5; i++) k[i] = m[i];
    unsigned char cur = 0;
    for (int b = 0; b < REG4_DIGITS; b++) {
        int d;
        if (b == REG4_DIGITS - 1) {
            d = (int)k[0];
        } else {
            d = (int)(k[0] & 31) - 16;
            const uint32_t addend = (uint32_t)(-d), ext = d > 0 ? 0xFFFFFFFFu : 0u;
            uint64_t c = 0;
#pragma unroll
            for (int i = 0; i < 5; i++) {
                c += (uint64_t)k[i] + (i == 0 ? addend : ext);
                k[i] = (uint32_t)c;
                c >>= 32;
            }
#pragma unroll
            for (int i = 0; i < 4; i++) k[i] = (k[i] >> 4) | (k[i + 1] << 28);
            k[4] >>= 4;
        }
        const unsigned char nib = (unsigned char)(((d < 0) ? 8 : 0) | (((d < 0 ? -d : d) >> 1) & 7));
        if (b & 1) {
            out[b >> 1] = cur | (unsigned char)(nib << 4);
            cur = 0;
        } else {
            cur = nib;
        }
    }
    out[REG4_DIGITS >> 1] = cur; // the odd count leaves the top digit in a low nibble
}
// digit b of half h of a window-4 job: the signed odd multiple
__device__ __forceinline__ int reg4_digit(const Job& J, int h, int b) {
    const int byte = J.wnaf[h][b >> 1];
    const int nib = (b & 1) ? (byte >> 4) : (byte & 15);
    const int mag = 2 * (nib & 7) + 1;
    return (nib & 8) ? -mag : mag;
}

// 10-limb two's complement -> magnitude (5 limbs) and sign
__device__ __forceinline__ bool abs10(uint32_t (&m)[5], uint32_t (&v)[10]) {
    const bool neg = (v[9] >> 31) != 0;
    if (neg) {
        uint64_t c = 1;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            c += (uint64_t)(~v[i]);
            v[i] = (uint32_t)c;
            c >>= 32;
        }
    }
#pragma unroll
    for (int i = 0; i < 5; i++) m[i] = v[i];
    return neg;
}

// a < n ?
__device__ __forceinline__ bool sc_lt_n(const fe& a) {
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t d = (uint64_t)a.v[i] - N_LIMBS[i] - borrow;
        borrow = (d >> 63) & 1;
    }
    return borrow != 0;
}

__device__ __forceinline__ void sc_sub_n(fe& a) {
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t d = (uint64_t)a.v[i] - N_LIMBS[i] - borrow;
        a.v[i] = (uint32_t)d;
        borrow = (d >> 63) & 1;
    }
}

// Montgomery product a*b/2^256 mod n (CIOS, 8 x 32-bit limbs).
__device__ __forceinline__ void sc_mont_mul(fe& r, const fe& a, const fe& b) {
    uint32_t t[10];
#pragma unroll
    for (int i = 0; i < 10; i++) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            c += (uint64_t)t[j] + (uint64_t)a.v[j] * b.v[i];
            t[j] = (uint32_t)c;
            c >>= 32;
        }
        uint64_t s2 = (uint64_t)t[8] + c;
        t[8] = (uint32_t)s2;
        t[9] = (uint32_t)(s2 >> 32);
        const uint32_t m = t[0] * N_INV32;
        c = ((uint64_t)t[0] + (uint64_t)m * N_LIMBS[0]) >> 32;
#pragma unroll
        for (int j = 1; j < 8; j++) {
            c += (uint64_t)t[j] + (uint64_t)m * N_LIMBS[j];
            t[j - 1] = (uint32_t)c;
            c >>= 32;
        }
        s2 = (uint64_t)t[8] + c;
        t[7] = (uint32_t)s2;
        t[8] = t[9] + (uint32_t)(s2 >> 32);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = t[i];
    if (t[8] || !sc_lt_n(r)) sc_sub_n(r);
}

__device__ __forceinline__ void store_be32(unsigned char* b, const fe& a) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        unsigned char* q = b + 28 - 4 * i;
        q[0] = (unsigned char)(a.v[i] >> 24);
        q[1] = (unsigned char)(a.v[i] >> 16);
        q[2] = (unsigned char)(a.v[i] >> 8);
        q[3] = (unsigned char)a.v[i];
    }
}

// s > n/2 ? (the high half of the group order)
__device__ __forceinline__ bool sc_is_high(const fe& a) {
    // n/2 = 7FFFFFFF FFFFFFFF FFFFFFFF FFFFFFFF 5D576E73 57A4501D DFE92F46 681B20A0
    const uint32_t H[8] = {0x681B20A0, 0xDFE92F46, 0x57A4501D, 0x5D576E73, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0x7FFFFFFF};
    for (int i = 7; i >= 0; i--)
        if (a.v[i] != H[i]) return a.v[i] > H[i];
    return false;
}

// One lane per signature: scalar checks, s^-1, u1, u2, wNAF(u2), r+n.
// Reads the packed host arrays (msg 32 B, compact sig 64 B, compressed key 33 B per
// signature: 129 B uploaded instead of a 272 B Job) and builds the Job on the device.
// DER: sig holds [length][72 DER bytes] slots, parsed and low-S normalised here; otherwise
// 64-byte compact r||s, already normalised by the host.
template <bool DER, bool W4>
__device__ __forceinline__ void prep_one(Job& J, const unsigned char* __restrict__ msg, const unsigned char* __restrict__ sig,
                                         const unsigned char* __restrict__ pub, int idx) {
    const unsigned char* pk = pub + (size_t)idx * 33;
    unsigned char c64[64];
    bool parsed = true;
    if constexpr (DER) {
        const unsigned char* slot = sig + (size_t)idx * VerifyLane::DER_SLOT;
        unsigned char der[72];
        const uint32_t len = slot[0] > 72 ? 72u : slot[0];
        for (uint32_t i = 0; i < 72; i++) der[i] = i < len ? slot[1 + i] : 0;
        parsed = bcpk::der_lax_parse(der, len, c64);
    } else {
        const unsigned char* sg = sig + (size_t)idx * 64;
        for (int i = 0; i < 64; i++) c64[i] = sg[i];
    }
#pragma unroll
    for (int i = 0; i < 33; i++) J.pub[i] = pk[i];
    fe r, s, z;
    load_be32(r, c64);
    load_be32(s, c64 + 32);
    load_be32(z, msg + (size_t)idx * 32);
    bool ok = parsed && sc_lt_n(r) && sc_lt_n(s);
    if (DER && ok && sc_is_high(s)) { // low-S normalisation (secp::sig_normalize)
        uint64_t br = 0;
        for (int i = 0; i < 8; i++) {
            const uint64_t d = (uint64_t)N_LIMBS[i] - s.v[i] - br;
            s.v[i] = (uint32_t)d;
            br = (d >> 63) & 1;
        }
    }
    // compact inputs must already be low-S, as secp::ecdsa_verify requires (s and n - s both
    // satisfy the verification equation, so a high-S input is a malleated signature)
    if (!DER && ok && sc_is_high(s)) ok = false;
    ok = ok && !fe_is_zero(r) && !fe_is_zero(s);
    if (!ok) {
#pragma unroll
        for (int i = 0; i < 8; i++) r.v[i] = 0;
    }
    store_be32(J.r, r);
    if (!sc_lt_n(z)) sc_sub_n(z); // z < 2^256 < 2n
    fe one;
#pragma unroll
    for (int i = 0; i < 8; i++) one.v[i] = i == 0 ? 1u : 0u;
    if (!ok) s = one;
    fe r2, acc;
#pragma unroll
    for (int i = 0; i < 8; i++) r2.v[i] = N_R2[i];
#if BCP_ECDSA_BINGCD
    // s^-1 by the binary extended Euclid (modinv.h: ~3x fewer VALU instructions than the
    // exponentiation below), then into the Montgomery domain: acc = s^-1 * R
    {
        uint32_t nl[8], inv[8];
#pragma unroll
        for (int i = 0; i < 8; i++) nl[i] = N_LIMBS[i];
        bcpk::modinv256(inv, s.v, nl);
        fe iv;
#pragma unroll
        for (int i = 0; i < 8; i++) iv.v[i] = inv[i];
        sc_mont_mul(acc, iv, r2);
    }
#else
    // s^(n-2) in the Montgomery domain, left-to-right binary over the constant exponent
    fe sm;
#pragma unroll
    for (int i = 0; i < 8; i++) acc.v[i] = N_ONE_M[i];
    sc_mont_mul(sm, s, r2);
    for (int w = 7; w >= 0; w--) {
        const uint32_t e = N_MINUS_2[w];
        for (int b = 31; b >= 0; b--) {
            sc_mont_mul(acc, acc, acc);
            if ((e >> b) & 1) sc_mont_mul(acc, acc, sm);
        }
    }
#endif
    // acc = s^-1 * R ; montmul with a plain value gives a plain product
    fe u1, u2;
    sc_mont_mul(u1, acc, z);
    sc_mont_mul(u2, acc, r);
    store_be32(J.u1, u1);
    J.scalar_ok = ok ? 1 : 0;
    // r + n (only meaningful when r + n < p)
    // p - n = 0x14551231950b75fc4402da1722fc9baee
    {
        // r < p - n  <=>  r + n < p
        const uint32_t pmn[8] = {0x2FC9BAEE, 0x402DA172, 0x50B75FC4, 0x45512319, 1, 0, 0, 0};
        uint64_t borrow = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint64_t d = (uint64_t)r.v[i] - pmn[i] - borrow;
            borrow = (d >> 63) & 1;
        }
        J.rplusn_ok = borrow ? 1 : 0;
        fe rn;
        uint64_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            c += (uint64_t)r.v[i] + N_LIMBS[i];
            rn.v[i] = (uint32_t)c;
            c >>= 32;
        }
        store_be32(J.rn, rn);
    }
    // GLV split of u2, then width-4 wNAF of each half
    uint32_t c1[4], c2[4];
    mul_shift384(c1, u2, GLV_G1);
    mul_shift384(c2, u2, GLV_G2);
    uint32_t p1[8], p2[8], p3[8], p4[9], k1[10], k2[10];
    mul_wide<4, 4>(p1, c1, GLV_B1N); // c1 * (-b1)
    mul_wide<4, 4>(p2, c2, GLV_B2);  // c2 * b2
    mul_wide<4, 4>(p3, c1, GLV_A1);  // c1 * a1
    mul_wide<4, 5>(p4, c2, GLV_A2);  // c2 * a2
    { // k2 = c1*(-b1) - c2*b2
        uint64_t br = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const uint64_t d = (uint64_t)(i < 8 ? p1[i] : 0u) - (i < 8 ? p2[i] : 0u) - br;
            k2[i] = (uint32_t)d;
            br = (d >> 63) & 1;
        }
    }
    { // k1 = u2 - c1*a1 - c2*a2 (two subtrahends: the borrow reaches 2)
        int64_t br = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const int64_t v = (int64_t)(i < 8 ? u2.v[i] : 0u) - (int64_t)(i < 8 ? p3[i] : 0u) -
                              (int64_t)(i < 9 ? p4[i] : 0u) - br;
            k1[i] = (uint32_t)v;
            br = -(v >> 32); // arithmetic shift: 0, 1 or 2
        }
    }
    uint32_t m1[5], m2[5];
    J.neg[0] = abs10(m1, k1) ? 1 : 0;
    J.neg[1] = abs10(m2, k2) ? 1 : 0;
#if BCP_ECDSA_REGULAR
    // an even half k is encoded as k + 1 and corrected by one subtraction of its point
    auto make_odd = [](uint32_t (&m)[5]) -> unsigned char {
        if (m[0] & 1) return 0;
        m[0] |= 1; // even: + 1 never carries
        return 1;
    };
    J.pad[0] = make_odd(m1);
    J.pad[1] = make_odd(m2);
    if constexpr (W4) {
        regw4(J.wnaf[0], m1);
        regw4(J.wnaf[1], m2);
        J.nwnaf[0] = J.nwnaf[1] = (unsigned char)REG4_DIGITS;
    } else {
        regw3(J.wnaf[0], m1);
        regw3(J.wnaf[1], m2);
        J.nwnaf[0] = J.nwnaf[1] = (unsigned char)REG_DIGITS;
    }
#else
    J.nwnaf[0] = (unsigned char)wnaf4(J.wnaf[0], m1);
    J.nwnaf[1] = (unsigned char)wnaf4(J.wnaf[1], m2);
#endif
}

template <bool DER, bool W4>
__global__ __launch_bounds__(256) void ecdsa_prep_kernel(Job* __restrict__ jobs, const unsigned char* __restrict__ msg,
                                                         const unsigned char* __restrict__ sig,
                                                         const unsigned char* __restrict__ pub, int n) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= n) return;
    prep_one<DER, W4>(jobs[idx], msg, sig, pub, idx);
}

__global__ __launch_bounds__(WG, 2) void ecdsa_verify_kernel(const Job* __restrict__ jobs, const uint32_t* __restrict__ gtab,
                                                          uint8_t* __restrict__ out, int n) {
    // word-major layout: lane-consecutive words -> conflict-free LDS access
    constexpr bool AFF = BCP_ECDSA_AFFINE_TABLE;
    __shared__ uint32_t preX[NPRE][8][WG], preY[NPRE][8][WG], preZ[AFF ? 1 : NPRE][8][AFF ? 1 : WG];
    const int tid = threadIdx.x;
    const int idx = blockIdx.x * WG + tid;
    if (idx >= n) return;
    const Job& J = jobs[idx];

    // ---- decompress Q
    fe qx, qy;
    load_be32(qx, J.pub + 1);
    bool ok = (J.pub[0] == 2 || J.pub[0] == 3) && fe_lt_p(qx);
    fe y2, seven;
#pragma unroll
    for (int i = 0; i < 8; i++) seven.v[i] = i == 0 ? 7u : 0u;
    fe_sqr(y2, qx);
    fe_mul(y2, y2, qx);
    fe_add(y2, y2, seven);
    ok = ok && fe_sqrt(qy, y2);
    fe_normalize(qy); // the parity of the canonical root
    if ((qy.v[0] & 1) != (uint32_t)(J.pub[0] & 1)) {
        fe zero;
#pragma unroll
        for (int i = 0; i < 8; i++) zero.v[i] = 0;
        fe_sub(qy, zero, qy);
    }

    // ---- odd multiples Q, 3Q, 5Q, 7Q (Jacobian) into LDS
    gej q1;
    q1.x = qx;
    q1.y = qy;
#pragma unroll
    for (int i = 0; i < 8; i++) q1.z.v[i] = i == 0 ? 1u : 0u;
    q1.inf = false;
    gej q2;
    gej_double(q2, q1);
    gej cur = q1;
    if constexpr (AFF) {
        // Q, 3Q, 5Q, 7Q in Jacobian, then all four Z inverted with one inversion (Montgomery's
        // trick) and stored affine: x = X/Z^2, y = Y/Z^3
        gej mult[NPRE];
        mult[0] = q1;
#pragma unroll
        for (int m = 1; m < NPRE; m++) gej_add(mult[m], mult[m - 1], q2);
        fe pre[NPRE], inv;
        pre[0] = mult[0].z;
#pragma unroll
        for (int m = 1; m < NPRE; m++) fe_mul(pre[m], pre[m - 1], mult[m].z);
        fe_inv(inv, pre[NPRE - 1]);
#pragma unroll
        for (int m = NPRE - 1; m >= 0; m--) {
            fe zi, zi2, zi3, ax, ay;
            if (m > 0) {
                fe_mul(zi, inv, pre[m - 1]);
                fe_mul(inv, inv, mult[m].z);
            } else {
                zi = inv;
            }
            fe_sqr(zi2, zi);
            fe_mul(zi3, zi2, zi);
            fe_mul(ax, mult[m].x, zi2);
            fe_mul(ay, mult[m].y, zi3);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                preX[m][k][tid] = ax.v[k];
                preY[m][k][tid] = ay.v[k];
            }
        }
    } else {
        for (int m = 0; m < NPRE; m++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                preX[m][k][tid] = cur.x.v[k];
                preY[m][k][tid] = cur.y.v[k];
                preZ[m][k][tid] = cur.z.v[k];
            }
            gej nx;
            gej_add(nx, cur, q2);
            cur = nx;
        }
    }

    // ---- u2*Q = k1*Q + k2*(lambda Q), both halves by interleaved width-4 wNAF; lambda*Q's
    //      multiples are Q's with X scaled by beta (same Y, Z)
    fe beta;
#pragma unroll
    for (int i = 0; i < 8; i++) beta.v[i] = GLV_BETA[i];
    gej acc;
    acc.inf = true;
    // signed multiple dg (odd, |dg| <= 7) of half h's point: m = |dg| >> 1 indexes Q, 3Q, 5Q, 7Q;
    // half 1 scales X by beta; the sign combines the digit's and the GLV half's (J.neg)
    auto add_multiple = [&](int h, int dg) {
        const int m = (dg > 0 ? dg : -dg) >> 1;
        gej p;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            p.x.v[k] = preX[m][k][tid];
            p.y.v[k] = preY[m][k][tid];
            if constexpr (!AFF) p.z.v[k] = preZ[m][k][tid];
        }
        p.inf = false;
        if (h == 1) fe_mul(p.x, p.x, beta);
        if ((dg < 0) != (J.neg[h] != 0)) {
            fe zero;
#pragma unroll
            for (int i = 0; i < 8; i++) zero.v[i] = 0;
            fe_sub(p.y, zero, p.y);
        }
        gej s;
        if constexpr (AFF)
            gej_add_ge(s, acc, p.x, p.y);
        else
            gej_add(s, acc, p);
        acc = s;
    };
#if BCP_ECDSA_REGULAR
    // ---- u2*Q = k1*Q + k2*(lambda Q): 44 regular window-3 digits per half, the same
    //      positions in every lane (3 doublings + 2 additions per digit, no divergence)
    for (int b = REG_DIGITS - 1; b >= 0; b--) {
        if (b < REG_DIGITS - 1) {
#pragma unroll
            for (int t = 0; t < 3; t++) {
                gej d;
                gej_double(d, acc);
                acc = d;
            }
        }
        add_multiple(0, wnaf_digit(J, 0, b));
        add_multiple(1, wnaf_digit(J, 1, b));
    }
    // halves that were even were encoded as k + 1: subtract their point once
    for (int h = 0; h < 2; h++)
        if (J.pad[h]) add_multiple(h, -1);
#else
    // ---- u2*Q = k1*Q + k2*(lambda Q), both halves by interleaved width-4 wNAF; lambda*Q's
    //      multiples are Q's with X scaled by beta (same Y, Z)
    const int len = max((int)J.nwnaf[0], (int)J.nwnaf[1]);
    for (int b = len - 1; b >= 0; b--) {
        gej d;
        gej_double(d, acc);
        acc = d;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int dg = wnaf_digit(J, h, b);
            if (dg) add_multiple(h, dg);
        }
    }
#endif

    // ---- + u1*G via byte-window comb table (affine, 16 words per entry)
    for (int i = 0; i < 32; i++) {
        const unsigned byte = J.u1[31 - i];
        if (!byte) continue;
        const uint32_t* e = gtab + ((size_t)i * 256 + byte) * 16;
        fe gx, gy;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            gx.v[k] = e[k];
            gy.v[k] = e[8 + k];
        }
        gej s;
        gej_add_ge(s, acc, gx, gy);
        acc = s;
    }

    // ---- x(R) == r (mod n) without inversion
    bool match = false;
    if (!acc.inf) {
        fe z2, rz, r;
        fe_sqr(z2, acc.z);
        load_be32(r, J.r);
        fe_mul(rz, r, z2);
        match = fe_eq(rz, acc.x);
        if (!match && J.rplusn_ok) {
            load_be32(r, J.rn);
            fe_mul(rz, r, z2);
            match = fe_eq(rz, acc.x);
        }
    }
    out[idx] = (ok && match && J.scalar_ok) ? 1 : 0;
}

// ------------------------------------------------------------------ 10 x 26 kernels
// Shared by the fused latency kernel and the one-lane-per-signature throughput kernel below:
// field elements are 10 x 26-bit limbs (fe10.h: products with per-column ILP, carry-free
// additions), Q's odd multiples Q..15Q are made "affine" without an inversion (they live on the
// isomorphic curve scaled by one global z, libsecp256k1's globalz table, whose factor multiplies
// the ladder's final z), and u2 is walked in regular window-4 digits (33 per GLV half: 128
// doublings and 33 additions per half).
using FE = f10::fe;
using GJ = f10::gej;

__device__ __forceinline__ void f10_load_words(f10::fe& r, const uint32_t* w) {
    uint32_t t[8];
#pragma unroll
    for (int k = 0; k < 8; k++) t[k] = w[k];
    f10::from_words(r, t);
}
__device__ __forceinline__ void f10_from_be32(f10::fe& r, const unsigned char* b) {
    fe t;
    load_be32(t, b);
    f10::from_words(r, t.v);
}

// compressed key -> (x, y) with y's parity from the prefix; false if it does not decode
__device__ __forceinline__ bool f10_decompress(FE& qx, FE& qy, const unsigned char* pk) {
    fe qx8;
    load_be32(qx8, pk + 1);
    bool ok = (pk[0] == 2 || pk[0] == 3) && fe_lt_p(qx8);
    FE t;
    f10::from_words(qx, qx8.v);
    f10::sqr(t, qx);
    f10::mul(t, t, qx);
    t.n[0] += 7;
    ok = f10::sqrt_var(qy, t) && ok;
    f10::normalize(qy);
    if ((qy.n[0] & 1u) != (uint32_t)(pk[0] & 1)) {
        f10::neg(qy, qy, 2);
        f10::norm(qy);
    }
    return ok;
}

// Q, 3Q, .., 15Q into tab(m, c, k) (m: multiple, c: 0 = x, 1 = y, k: limb), every x times bmul
// (1, or beta for lambda*Q). Returns the global z.
//   2Q = d is made affine on the curve scaled by zeta = z(d): Q becomes (x zeta^2, y zeta^3),
//   each next multiple is one mixed addition of d, and each entry is brought to the last one's z
//   through the additions' z ratios (s = z(15Q) / z(iQ)): (x s^2, y s^3).
template <class Tab>
__device__ __forceinline__ FE f10_odd_multiples(const FE& qx, const FE& qy, const FE& bmul, Tab&& tab) {
    using namespace f10;
    GJ q1, d;
    q1.x = qx;
    q1.y = qy;
    set_int(q1.z, 1);
    q1.inf = false;
    dbl(d, q1);
    FE z2, z3;
    sqr(z2, d.z);
    mul(z3, z2, d.z);
    GJ cur;
    mul(cur.x, qx, z2);
    mul(cur.y, qy, z3);
    set_int(cur.z, 1);
    cur.inf = false;
    auto put = [&](int m, const FE& x, const FE& y) {
#pragma unroll
        for (int k = 0; k < 10; k++) {
            tab(m, 0, k) = x.n[k];
            tab(m, 1, k) = y.n[k];
        }
    };
    put(0, cur.x, cur.y);
    FE rr[NPRE4 - 1]; // z ratios (2i+3)Q / (2i+1)Q
#pragma unroll
    for (int i = 0; i < NPRE4 - 1; i++) {
        GJ nx;
        add_ge(nx, cur, d.x, d.y, &rr[i]);
        cur = nx;
        put(i + 1, cur.x, cur.y);
    }
    FE zg;
    mul(zg, d.z, cur.z);
    FE sc = rr[NPRE4 - 2];
#pragma unroll
    for (int i = NPRE4 - 2; i >= 0; i--) {
        FE x, y, s2, s3;
#pragma unroll
        for (int k = 0; k < 10; k++) {
            x.n[k] = tab(i, 0, k);
            y.n[k] = tab(i, 1, k);
        }
        sqr(s2, sc);
        mul(s3, s2, sc);
        mul(x, x, s2);
        mul(y, y, s3);
        mul(x, x, bmul);
        put(i, x, y);
        if (i > 0) mul(sc, sc, rr[i - 1]);
    }
    FE x;
#pragma unroll
    for (int k = 0; k < 10; k++) x.n[k] = tab(NPRE4 - 1, 0, k);
    mul(x, x, bmul);
#pragma unroll
    for (int k = 0; k < 10; k++) tab(NPRE4 - 1, 0, k) = x.n[k];
    return zg;
}

// acc += dg * P (dg odd, |dg| <= 15) from the table; flip: the half's sign; bmul: x factor applied
// per addition (nullptr: none)
template <class Tab>
__device__ __forceinline__ void f10_add_digit(GJ& acc, int dg, bool hneg, Tab&& tab, const FE* bmul) {
    using namespace f10;
    const int m = ((dg < 0 ? -dg : dg) >> 1) & (NPRE4 - 1);
    FE tx, ty, ny;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        tx.n[k] = tab(m, 0, k);
        ty.n[k] = tab(m, 1, k);
    }
    if (bmul) mul(tx, tx, *bmul);
    neg(ny, ty, 2);
    const bool flip = (dg < 0) != hneg;
#pragma unroll
    for (int k = 0; k < 10; k++) ty.n[k] = flip ? ny.n[k] : ty.n[k];
    GJ s;
    add_ge(s, acc, tx, ty);
    acc = s;
}

// acc += u1 * G by the 11-bit comb (gtab11: 24 windows x 2048 affine entries): windows [w0, w1)
constexpr int G11_WINDOWS = 24;
__device__ __forceinline__ void f10_gcomb11(GJ& acc, const unsigned char* u1be, const uint32_t* __restrict__ gtab11,
                                            int w0, int w1) {
    fe u;
    load_be32(u, u1be); // little-endian words
    for (int i = w0; i < w1; i++) {
        const int bit = 11 * i, q = bit >> 5, sh = bit & 31;
        const uint32_t lo = u.v[q], hi = q + 1 < 8 ? u.v[q + 1] : 0u;
        const unsigned win = (unsigned)(((uint64_t)hi << 32 | lo) >> sh) & 2047u;
        if (!win) continue;
        const uint32_t* e = gtab11 + ((size_t)i * 2048 + win) * 16;
        FE gx, gy;
        f10_load_words(gx, e);
        f10_load_words(gy, e + 8);
        GJ s;
        f10::add_ge(s, acc, gx, gy);
        acc = s;
    }
}

// x(R) == r (mod n), without an inversion: X == r Z^2 or (r + n) Z^2 when r + n < p
__device__ __forceinline__ bool f10_check_r(const GJ& R, const Job& J) {
    using namespace f10;
    if (R.inf) return false;
    FE z2, r, rz, dlt;
    sqr(z2, R.z);
    f10_from_be32(r, J.r);
    mul(rz, r, z2);
    sub(dlt, R.x, rz, 2);
    norm(dlt);
    if (is_zero(dlt)) return true;
    if (!J.rplusn_ok) return false;
    f10_from_be32(r, J.rn);
    mul(rz, r, z2);
    sub(dlt, R.x, rz, 2);
    norm(dlt);
    return is_zero(dlt);
}

__device__ __forceinline__ FE f10_beta() {
    uint32_t bw[8];
#pragma unroll
    for (int k = 0; k < 8; k++) bw[k] = GLV_BETA[k];
    FE b;
    f10::from_words(b, bw);
    return b;
}

// ------------------------------------------------------------------ fused latency kernel
// Small batches leave most SIMDs idle and each wave alone on its SIMD, so the verify time is
// the latency of one lane's chain of field operations. This kernel shortens that chain:
//   * one 192-thread workgroup per 64 signatures; wave 0 runs the scalar work (prep_one: s^-1,
//     u1, u2, GLV split, recoding) while waves 1-2 decompress the keys and build the tables,
//     so the prep and the square root overlap instead of running as two kernels;
//   * waves 1-2 give each GLV half of u2*Q its own lane (lanes 0-31: k1*Q, 32-63: k2*lambdaQ),
//     halving the additions on the critical path, while wave 0 runs the u1*G comb.
// Wave 0 adds the three partial points and checks x(R) == r.
constexpr int FWG = 192;
constexpr int FSIG = 64; // signatures per workgroup

template <bool DER>
__global__ __launch_bounds__(FWG) void ecdsa_fused_kernel(const unsigned char* __restrict__ msg,
                                                          const unsigned char* __restrict__ sig,
                                                          const unsigned char* __restrict__ pub,
                                                          const uint32_t* __restrict__ gtab11, uint8_t* __restrict__ out,
                                                          int n) {
    __shared__ Job sj[FSIG];
    __shared__ uint32_t tab[2][NPRE4][2][10][64]; // ladder wave, multiple, x|y, limb, lane
    __shared__ uint32_t res[2][3][10][64];        // ladder wave, x|y|z, limb, lane
    __shared__ unsigned char rflag[2][64];        // bit 0: point at infinity, bit 1: key decoded
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int base = blockIdx.x * FSIG;
    GJ acc; // wave 0: u1*G; waves 1-2: one GLV half of u2*Q
    FE zg;
    bool ok = false;
    if (wave == 0) {
        prep_one<DER, true>(sj[lane], msg, sig, pub, min(base + lane, n - 1));
    } else {
        const int w = wave - 1, slot = w * 32 + (lane & 31), half = lane >> 5;
        FE qx, qy;
        ok = f10_decompress(qx, qy, pub + (size_t)min(base + slot, n - 1) * 33);
        FE bmul;
        if (half) bmul = f10_beta();
        else f10::set_int(bmul, 1);
        zg = f10_odd_multiples(qx, qy, bmul, [&](int m, int c, int k) -> uint32_t& { return tab[w][m][c][k][lane]; });
    }
    __syncthreads();
    if (wave == 0) {
        acc.inf = true;
        f10_gcomb11(acc, sj[lane].u1, gtab11, 0, G11_WINDOWS);
    } else {
        const int w = wave - 1, slot = w * 32 + (lane & 31), half = lane >> 5;
        const Job& J = sj[slot];
        const bool hneg = J.neg[half] != 0;
        auto tb = [&](int m, int c, int k) -> uint32_t& { return tab[w][m][c][k][lane]; };
        acc.inf = true;
#pragma unroll 1
        for (int b = REG4_DIGITS - 1; b >= 0; b--) {
            if (b < REG4_DIGITS - 1) {
#pragma unroll 1
                for (int t = 0; t < 4; t++) {
                    GJ d;
                    f10::dbl(d, acc);
                    acc = d;
                }
            }
            f10_add_digit(acc, reg4_digit(J, half, b), hneg, tb, nullptr);
        }
        if (J.pad[half]) f10_add_digit(acc, -1, hneg, tb, nullptr); // an even half was encoded as k + 1
        FE z;
        f10::mul(z, acc.z, zg);
#pragma unroll
        for (int k = 0; k < 10; k++) {
            res[w][0][k][lane] = acc.x.n[k];
            res[w][1][k][lane] = acc.y.n[k];
            res[w][2][k][lane] = z.n[k];
        }
        rflag[w][lane] = (unsigned char)((acc.inf ? 1 : 0) | (ok ? 2 : 0));
    }
    __syncthreads();
    if (wave != 0 || base + lane >= n) return;
    const Job& J = sj[lane];
    const int w = lane >> 5, l0 = lane & 31;
    ok = (rflag[w][l0] & 2) != 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int l = l0 + 32 * h;
        GJ q;
#pragma unroll
        for (int k = 0; k < 10; k++) {
            q.x.n[k] = res[w][0][k][l];
            q.y.n[k] = res[w][1][k][l];
            q.z.n[k] = res[w][2][k][l];
        }
        q.inf = (rflag[w][l] & 1) != 0;
        GJ s;
        f10::add_gej(s, acc, q);
        acc = s;
    }
    out[base + lane] = (ok && f10_check_r(acc, J) && J.scalar_ok) ? 1 : 0;
}

// ------------------------------------------------------------------ throughput kernel, 10 x 26
// One lane per signature after ecdsa_prep_kernel<DER, true>, like ecdsa_verify_kernel, with the
// 10 x 26 field, the global-z table (x, y only in LDS: 640 B per lane) and window-4 digits.
// Both GLV halves share one accumulator (4 doublings and 2 additions per digit; the lambda half
// scales x by beta per addition); then z is moved back to the original curve and u1*G is added
// by the byte comb.
constexpr int WG10 = 64;
__global__ __launch_bounds__(WG10) void ecdsa_verify10_kernel(const Job* __restrict__ jobs,
                                                              const uint32_t* __restrict__ gtab11,
                                                              uint8_t* __restrict__ out, int n) {
    __shared__ uint32_t tab[NPRE4][2][10][WG10];
    const int tid = threadIdx.x;
    const int idx = blockIdx.x * WG10 + tid;
    if (idx >= n) return;
    const Job& J = jobs[idx];
    FE qx, qy, one;
    const bool ok = f10_decompress(qx, qy, J.pub);
    f10::set_int(one, 1);
    auto tb = [&](int m, int c, int k) -> uint32_t& { return tab[m][c][k][tid]; };
    const FE zg = f10_odd_multiples(qx, qy, one, tb);
    const FE beta = f10_beta();
    const bool hneg0 = J.neg[0] != 0, hneg1 = J.neg[1] != 0;
    GJ acc;
    acc.inf = true;
#pragma unroll 1
    for (int b = REG4_DIGITS - 1; b >= 0; b--) {
        if (b < REG4_DIGITS - 1) {
#pragma unroll 1
            for (int i = 0; i < 4; i++) {
                GJ d;
                f10::dbl(d, acc);
                acc = d;
            }
        }
        f10_add_digit(acc, reg4_digit(J, 0, b), hneg0, tb, nullptr);
        f10_add_digit(acc, reg4_digit(J, 1, b), hneg1, tb, &beta);
    }
    if (J.pad[0]) f10_add_digit(acc, -1, hneg0, tb, nullptr);
    if (J.pad[1]) f10_add_digit(acc, -1, hneg1, tb, &beta);
    {
        FE z;
        f10::mul(z, acc.z, zg); // back to the original curve
        acc.z = z;
    }
    f10_gcomb11(acc, J.u1, gtab11, 0, G11_WINDOWS);
    out[idx] = (ok && f10_check_r(acc, J) && J.scalar_ok) ? 1 : 0;
}

// The same work with one GLV half per lane (32 signatures per wave): lanes 0-31 run k1*Q plus
// comb windows 0-11, lanes 32-63 k2*lambdaQ plus windows 12-23, and lane l adds lane l+32's point.
// A wave takes about two thirds of ecdsa_verify10_kernel's time for half the signatures: the
// launcher gives it the last, partly filled round of a batch (at most half a round), which the
// one-lane kernel would stretch to a whole round (199,680 signatures = 3.05 rounds of 65,536).
__global__ __launch_bounds__(WG10) void ecdsa_verify10h_kernel(const Job* __restrict__ jobs,
                                                               const uint32_t* __restrict__ gtab11,
                                                               uint8_t* __restrict__ out, int lo, int n) {
    // lanes 32-63 hand their points over through the table's LDS once the table is dead (40 KiB
    // per workgroup in all: 4 workgroups, one wave per SIMD, per CU)
    __shared__ uint32_t tab[NPRE4][2][10][WG10];
    uint32_t(&xr)[3][10][32] = *reinterpret_cast<uint32_t(*)[3][10][32]>(&tab[0][0][0][0]);
    unsigned char* xinf = reinterpret_cast<unsigned char*>(&tab[0][0][0][0]) + sizeof(xr);
    const int tid = threadIdx.x, half = tid >> 5, l0 = tid & 31;
    const int idx = min(lo + (int)blockIdx.x * 32 + l0, n - 1); // past n: recompute the last one
    const Job& J = jobs[idx];
    FE qx, qy, bmul;
    const bool ok = f10_decompress(qx, qy, J.pub);
    if (half) bmul = f10_beta();
    else f10::set_int(bmul, 1);
    auto tb = [&](int m, int c, int k) -> uint32_t& { return tab[m][c][k][tid]; };
    const FE zg = f10_odd_multiples(qx, qy, bmul, tb);
    const bool hneg = J.neg[half] != 0;
    GJ acc;
    acc.inf = true;
#pragma unroll 1
    for (int b = REG4_DIGITS - 1; b >= 0; b--) {
        if (b < REG4_DIGITS - 1) {
#pragma unroll 1
            for (int i = 0; i < 4; i++) {
                GJ d;
                f10::dbl(d, acc);
                acc = d;
            }
        }
        f10_add_digit(acc, reg4_digit(J, half, b), hneg, tb, nullptr);
    }
    if (J.pad[half]) f10_add_digit(acc, -1, hneg, tb, nullptr);
    {
        FE z;
        f10::mul(z, acc.z, zg);
        acc.z = z;
    }
    f10_gcomb11(acc, J.u1, gtab11, 12 * half, 12 * half + 12);
    __syncthreads(); // every lane is past its last table read
    if (half) {
#pragma unroll
        for (int k = 0; k < 10; k++) {
            xr[0][k][l0] = acc.x.n[k];
            xr[1][k][l0] = acc.y.n[k];
            xr[2][k][l0] = acc.z.n[k];
        }
        xinf[l0] = acc.inf ? 1 : 0;
    }
    __syncthreads();
    if (half || lo + (int)blockIdx.x * 32 + l0 >= n) return;
    GJ q, s;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        q.x.n[k] = xr[0][k][l0];
        q.y.n[k] = xr[1][k][l0];
        q.z.n[k] = xr[2][k][l0];
    }
    q.inf = xinf[l0] != 0;
    f10::add_gej(s, acc, q);
    out[idx] = (ok && f10_check_r(s, J) && J.scalar_ok) ? 1 : 0;
}

// Generator comb table, one per HIP device (read-only once built, shared by every lane).
struct Table {
    std::once_flag once;
    uint32_t* d_gtab = nullptr;   // 8-bit comb (ecdsa_verify_kernel)
    uint32_t* d_gtab11 = nullptr; // 11-bit comb (the 10 x 26 kernels)
};
constexpr int MAX_DEVICES = 64;
Table& T(int device) {
    static Table t[MAX_DEVICES];
    if (device < 0 || device >= MAX_DEVICES) throw std::runtime_error("EcdsaVerifyBatch: device id out of range");
    return t[device];
}

// Builds the table on the current device (the caller made `tb`'s device current).
// affine points as 8 LE limbs of x then 8 of y (the point at infinity stays zero, never read)
std::vector<uint32_t> TableWords(const std::vector<secp::Ge>& t) {
    std::vector<uint32_t> h(t.size() * 16, 0);
    for (size_t e = 0; e < t.size(); e++) {
        unsigned char bx[32], by[32];
        if (t[e].inf) continue;
        secp::fe_get_b32(bx, t[e].x);
        secp::fe_get_b32(by, t[e].y);
        for (int k = 0; k < 8; k++) {
            const unsigned char* q = bx + 28 - 4 * k;
            h[e * 16 + k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
            q = by + 28 - 4 * k;
            h[e * 16 + 8 + k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
        }
    }
    return h;
}

// Builds the tables on the current device (the caller made `tb`'s device current).
void InitTable(Table& tb) {
    const std::vector<uint32_t> h = TableWords(secp::generator_table());     // 32 x 256
    const std::vector<uint32_t> h11 = TableWords(secp::generator_table11()); // 24 x 2048
    BCP_HIP_CHECK(hipMalloc(&tb.d_gtab, h.size() * 4));
    BCP_HIP_CHECK(hipMemcpy(tb.d_gtab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    BCP_HIP_CHECK(hipMalloc(&tb.d_gtab11, h11.size() * 4));
    BCP_HIP_CHECK(hipMemcpy(tb.d_gtab11, h11.data(), h11.size() * 4, hipMemcpyHostToDevice));
}

} // namespace

// Host: pack z / (r,s) / key into the lane's pinned staging (one H2D copy); the prep kernel builds
// the Jobs and does all scalar arithmetic; one D2H copy of the verdicts.
void VerifyLane::Ecdsa(const unsigned char* msg32, const unsigned char* sig64, const unsigned char* pub33, size_t n,
                       uint8_t* result) {
    EcdsaFill(
        n,
        [&](unsigned char* m, unsigned char* s, unsigned char* p) {
            memcpy(m, msg32, n * 32);
            memcpy(s, sig64, n * 64);
            memcpy(p, pub33, n * 33);
        },
        result);
}

std::atomic<size_t> g_fusedMax{BCP_ECDSA_FUSED_MAX};
std::atomic<int> g_splitKernel{BCP_ECDSA_SPLIT_KERNEL};

namespace {
// compute units of the current device (cached per device)
int DeviceCUs() {
    static std::atomic<int> cus[MAX_DEVICES];
    int dev = 0;
    BCP_HIP_CHECK(hipGetDevice(&dev));
    if (dev < 0 || dev >= MAX_DEVICES) return 256;
    int c = cus[dev].load(std::memory_order_relaxed);
    if (!c) {
        BCP_HIP_CHECK(hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev));
        cus[dev].store(c, std::memory_order_relaxed);
    }
    return c;
}
// Batches up to EcdsaFusedMax() run the fused latency kernel (no job records); larger ones the
// prep + verify throughput pair.
void LaunchVerify(bool der, const unsigned char* dm, const unsigned char* ds, const unsigned char* dp, Job* d_jobs,
                  const Table& tb, uint8_t* d_out, size_t n, hipStream_t stream) {
    const uint32_t* gtab = tb.d_gtab;
    const uint32_t* gtab11 = tb.d_gtab11;
    if (n <= g_fusedMax.load(std::memory_order_relaxed)) {
        const dim3 fg((unsigned)((n + FSIG - 1) / FSIG));
        if (der) hipLaunchKernelGGL(ecdsa_fused_kernel<true>, fg, dim3(FWG), 0, stream, dm, ds, dp, gtab11, d_out, (int)n);
        else hipLaunchKernelGGL(ecdsa_fused_kernel<false>, fg, dim3(FWG), 0, stream, dm, ds, dp, gtab11, d_out, (int)n);
        BCP_HIP_CHECK(hipGetLastError());
        return;
    }
    const dim3 pg((unsigned)((n + 255) / 256));
    const int sk = g_splitKernel.load(std::memory_order_relaxed);
    const bool k10 = sk != 0; // window-4 digits for the 10 x 26 kernels
    if (der && k10) hipLaunchKernelGGL((ecdsa_prep_kernel<true, true>), pg, dim3(256), 0, stream, d_jobs, dm, ds, dp, (int)n);
    else if (der) hipLaunchKernelGGL((ecdsa_prep_kernel<true, false>), pg, dim3(256), 0, stream, d_jobs, dm, ds, dp, (int)n);
    else if (k10) hipLaunchKernelGGL((ecdsa_prep_kernel<false, true>), pg, dim3(256), 0, stream, d_jobs, dm, ds, dp, (int)n);
    else hipLaunchKernelGGL((ecdsa_prep_kernel<false, false>), pg, dim3(256), 0, stream, d_jobs, dm, ds, dp, (int)n);
    BCP_HIP_CHECK(hipGetLastError());
    if (k10) {
        // one-lane kernel for whole rounds (one wave per SIMD: CUs x 4 x 64 signatures), the
        // half-lane kernel for a last round at most half full
        const size_t round = (size_t)DeviceCUs() * 4 * 64;
        size_t nf = n / round * round;
        if (n - nf > round / 2) nf = n;
        if (sk == 2) nf = n; // pinned: one-lane kernel only
        if (sk == 3) nf = 0; // pinned: half-lane kernel only
        if (nf)
            hipLaunchKernelGGL(ecdsa_verify10_kernel, dim3((unsigned)((nf + WG10 - 1) / WG10)), dim3(WG10), 0, stream,
                               d_jobs, gtab11, d_out, (int)nf);
        if (nf < n)
            hipLaunchKernelGGL(ecdsa_verify10h_kernel, dim3((unsigned)((n - nf + 31) / 32)), dim3(WG10), 0, stream,
                               d_jobs, gtab11, d_out, (int)nf, (int)n);
    } else
        hipLaunchKernelGGL(ecdsa_verify_kernel, dim3((unsigned)((n + WG - 1) / WG)), dim3(WG), 0, stream, d_jobs, gtab,
                           d_out, (int)n);
    BCP_HIP_CHECK(hipGetLastError());
}
} // namespace

void SetEcdsaFusedMax(size_t n) { g_fusedMax.store(n, std::memory_order_relaxed); }
void SetEcdsaSplitKernel(int k) { g_splitKernel.store(k >= 0 && k <= 3 ? k : 1, std::memory_order_relaxed); }
int EcdsaSplitKernel() { return g_splitKernel.load(std::memory_order_relaxed); }
size_t EcdsaFusedMax() { return g_fusedMax.load(std::memory_order_relaxed); }

namespace {
// Shared by EcdsaFill (compact sigs, sigBytes 64) and EcdsaDerFill (DER slots): staging is
// msg n x 32 | sig n x sigBytes | pub n x 33, one H2D copy, prep + verify, one D2H copy.
void LaneEcdsa(LaneState& L, size_t n, size_t sigBytes,
               const std::function<void(unsigned char*, unsigned char*, unsigned char*)>& fill, uint8_t* result) {
    if (n == 0) return;
    BCP_HIP_CHECK(hipSetDevice(L.device));
    Table& tb = T(L.device);
    // a throwing init leaves the once_flag unset, so the next call retries it
    std::call_once(tb.once, [&] { InitTable(tb); });
    const size_t bytes = n * (32 + sigBytes + 33);
    unsigned char* h_in = L.Host(0, bytes);
    uint8_t* h_out = L.Host(1, n);
    const auto t0 = std::chrono::steady_clock::now();
    fill(h_in, h_in + n * 32, h_in + n * (32 + sigBytes));
    const auto t1 = std::chrono::steady_clock::now();
    unsigned char* d_in = L.Dev(0, bytes);
    Job* d_jobs = reinterpret_cast<Job*>(L.Dev(1, n * sizeof(Job)));
    uint8_t* d_out = L.Dev(2, n);
    BCP_HIP_CHECK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, L.stream));
    const unsigned char *dm = d_in, *ds = d_in + n * 32, *dp = d_in + n * (32 + sigBytes);
    LaunchVerify(sigBytes != 64, dm, ds, dp, d_jobs, tb, d_out, n, L.stream);
    BCP_HIP_CHECK(hipMemcpyAsync(h_out, d_out, n, hipMemcpyDeviceToHost, L.stream));
    BCP_HIP_CHECK(hipStreamSynchronize(L.stream));
    memcpy(result, h_out, n);
    const auto t2 = std::chrono::steady_clock::now();
    L.fillMicros += std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
    L.deviceMicros += std::chrono::duration_cast<std::chrono::microseconds>(t2 - t1).count();
    L.batches++;
    L.items += n;
}
} // namespace

void VerifyLane::EcdsaFill(size_t n, const std::function<void(unsigned char*, unsigned char*, unsigned char*)>& fill,
                           uint8_t* result) {
    LaneEcdsa(*impl, n, 64, fill, result);
}

void VerifyLane::EcdsaDerFill(size_t n, const std::function<void(unsigned char*, unsigned char*, unsigned char*)>& fill,
                              uint8_t* result) {
    LaneEcdsa(*impl, n, DER_SLOT, fill, result);
}

size_t EcdsaJobBytes() { return sizeof(Job); }

void EcdsaVerifyDevice(const void* msg32, const void* sig64, const void* pub33, void* jobs, void* result, size_t n,
                       int device, uintptr_t stream) {
    if (!n) return;
    if (reinterpret_cast<uintptr_t>(jobs) % alignof(Job)) throw std::invalid_argument("EcdsaVerifyDevice: job scratch alignment");
    DeviceScope ds(device);
    Table& tb = T(ds.device);
    std::call_once(tb.once, [&] { InitTable(tb); });
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    LaunchVerify(false, static_cast<const unsigned char*>(msg32), static_cast<const unsigned char*>(sig64),
                 static_cast<const unsigned char*>(pub33), static_cast<Job*>(jobs), tb,
                 static_cast<uint8_t*>(result), n, s);
}

std::vector<uint8_t> EcdsaVerifyBatch(const std::vector<unsigned char>& msg32, const std::vector<unsigned char>& sig64,
                                      const std::vector<unsigned char>& pub33, int device) {
    const size_t n = msg32.size() / 32;
    if (msg32.size() != n * 32 || sig64.size() != n * 64 || pub33.size() != n * 33)
        throw std::invalid_argument("EcdsaVerifyBatch: sizes");
    std::vector<uint8_t> result(n, 0);
    if (n == 0) return result;
    // one normal-priority lane per device for the plain batch API
    static std::mutex m;
    static std::unique_ptr<VerifyLane> lanes[MAX_DEVICES];
    static std::mutex use[MAX_DEVICES];
    const int dev = UseDevice(device);
    if (dev >= MAX_DEVICES) throw std::runtime_error("EcdsaVerifyBatch: device id out of range");
    {
        std::lock_guard<std::mutex> l(m);
        if (!lanes[dev]) lanes[dev].reset(new VerifyLane(dev, false));
    }
    std::lock_guard<std::mutex> hold(use[dev]);
    lanes[dev]->Ecdsa(msg32.data(), sig64.data(), pub33.data(), n, result.data());
    return result;
}

} // namespace gpu
} // namespace bcp
