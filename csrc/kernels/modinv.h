// 256-bit modular inverse by the binary extended Euclid algorithm, for the ECDSA kernels.
//
// The verification inputs are public, so a variable-time inverse is fine. It replaces the Fermat
// powers in the kernels (reference secp256k1 uses a constant-time exponentiation for scalars,
// src/secp256k1/src/scalar_impl.h secp256k1_scalar_inverse, and a variable-time one for
// verification, secp256k1_scalar_inverse_var). A Fermat inverse costs ~384 Montgomery products
// of 8x8 limbs (290k VALU instructions per wave in ecdsa_prep_kernel); this one about 256 steps
// of subtractions, selects and one 32x256-bit multiply-shift.
//
// Step (invariants: xa * a0 == a, xb * a0 == b (mod m); b odd; 0 <= a, b):
//   if a is odd: if a >= b then (a, xa) -= (b, xb), else (a, b, xa, xb) = (b - a, a, xb - xa, xa);
//   a is now even: a /= 2^k, xa /= 2^k (mod m) for its k trailing zero bits (k <= 31).
// Each step shrinks bits(a) + bits(b), so a reaches 0 within 512 steps (about 2 bits per step
// on average) and then b = gcd = 1, xb = a0^-1. The subtract/swap selects are branch-free.
//
// Host-compilable: the host unit test (csrc/test/modinv_tests.cpp) runs the same code.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define BCP_MODINV_HD __host__ __device__
#else
#define BCP_MODINV_HD
#endif

namespace bcpk {

// out = a0^-1 mod m. m odd, 0 < a0 < m, gcd(a0, m) = 1. Returns false if that did not hold
// (a0 == 0, or not coprime): out is then unspecified.
BCP_MODINV_HD inline bool modinv256(uint32_t out[8], const uint32_t a0[8], const uint32_t m[8]) {
    // minv = -m^-1 mod 2^32 (Newton: each step doubles the correct low bits of the inverse)
    uint32_t inv = m[0];
    for (int i = 0; i < 5; i++) inv *= 2u - m[0] * inv;
    const uint32_t minv = 0u - inv;
    uint32_t a[8], b[8], xa[8], xb[8];
    for (int i = 0; i < 8; i++) {
        a[i] = a0[i];
        b[i] = m[i];
        xa[i] = i == 0 ? 1u : 0u;
        xb[i] = 0;
    }
    for (int step = 0; step < 520; step++) { // each step shrinks bits(a) + bits(b) by >= 1
        uint32_t any = 0;
        for (int i = 0; i < 8; i++) any |= a[i];
        if (!any) break;
        const uint32_t odd = 0u - (a[0] & 1u);
        // d = a - b, and whether it borrowed (a < b)
        uint32_t d[8];
        uint32_t bw = 0;
        for (int i = 0; i < 8; i++) {
            const uint64_t t = (uint64_t)a[i] - b[i] - bw;
            d[i] = (uint32_t)t;
            bw = (uint32_t)(t >> 63);
        }
        const uint32_t lt = odd & (0u - bw), ge = odd & ~lt;
        // nd = b - a = -d
        uint32_t nd[8];
        uint32_t c = 1;
        for (int i = 0; i < 8; i++) {
            const uint64_t t = (uint64_t)(~d[i]) + c;
            nd[i] = (uint32_t)t;
            c = (uint32_t)(t >> 32);
        }
        // dx = xa - xb (mod m), ndx = xb - xa (mod m)
        uint32_t dx[8], ndx[8];
        uint32_t bx = 0, by = 0;
        for (int i = 0; i < 8; i++) {
            const uint64_t t = (uint64_t)xa[i] - xb[i] - bx;
            dx[i] = (uint32_t)t;
            bx = (uint32_t)(t >> 63);
            const uint64_t u = (uint64_t)xb[i] - xa[i] - by;
            ndx[i] = (uint32_t)u;
            by = (uint32_t)(u >> 63);
        }
        const uint32_t fx = 0u - bx, fy = 0u - by; // add m back where the difference went negative
        uint32_t cx = 0, cy = 0;
        for (int i = 0; i < 8; i++) {
            const uint64_t t = (uint64_t)dx[i] + (m[i] & fx) + cx;
            dx[i] = (uint32_t)t;
            cx = (uint32_t)(t >> 32);
            const uint64_t u = (uint64_t)ndx[i] + (m[i] & fy) + cy;
            ndx[i] = (uint32_t)u;
            cy = (uint32_t)(u >> 32);
        }
        for (int i = 0; i < 8; i++) {
            const uint32_t an = (ge & d[i]) | (lt & nd[i]) | (~odd & a[i]);
            const uint32_t xan = (ge & dx[i]) | (lt & ndx[i]) | (~odd & xa[i]);
            b[i] = (lt & a[i]) | (~lt & b[i]);
            xb[i] = (lt & xa[i]) | (~lt & xb[i]);
            a[i] = an;
            xa[i] = xan;
        }
        // a is even (or zero): strip all its trailing zero bits at once, k <= 31 of them, and
        // divide xa by 2^k mod m the Montgomery way: xa = (xa + t*m) / 2^k with
        // t = -xa * m^-1 mod 2^k (xa + t*m < 2^(257+k), so 9 limbs before the shift)
        const uint32_t lo = a[0];
        const uint32_t k = lo ? (uint32_t)__builtin_ctz(lo) : 31u;
        const uint32_t t = (xa[0] * minv) & ((1u << k) - 1u);
        uint32_t h[9];
        uint64_t cm = 0;
        for (int i = 0; i < 8; i++) {
            cm += (uint64_t)xa[i] + (uint64_t)t * m[i];
            h[i] = (uint32_t)cm;
            cm >>= 32;
        }
        h[8] = (uint32_t)cm;
        if (k) {
            for (int i = 0; i < 7; i++) {
                a[i] = (a[i] >> k) | (a[i + 1] << (32 - k));
                xa[i] = (h[i] >> k) | (h[i + 1] << (32 - k));
            }
            a[7] >>= k;
            xa[7] = (h[7] >> k) | (h[8] << (32 - k));
        }
    }
    uint32_t one = b[0] ^ 1u, rest = 0;
    for (int i = 1; i < 8; i++) rest |= b[i];
    for (int i = 0; i < 8; i++) out[i] = xb[i];
    uint32_t az = 0;
    for (int i = 0; i < 8; i++) az |= a[i];
    return (one | rest | az) == 0;
}

} // namespace bcpk
