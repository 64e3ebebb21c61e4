// secp256k1 CPU implementation. See secp256k1.h.
#include "secp256k1/secp256k1.h"
#include "crypto/hashes.h"
#include "crypto/common.h"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <mutex>
#include <stdexcept>

namespace bcp {
namespace secp {

typedef unsigned __int128 u128;

// ---------------------------------------------------------------- field
static const uint64_t P[4] = {0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL};
static const uint64_t PC = 0x1000003D1ULL; // 2^256 - p

static inline bool geq4(const uint64_t* a, const uint64_t* b) {
    for (int i = 3; i >= 0; --i) {
        if (a[i] != b[i]) return a[i] > b[i];
    }
    return true;
}
static inline uint64_t sub4(uint64_t* r, const uint64_t* a, const uint64_t* b) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a[i] - b[i] - borrow;
        r[i] = (uint64_t)d;
        borrow = (uint64_t)(d >> 127) & 1;
    }
    return borrow;
}
static inline uint64_t add4(uint64_t* r, const uint64_t* a, const uint64_t* b) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
        c += (u128)a[i] + b[i];
        r[i] = (uint64_t)c;
        c >>= 64;
    }
    return (uint64_t)c;
}

// Branch-free helpers: every field and scalar operation below runs the same instruction
// sequence for every input (secret keys and nonces pass through them when signing).
static inline uint64_t mask_of(uint64_t bit) { return (uint64_t)0 - bit; } // 0 or all-ones
static inline void cmov4(uint64_t* r, const uint64_t* a, uint64_t mask) {
    for (int i = 0; i < 4; ++i) r[i] = (r[i] & ~mask) | (a[i] & mask);
}
// r -= m when r >= m (one conditional subtraction, no branch)
static inline void csub4(uint64_t* r, const uint64_t* m) {
    uint64_t t[4];
    const uint64_t borrow = sub4(t, r, m);
    cmov4(r, t, mask_of(borrow ^ 1));
}
// r += c * PC over all four limbs (c in {0, 1})
static inline uint64_t add_pc(uint64_t* r, uint64_t c) {
    u128 t = (u128)r[0] + (PC & mask_of(c));
    r[0] = (uint64_t)t;
    for (int i = 1; i < 4; ++i) {
        t = (u128)r[i] + (uint64_t)(t >> 64);
        r[i] = (uint64_t)t;
    }
    return (uint64_t)(t >> 64);
}

static inline void fe_reduce_once(uint64_t* r) { csub4(r, P); }

void fe_set_b32(Fe& r, const unsigned char* b, bool* overflow) {
    for (int i = 0; i < 4; ++i) {
        uint64_t v = 0;
        for (int j = 0; j < 8; ++j) v = (v << 8) | b[(3 - i) * 8 + j];
        r.n[i] = v;
    }
    uint64_t t[4];
    const uint64_t of = sub4(t, r.n, P) ^ 1;
    cmov4(r.n, t, mask_of(of));
    if (overflow) *overflow = of;
}
void fe_get_b32(unsigned char* b, const Fe& a) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (unsigned char)(a.n[i] >> (56 - 8 * j));
}
void fe_set_int(Fe& r, uint64_t v) { r.n[0] = v; r.n[1] = r.n[2] = r.n[3] = 0; }
bool fe_is_zero(const Fe& a) { return (a.n[0] | a.n[1] | a.n[2] | a.n[3]) == 0; }
bool fe_equal(const Fe& a, const Fe& b) { return memcmp(a.n, b.n, 32) == 0; }
bool fe_is_odd(const Fe& a) { return a.n[0] & 1; }
// all-ones when a == 0 (branch-free)
static inline uint64_t fe_zero_mask(const Fe& a) {
    const uint64_t x = a.n[0] | a.n[1] | a.n[2] | a.n[3];
    return mask_of(((x | ((uint64_t)0 - x)) >> 63) ^ 1);
}

void fe_add(Fe& r, const Fe& a, const Fe& b) {
    // a + b = 2^256 * c + r  ==  r + c * PC (mod p); that sum cannot carry again
    const uint64_t c = add4(r.n, a.n, b.n);
    add_pc(r.n, c);
    fe_reduce_once(r.n);
}
void fe_sub(Fe& r, const Fe& a, const Fe& b) {
    // a wrapped difference is a - b + 2^256: subtract PC to land on a - b + p
    const uint64_t borrow = sub4(r.n, a.n, b.n);
    u128 t = (u128)r.n[0] - (PC & mask_of(borrow));
    r.n[0] = (uint64_t)t;
    for (int i = 1; i < 4; ++i) {
        t = (u128)r.n[i] - ((uint64_t)(t >> 127) & 1);
        r.n[i] = (uint64_t)t;
    }
}
void fe_neg(Fe& r, const Fe& a) {
    Fe z;
    fe_set_int(z, 0);
    fe_sub(r, z, a);
}

// Reduce an 8-limb product mod p.
static void fe_reduce8(uint64_t* r, const uint64_t* t) {
    // u = lo + hi * PC   (hi * PC < 2^290)
    uint64_t u[5];
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
        c += (u128)t[i] + (u128)t[4 + i] * PC;
        u[i] = (uint64_t)c;
        c >>= 64;
    }
    u[4] = (uint64_t)c;
    // fold u[4] (<= 2^34) once more
    c = (u128)u[0] + (u128)u[4] * PC;
    r[0] = (uint64_t)c;
    c >>= 64;
    for (int i = 1; i < 4; ++i) {
        c += u[i];
        r[i] = (uint64_t)c;
        c >>= 64;
    }
    add_pc(r, (uint64_t)c); // one more 2^256 -> PC
    fe_reduce_once(r);
}

void fe_mul(Fe& r, const Fe& a, const Fe& b) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += (u128)a.n[i] * b.n[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
        t[i + 4] = (uint64_t)c;
    }
    fe_reduce8(r.n, t);
}
void fe_sqr(Fe& r, const Fe& a) { fe_mul(r, a, a); }

static void fe_pow(Fe& r, const Fe& a, const uint64_t* e) {
    Fe acc;
    fe_set_int(acc, 1);
    for (int i = 255; i >= 0; --i) {
        fe_sqr(acc, acc);
        if ((e[i / 64] >> (i % 64)) & 1) fe_mul(acc, acc, a);
    }
    r = acc;
}
// a^(2^223 - 1) and the shorter runs of ones the exponents p - 2 and (p + 1)/4 are made of:
// xk = a^(2^k - 1). 222 squarings and 11 multiplications instead of a plain square-and-multiply
// over 256 mostly-one bits (~500 operations).
struct FeRuns {
    Fe x2, x3, x22, x223;
};
static void fe_sqr_n(Fe& r, const Fe& a, int n) {
    r = a;
    for (int i = 0; i < n; ++i) fe_sqr(r, r);
}
static void fe_runs(FeRuns& R, const Fe& a) {
    Fe x6, x9, x11, x44, x88, x176, x220, t;
    fe_sqr(t, a);
    fe_mul(R.x2, t, a);
    fe_sqr(t, R.x2);
    fe_mul(R.x3, t, a);
    fe_sqr_n(t, R.x3, 3);
    fe_mul(x6, t, R.x3);
    fe_sqr_n(t, x6, 3);
    fe_mul(x9, t, R.x3);
    fe_sqr_n(t, x9, 2);
    fe_mul(x11, t, R.x2);
    fe_sqr_n(t, x11, 11);
    fe_mul(R.x22, t, x11);
    fe_sqr_n(t, R.x22, 22);
    fe_mul(x44, t, R.x22);
    fe_sqr_n(t, x44, 44);
    fe_mul(x88, t, x44);
    fe_sqr_n(t, x88, 88);
    fe_mul(x176, t, x88);
    fe_sqr_n(t, x176, 44);
    fe_mul(x220, t, x44);
    fe_sqr_n(t, x220, 3);
    fe_mul(R.x223, t, R.x3);
}
void fe_inv(Fe& r, const Fe& a) {
    // p - 2 = [223 ones] 0 [22 ones] 0000 1 0 11 0 1
    FeRuns R;
    fe_runs(R, a);
    Fe t;
    fe_sqr_n(t, R.x223, 23);
    fe_mul(t, t, R.x22);
    fe_sqr_n(t, t, 5);
    fe_mul(t, t, a);
    fe_sqr_n(t, t, 3);
    fe_mul(t, t, R.x2);
    fe_sqr_n(t, t, 2);
    fe_mul(r, t, a);
}
void fe_inv_slow(Fe& r, const Fe& a) {
    static const uint64_t PM2[4] = {0xFFFFFFFEFFFFFC2DULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL,
                                    0xFFFFFFFFFFFFFFFFULL};
    fe_pow(r, a, PM2);
}
bool fe_sqrt(Fe& r, const Fe& a) {
    // (p + 1)/4 = [223 ones] 0 [22 ones] 0000 11 00
    FeRuns R;
    fe_runs(R, a);
    Fe s, chk;
    fe_sqr_n(s, R.x223, 23);
    fe_mul(s, s, R.x22);
    fe_sqr_n(s, s, 6);
    fe_mul(s, s, R.x2);
    fe_sqr_n(s, s, 2);
    fe_sqr(chk, s);
    r = s;
    return fe_equal(chk, a);
}

// ---------------------------------------------------------------- scalar
static const uint64_t N[4] = {0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL};
static const uint64_t NC[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 0x1ULL}; // 2^256 - n
static const uint64_t NH[4] = {0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL,
                               0x7FFFFFFFFFFFFFFFULL}; // n/2

void sc_set_b32(Scalar& r, const unsigned char* b, bool* overflow) {
    for (int i = 0; i < 4; ++i) {
        uint64_t v = 0;
        for (int j = 0; j < 8; ++j) v = (v << 8) | b[(3 - i) * 8 + j];
        r.n[i] = v;
    }
    uint64_t t[4];
    const uint64_t of = sub4(t, r.n, N) ^ 1;
    cmov4(r.n, t, mask_of(of));
    if (overflow) *overflow = of;
}
void sc_get_b32(unsigned char* b, const Scalar& a) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (unsigned char)(a.n[i] >> (56 - 8 * j));
}
bool sc_is_zero(const Scalar& a) { return (a.n[0] | a.n[1] | a.n[2] | a.n[3]) == 0; }
bool sc_is_high(const Scalar& a) {
    // a > n/2  <=>  n/2 - a borrows
    uint64_t t[4];
    return sub4(t, NH, a.n) != 0;
}
void sc_add(Scalar& r, const Scalar& a, const Scalar& b) {
    const uint64_t c = add4(r.n, a.n, b.n);
    uint64_t t[4];
    const uint64_t borrow = sub4(t, r.n, N);
    // subtract n when the sum carried out of 2^256 or is >= n
    cmov4(r.n, t, mask_of(c | (borrow ^ 1)));
}
void sc_neg(Scalar& r, const Scalar& a) {
    // n - a, and 0 for a == 0
    const uint64_t x = a.n[0] | a.n[1] | a.n[2] | a.n[3];
    const uint64_t nz = mask_of((x | ((uint64_t)0 - x)) >> 63);
    uint64_t t[4];
    sub4(t, N, a.n);
    for (int i = 0; i < 4; ++i) r.n[i] = t[i] & nz;
}
// Reduce a 512-bit product mod n with a fixed sequence of operations: n = 2^256 - NC (NC < 2^129),
// so t = lo + hi * 2^256 == lo + hi * NC. Three folds bring any 512-bit value below 2^256 + 2^132,
// a fourth below 2^256; one conditional subtraction finishes (2^256 < 2n).
static void sc_reduce(uint64_t* out, const uint64_t* tin) {
    uint64_t t[9] = {0};
    memcpy(t, tin, 8 * sizeof(uint64_t));
    for (int iter = 0; iter < 4; ++iter) {
        uint64_t acc[9] = {t[0], t[1], t[2], t[3], 0, 0, 0, 0, 0};
        for (int i = 0; i < 5; ++i) { // acc += hi[i] * NC << 64i; every limb, zeros included
            u128 c = 0;
            for (int j = 0; j < 3; ++j) {
                c += (u128)t[4 + i] * NC[j] + acc[i + j];
                acc[i + j] = (uint64_t)c;
                c >>= 64;
            }
            for (int k = i + 3; k < 9; ++k) {
                c += acc[k];
                acc[k] = (uint64_t)c;
                c >>= 64;
            }
        }
        memcpy(t, acc, sizeof(acc));
    }
    csub4(t, N);
    memcpy(out, t, 32);
}
void sc_mul(Scalar& r, const Scalar& a, const Scalar& b) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += (u128)a.n[i] * b.n[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
        t[i + 4] = (uint64_t)c;
    }
    sc_reduce(r.n, t);
}
void sc_inv(Scalar& r, const Scalar& a) {
    // a^(n-2) with a fixed 4-bit window: 256 squarings and 64 multiplications (plus 14 for the
    // table) instead of ~200 multiplications of plain square-and-multiply
    static const uint64_t NM2[4] = {0xBFD25E8CD036413FULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL,
                                    0xFFFFFFFFFFFFFFFFULL};
    Scalar tab[16];
    tab[0] = {{1, 0, 0, 0}};
    tab[1] = a;
    for (int i = 2; i < 16; ++i) sc_mul(tab[i], tab[i - 1], a);
    Scalar acc = {{1, 0, 0, 0}};
    for (int i = 63; i >= 0; --i) {
        for (int k = 0; k < 4; ++k) sc_mul(acc, acc, acc);
        const unsigned w = (unsigned)(NM2[i / 16] >> ((i % 16) * 4)) & 15;
        if (w) sc_mul(acc, acc, tab[w]);
    }
    r = acc;
}

// ---------------------------------------------------------------- group
static Ge make_generator() {
    static const unsigned char gx[32] = {0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62,
                                         0x95, 0xCE, 0x87, 0x0B, 0x07, 0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE,
                                         0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98};
    static const unsigned char gy[32] = {0x48, 0x3A, 0xDA, 0x77, 0x26, 0xA3, 0xC4, 0x65, 0x5D, 0xA4, 0xFB,
                                         0xFC, 0x0E, 0x11, 0x08, 0xA8, 0xFD, 0x17, 0xB4, 0x48, 0xA6, 0x85,
                                         0x54, 0x19, 0x9C, 0x47, 0xD0, 0x8F, 0xFB, 0x10, 0xD4, 0xB8};
    Ge g;
    fe_set_b32(g.x, gx);
    fe_set_b32(g.y, gy);
    g.inf = false;
    return g;
}
const Ge& generator() {
    static const Ge g = make_generator();
    return g;
}

void gej_set_ge(Gej& r, const Ge& a) {
    r.inf = a.inf;
    r.x = a.x;
    r.y = a.y;
    fe_set_int(r.z, 1);
}

void gej_double(Gej& r, const Gej& a) {
    if (a.inf || fe_is_zero(a.y)) {
        r.inf = true;
        return;
    }
    Fe A, B, C, D, E, F, t, X3, Y3, Z3;
    fe_sqr(A, a.x);
    fe_sqr(B, a.y);
    fe_sqr(C, B);
    fe_add(t, a.x, B);
    fe_sqr(t, t);
    fe_sub(t, t, A);
    fe_sub(t, t, C);
    fe_add(D, t, t);
    fe_add(E, A, A);
    fe_add(E, E, A);
    fe_sqr(F, E);
    fe_add(t, D, D);
    fe_sub(X3, F, t);
    fe_sub(t, D, X3);
    fe_mul(Y3, E, t);
    fe_add(t, C, C);
    fe_add(t, t, t);
    fe_add(t, t, t);
    fe_sub(Y3, Y3, t);
    fe_mul(Z3, a.y, a.z);
    fe_add(Z3, Z3, Z3);
    r.x = X3;
    r.y = Y3;
    r.z = Z3;
    r.inf = false;
}

void gej_add_ge(Gej& r, const Gej& a, const Ge& b) {
    if (b.inf) {
        r = a;
        return;
    }
    if (a.inf) {
        gej_set_ge(r, b);
        return;
    }
    Fe Z1Z1, U2, S2, H, rr, HH, I, J, V, t, X3, Y3, Z3;
    fe_sqr(Z1Z1, a.z);
    fe_mul(U2, b.x, Z1Z1);
    fe_mul(S2, b.y, a.z);
    fe_mul(S2, S2, Z1Z1);
    fe_sub(H, U2, a.x);
    fe_sub(rr, S2, a.y);
    fe_add(rr, rr, rr);
    if (fe_is_zero(H)) {
        if (fe_is_zero(rr)) {
            gej_double(r, a);
        } else {
            r.inf = true;
        }
        return;
    }
    fe_sqr(HH, H);
    fe_add(I, HH, HH);
    fe_add(I, I, I);
    fe_mul(J, H, I);
    fe_mul(V, a.x, I);
    fe_sqr(X3, rr);
    fe_sub(X3, X3, J);
    fe_sub(X3, X3, V);
    fe_sub(X3, X3, V);
    fe_sub(t, V, X3);
    fe_mul(Y3, rr, t);
    fe_mul(t, a.y, J);
    fe_add(t, t, t);
    fe_sub(Y3, Y3, t);
    fe_add(Z3, a.z, H);
    fe_sqr(Z3, Z3);
    fe_sub(Z3, Z3, Z1Z1);
    fe_sub(Z3, Z3, HH);
    r.x = X3;
    r.y = Y3;
    r.z = Z3;
    r.inf = false;
}

void gej_add(Gej& r, const Gej& a, const Gej& b) {
    if (a.inf) {
        r = b;
        return;
    }
    if (b.inf) {
        r = a;
        return;
    }
    Fe Z1Z1, Z2Z2, U1, U2, S1, S2, H, rr, I, J, V, t, X3, Y3, Z3;
    fe_sqr(Z1Z1, a.z);
    fe_sqr(Z2Z2, b.z);
    fe_mul(U1, a.x, Z2Z2);
    fe_mul(U2, b.x, Z1Z1);
    fe_mul(S1, a.y, b.z);
    fe_mul(S1, S1, Z2Z2);
    fe_mul(S2, b.y, a.z);
    fe_mul(S2, S2, Z1Z1);
    fe_sub(H, U2, U1);
    fe_sub(rr, S2, S1);
    fe_add(rr, rr, rr);
    if (fe_is_zero(H)) {
        if (fe_is_zero(rr)) {
            gej_double(r, a);
        } else {
            r.inf = true;
        }
        return;
    }
    fe_add(I, H, H);
    fe_sqr(I, I);
    fe_mul(J, H, I);
    fe_mul(V, U1, I);
    fe_sqr(X3, rr);
    fe_sub(X3, X3, J);
    fe_sub(X3, X3, V);
    fe_sub(X3, X3, V);
    fe_sub(t, V, X3);
    fe_mul(Y3, rr, t);
    fe_mul(t, S1, J);
    fe_add(t, t, t);
    fe_sub(Y3, Y3, t);
    fe_add(Z3, a.z, b.z);
    fe_sqr(Z3, Z3);
    fe_sub(Z3, Z3, Z1Z1);
    fe_sub(Z3, Z3, Z2Z2);
    fe_mul(Z3, Z3, H);
    r.x = X3;
    r.y = Y3;
    r.z = Z3;
    r.inf = false;
}

void ge_set_gej(Ge& r, const Gej& a) {
    if (a.inf) {
        r.inf = true;
        return;
    }
    Fe zi, zi2, zi3;
    fe_inv(zi, a.z);
    fe_sqr(zi2, zi);
    fe_mul(zi3, zi2, zi);
    fe_mul(r.x, a.x, zi2);
    fe_mul(r.y, a.y, zi3);
    r.inf = false;
}

// Batch Jacobian -> affine with one inversion (Montgomery's trick).
static void batch_to_affine(Ge* out, const Gej* in, size_t n) {
    std::vector<Fe> acc(n);
    Fe run;
    fe_set_int(run, 1);
    for (size_t i = 0; i < n; ++i) {
        acc[i] = run;
        if (!in[i].inf) fe_mul(run, run, in[i].z);
    }
    Fe inv;
    fe_inv(inv, run);
    for (size_t i = n; i-- > 0;) {
        if (in[i].inf) {
            out[i].inf = true;
            continue;
        }
        Fe zi, zi2, zi3;
        fe_mul(zi, inv, acc[i]);
        fe_mul(inv, inv, in[i].z);
        fe_sqr(zi2, zi);
        fe_mul(zi3, zi2, zi);
        fe_mul(out[i].x, in[i].x, zi2);
        fe_mul(out[i].y, in[i].y, zi3);
        out[i].inf = false;
    }
}

bool ge_is_valid(const Ge& a) {
    if (a.inf) return false;
    Fe y2, x3, seven;
    fe_sqr(y2, a.y);
    fe_sqr(x3, a.x);
    fe_mul(x3, x3, a.x);
    fe_set_int(seven, 7);
    fe_add(x3, x3, seven);
    return fe_equal(y2, x3);
}

// table[i][j] = j * 256^i * G  (i < 32, 1 <= j < 256)
static std::vector<Ge>* g_gen_table = nullptr;
static std::once_flag g_gen_once;
static void build_gen_table() {
    std::vector<Gej> jac(32 * 256);
    Gej base;
    gej_set_ge(base, generator());
    for (int i = 0; i < 32; ++i) {
        Gej acc;
        acc.inf = true;
        jac[i * 256].inf = true;
        for (int j = 1; j < 256; ++j) {
            gej_add(acc, acc, base);
            jac[i * 256 + j] = acc;
        }
        // base *= 256
        for (int k = 0; k < 8; ++k) gej_double(base, base);
    }
    auto* t = new std::vector<Ge>(32 * 256);
    batch_to_affine(t->data(), jac.data(), jac.size());
    g_gen_table = t;
}

const std::vector<Ge>& generator_table() {
    std::call_once(g_gen_once, build_gen_table);
    return *g_gen_table;
}

// 11-bit windows for the GPU's 10 x 26 kernels: [i * 2048 + j] = j * 2^(11 i) * G, i < 24
// (24 additions per u1*G instead of 32; 3 MiB as device affine words, L2-resident)
static std::vector<Ge>* g_gen_table11 = nullptr;
static std::once_flag g_gen_once11;
static void build_gen_table11() {
    constexpr int W = 24, E = 2048;
    std::vector<Gej> jac((size_t)W * E);
    Gej base;
    gej_set_ge(base, generator());
    for (int i = 0; i < W; ++i) {
        Gej acc;
        acc.inf = true;
        jac[(size_t)i * E].inf = true;
        for (int j = 1; j < E; ++j) {
            gej_add(acc, acc, base);
            jac[(size_t)i * E + j] = acc;
        }
        for (int k = 0; k < 11; ++k) gej_double(base, base);
    }
    auto* t = new std::vector<Ge>((size_t)W * E);
    batch_to_affine(t->data(), jac.data(), jac.size());
    g_gen_table11 = t;
}

const std::vector<Ge>& generator_table11() {
    std::call_once(g_gen_once11, build_gen_table11);
    return *g_gen_table11;
}

// Variable-time k*G for PUBLIC scalars only (signature verification, ecmult): one table add per
// non-zero byte of k.
void ecmult_gen_var(Gej& r, const Scalar& k) {
    std::call_once(g_gen_once, build_gen_table);
    r.inf = true;
    for (int i = 0; i < 32; ++i) {
        const unsigned byte = (unsigned)(k.n[i / 8] >> ((i % 8) * 8)) & 0xff;
        if (byte) gej_add_ge(r, r, (*g_gen_table)[i * 256 + byte]);
    }
}

// ---------------------------------------------------------------- constant-time k*G
// For SECRET scalars (signing nonces, private keys). Same method as libsecp256k1's
// secp256k1_ecmult_gen (reference src/secp256k1/src/ecmult_gen_impl.h:124-156):
//  * a comb of 64 rows x 16 affine entries, CT_TAB[j][i] = (i * 16^j + 1) * G, so no entry is
//    the point at infinity;
//  * the scalar is blinded, s = k + b (b random per process), and the accumulator starts at
//    A0 = (-b - 64) * G with randomised Jacobian Z, so sum_j CT_TAB[j][nibble_j(s)] + A0 = k * G;
//  * every row lookup reads ALL 16 entries and keeps the wanted one with masks (cmov), and every
//    addition runs the full formula (its exceptional cases are selected with masks), so the
//    sequence of memory reads and field operations is the same for every k.
namespace {
struct CtGenTable {
    Ge e[64][16];
};
CtGenTable* g_ct_tab = nullptr;
std::once_flag g_ct_once;
struct CtBlind {
    Scalar b;  // blinding scalar
    Gej a0;    // (-b - 64) * G, Z randomised
};
std::mutex g_blind_mu;
CtBlind g_blind;
bool g_blind_set = false;
thread_local EcmultGenTrace* g_trace = nullptr;

void build_ct_table() {
    std::vector<Gej> jac(64 * 16);
    Gej base, one;
    gej_set_ge(base, generator());
    gej_set_ge(one, generator());
    for (int j = 0; j < 64; ++j) {
        Gej acc = one; // 1 * G, then + base each step: (i * 16^j + 1) * G
        for (int i = 0; i < 16; ++i) {
            jac[j * 16 + i] = acc;
            gej_add(acc, acc, base);
        }
        for (int k = 0; k < 4; ++k) gej_double(base, base);
    }
    auto* t = new CtGenTable;
    batch_to_affine(&t->e[0][0], jac.data(), jac.size());
    g_ct_tab = t;
}

void read_urandom(unsigned char* out, size_t n) {
    size_t got = 0;
    if (FILE* f = fopen("/dev/urandom", "rb")) {
        got = fread(out, 1, n, f);
        fclose(f);
    }
    if (got != n) throw std::runtime_error("secp256k1: cannot read /dev/urandom for the signing blind");
}

// Constant-time Jacobian doubling (the formula of gej_double without its early exits; the
// infinity flag passes through, and secp256k1 has no point with y = 0).
void gej_double_ct(Gej& r, const Gej& a) {
    Fe A, B, C, D, E, F, t, X3, Y3, Z3;
    fe_sqr(A, a.x);
    fe_sqr(B, a.y);
    fe_sqr(C, B);
    fe_add(t, a.x, B);
    fe_sqr(t, t);
    fe_sub(t, t, A);
    fe_sub(t, t, C);
    fe_add(D, t, t);
    fe_add(E, A, A);
    fe_add(E, E, A);
    fe_sqr(F, E);
    fe_add(t, D, D);
    fe_sub(X3, F, t);
    fe_sub(t, D, X3);
    fe_mul(Y3, E, t);
    fe_add(t, C, C);
    fe_add(t, t, t);
    fe_add(t, t, t);
    fe_sub(Y3, Y3, t);
    fe_mul(Z3, a.y, a.z);
    fe_add(Z3, Z3, Z3);
    r.x = X3;
    r.y = Y3;
    r.z = Z3;
    r.inf = a.inf;
}

void fe_cmov(Fe& r, const Fe& a, uint64_t mask) { cmov4(r.n, a.n, mask); }

// Constant-time r = a + b (b affine, never infinity): the general formula, the doubling of a
// (for a == b) and b itself (for a = infinity) are all computed; masks pick the result, and
// a == -b yields infinity.
void gej_add_ge_ct(Gej& r, const Gej& a, const Ge& b) {
    Fe Z1Z1, U2, S2, H, rr, HH, I, J, V, t, X3, Y3, Z3;
    fe_sqr(Z1Z1, a.z);
    fe_mul(U2, b.x, Z1Z1);
    fe_mul(S2, b.y, a.z);
    fe_mul(S2, S2, Z1Z1);
    fe_sub(H, U2, a.x);
    fe_sub(rr, S2, a.y);
    fe_add(rr, rr, rr);
    fe_sqr(HH, H);
    fe_add(I, HH, HH);
    fe_add(I, I, I);
    fe_mul(J, H, I);
    fe_mul(V, a.x, I);
    fe_sqr(X3, rr);
    fe_sub(X3, X3, J);
    fe_sub(X3, X3, V);
    fe_sub(X3, X3, V);
    fe_sub(t, V, X3);
    fe_mul(Y3, rr, t);
    fe_mul(t, a.y, J);
    fe_add(t, t, t);
    fe_sub(Y3, Y3, t);
    fe_add(Z3, a.z, H);
    fe_sqr(Z3, Z3);
    fe_sub(Z3, Z3, Z1Z1);
    fe_sub(Z3, Z3, HH);
    Gej d;
    gej_double_ct(d, a);
    const uint64_t ainf = mask_of((uint64_t)a.inf);
    const uint64_t hz = fe_zero_mask(H) & ~ainf, rz = fe_zero_mask(rr);
    const uint64_t dbl = hz & rz, neg = hz & ~rz; // a == b, a == -b
    Gej out;
    out.x = X3;
    out.y = Y3;
    out.z = Z3;
    fe_cmov(out.x, d.x, dbl);
    fe_cmov(out.y, d.y, dbl);
    fe_cmov(out.z, d.z, dbl);
    Fe one;
    fe_set_int(one, 1);
    fe_cmov(out.x, b.x, ainf);
    fe_cmov(out.y, b.y, ainf);
    fe_cmov(out.z, one, ainf);
    out.inf = (bool)(neg & 1);
    r = out;
}

// Set the blind from 32 seed bytes (caller holds g_blind_mu).
void set_blind_locked(const unsigned char* seed32) {
    unsigned char h[32], z32[32];
    CSHA256().Write(seed32, 32).Write((const unsigned char*)"bcp-ecmult-gen-blind", 20).Finalize(h);
    CSHA256().Write(h, 32).Write((const unsigned char*)"z", 1).Finalize(z32);
    Scalar b, nb, c64;
    sc_set_b32(b, h);
    if (sc_is_zero(b)) b.n[0] = 1;
    // A0 = (-b - 64) * G: computed by the public-scalar path (b is not used on its own
    // anywhere an attacker can time it; the value is fixed for the process)
    c64 = {{64, 0, 0, 0}};
    sc_add(nb, b, c64);
    sc_neg(nb, nb);
    Gej a0;
    ecmult_gen_var(a0, nb);
    Fe z, z2, z3;
    bool of;
    fe_set_b32(z, z32, &of);
    if (fe_is_zero(z)) fe_set_int(z, 1);
    fe_sqr(z2, z);
    fe_mul(z3, z2, z);
    fe_mul(a0.x, a0.x, z2);
    fe_mul(a0.y, a0.y, z3);
    fe_mul(a0.z, a0.z, z);
    g_blind.b = b;
    g_blind.a0 = a0;
    g_blind_set = true;
    memory_cleanse(h, sizeof(h));
    memory_cleanse(z32, sizeof(z32));
}
} // namespace

void ecmult_gen_blind(const unsigned char* seed32) {
    std::call_once(g_gen_once, build_gen_table);
    unsigned char seed[32];
    if (seed32) memcpy(seed, seed32, 32);
    else read_urandom(seed, 32);
    std::lock_guard<std::mutex> lk(g_blind_mu);
    set_blind_locked(seed);
    memory_cleanse(seed, sizeof(seed));
}

void ecmult_gen_trace(EcmultGenTrace* t) { g_trace = t; }

void ecmult_gen(Gej& r, const Scalar& k) {
    std::call_once(g_ct_once, build_ct_table);
    std::call_once(g_gen_once, build_gen_table);
    CtBlind bl;
    {
        std::lock_guard<std::mutex> lk(g_blind_mu);
        if (!g_blind_set) {
            unsigned char seed[32];
            read_urandom(seed, 32);
            set_blind_locked(seed);
            memory_cleanse(seed, sizeof(seed));
        }
        bl = g_blind;
    }
    Scalar s;
    sc_add(s, k, bl.b);
    Gej acc = bl.a0;
    EcmultGenTrace* tr = g_trace;
    for (int j = 0; j < 64; ++j) {
        const uint64_t nib = (s.n[j / 16] >> ((j % 16) * 4)) & 15;
        Ge e;
        e.inf = false;
        fe_set_int(e.x, 0);
        fe_set_int(e.y, 0);
        for (uint64_t i = 0; i < 16; ++i) { // every entry of the row is read
            const Ge& c = g_ct_tab->e[j][i];
            const uint64_t m = mask_of((((i ^ nib) | ((uint64_t)0 - (i ^ nib))) >> 63) ^ 1);
            fe_cmov(e.x, c.x, m);
            fe_cmov(e.y, c.y, m);
            if (tr) tr->reads.push_back((uint32_t)(j * 16 + i));
        }
        gej_add_ge_ct(acc, acc, e);
        if (tr) tr->adds++;
    }
    r = acc;
    memory_cleanse(&s, sizeof(s));
}

// width-w NAF of a scalar; returns number of digits
static int wnaf(int* digits, const Scalar& s, int w) {
    uint64_t k[5] = {s.n[0], s.n[1], s.n[2], s.n[3], 0};
    int len = 0;
    auto is_zero = [&] { return (k[0] | k[1] | k[2] | k[3] | k[4]) == 0; };
    while (!is_zero()) {
        int d = 0;
        if (k[0] & 1) {
            d = (int)(k[0] & ((1u << w) - 1));
            if (d >= (1 << (w - 1))) d -= (1 << w);
            // k -= d
            if (d > 0) {
                u128 t = (u128)k[0] - (uint64_t)d;
                k[0] = (uint64_t)t;
                uint64_t br = (uint64_t)(t >> 127) & 1;
                for (int i = 1; i < 5 && br; ++i) {
                    u128 u = (u128)k[i] - 1;
                    k[i] = (uint64_t)u;
                    br = (uint64_t)(u >> 127) & 1;
                }
            } else {
                u128 t = (u128)k[0] + (uint64_t)(-d);
                k[0] = (uint64_t)t;
                uint64_t c = (uint64_t)(t >> 64);
                for (int i = 1; i < 5 && c; ++i) {
                    u128 u = (u128)k[i] + 1;
                    k[i] = (uint64_t)u;
                    c = (uint64_t)(u >> 64);
                }
            }
        }
        digits[len++] = d;
        // k >>= 1
        for (int i = 0; i < 4; ++i) k[i] = (k[i] >> 1) | (k[i + 1] << 63);
        k[4] >>= 1;
    }
    return len;
}

// ---- GLV endomorphism: lambda * (x, y) = (beta * x, y), so na = k1 + k2 * lambda (mod n) with
// |k1|, |k2| < 2^129 halves the doublings of na * A. The lattice constants are the GPU verify
// kernel's (csrc/kernels/secp256k1.hip GLV_*, range-checked there), as 32-bit little-endian limbs:
// c1 = round(k * g1 / 2^384), c2 = round(k * g2 / 2^384), k2 = c1 * (-b1) - c2 * b2,
// k1 = k - c1 * a1 - c2 * a2.
namespace {
const uint32_t GLV_G1[8] = {0x45DBB031, 0xE893209A, 0x71E8CA7F, 0x3DAA8A14,
                            0x9284EB15, 0xE86C90E4, 0xA7D46BCD, 0x3086D221};
const uint32_t GLV_G2[8] = {0x8AC47F71, 0x1571B4AE, 0x9DF506C6, 0x221208AC,
                            0x0ABFE4C4, 0x6F547FA9, 0x010E8828, 0xE4437ED6};
const uint32_t GLV_A1[4] = {0x9284EB15, 0xE86C90E4, 0xA7D46BCD, 0x3086D221};
const uint32_t GLV_B1N[4] = {0x0ABFE4C3, 0x6F547FA9, 0x010E8828, 0xE4437ED6}; // -b1
const uint32_t GLV_A2[5] = {0x9D44CFD8, 0x57C1108D, 0xA8E2F3F6, 0x14CA50F7, 0x00000001};
const uint32_t GLV_B2[4] = {0x9284EB15, 0xE86C90E4, 0xA7D46BCD, 0x3086D221};
// beta, big-endian bytes: a cube root of unity mod p
const unsigned char GLV_BETA_BE[32] = {0x7A, 0xE9, 0x6A, 0x2B, 0x65, 0x7C, 0x07, 0x10, 0x6E, 0x64, 0x47,
                                       0x9E, 0xAC, 0x34, 0x34, 0xE9, 0x9C, 0xF0, 0x49, 0x75, 0x12, 0xF5,
                                       0x89, 0x95, 0xC1, 0x39, 0x6C, 0x28, 0x71, 0x95, 0x01, 0xEE};

template <int NA, int NB> void mul_wide32(uint32_t* r, const uint32_t* a, const uint32_t* b) {
    for (int i = 0; i < NA + NB; i++) r[i] = 0;
    for (int i = 0; i < NA; i++) {
        uint64_t c = 0;
        for (int j = 0; j < NB; j++) {
            c += (uint64_t)r[i + j] + (uint64_t)a[i] * b[j];
            r[i + j] = (uint32_t)c;
            c >>= 32;
        }
        r[i + NB] = (uint32_t)c;
    }
}

// |v| of a 10-limb two's-complement value into a Scalar-shaped magnitude (< 2^130); true if v < 0
bool abs10(Scalar& m, const uint32_t* v) {
    uint32_t t[10];
    const bool neg = v[9] >> 31;
    if (neg) {
        uint64_t c = 1;
        for (int i = 0; i < 10; i++) {
            c += (uint64_t)(uint32_t)~v[i];
            t[i] = (uint32_t)c;
            c >>= 32;
        }
    } else {
        for (int i = 0; i < 10; i++) t[i] = v[i];
    }
    for (int i = 0; i < 4; i++) m.n[i] = (uint64_t)t[2 * i] | ((uint64_t)t[2 * i + 1] << 32);
    return neg;
}

void glv_split(const Scalar& k, Scalar& m1, bool& neg1, Scalar& m2, bool& neg2) {
    uint32_t kv[8];
    for (int i = 0; i < 4; i++) {
        kv[2 * i] = (uint32_t)k.n[i];
        kv[2 * i + 1] = (uint32_t)(k.n[i] >> 32);
    }
    auto mul_shift384 = [&](uint32_t (&c)[4], const uint32_t* g) {
        uint32_t t[16];
        mul_wide32<8, 8>(t, kv, g);
        uint64_t carry = t[11] >> 31; // rounding bit 383
        for (int i = 0; i < 4; i++) {
            carry += t[12 + i];
            c[i] = (uint32_t)carry;
            carry >>= 32;
        }
    };
    uint32_t c1[4], c2[4];
    mul_shift384(c1, GLV_G1);
    mul_shift384(c2, GLV_G2);
    uint32_t p1[8], p2[8], p3[8], p4[9], k1[10], k2[10];
    mul_wide32<4, 4>(p1, c1, GLV_B1N);
    mul_wide32<4, 4>(p2, c2, GLV_B2);
    mul_wide32<4, 4>(p3, c1, GLV_A1);
    mul_wide32<4, 5>(p4, c2, GLV_A2);
    uint64_t br = 0;
    for (int i = 0; i < 10; i++) { // k2 = c1*(-b1) - c2*b2
        const uint64_t d = (uint64_t)(i < 8 ? p1[i] : 0u) - (i < 8 ? p2[i] : 0u) - br;
        k2[i] = (uint32_t)d;
        br = (d >> 63) & 1;
    }
    int64_t sb = 0;
    for (int i = 0; i < 10; i++) { // k1 = k - c1*a1 - c2*a2 (the borrow reaches 2)
        const int64_t v = (int64_t)(i < 8 ? kv[i] : 0u) - (int64_t)(i < 8 ? p3[i] : 0u) -
                          (int64_t)(i < 9 ? p4[i] : 0u) - sb;
        k1[i] = (uint32_t)v;
        sb = -(v >> 32);
    }
    neg1 = abs10(m1, k1);
    neg2 = abs10(m2, k2);
}
} // namespace

bool glv_check(const Scalar& k) {
    // k1 + k2 * lambda == k (mod n), for tests
    Scalar m1, m2;
    bool n1, n2;
    glv_split(k, m1, n1, m2, n2);
    static const unsigned char LAMBDA_BE[32] = {0x53, 0x63, 0xAD, 0x4C, 0xC0, 0x5C, 0x30, 0xE0, 0xA5, 0x26, 0x1C,
                                                0x02, 0x88, 0x12, 0x64, 0x5A, 0x12, 0x2E, 0x22, 0xEA, 0x20, 0x81,
                                                0x66, 0x78, 0xDF, 0x02, 0x96, 0x7C, 0x1B, 0x23, 0xBD, 0x72};
    if (m1.n[3] || (m1.n[2] >> 2) || m2.n[3] || (m2.n[2] >> 2)) return false; // |k1|,|k2| < 2^130
    Scalar lambda, t, r;
    sc_set_b32(lambda, LAMBDA_BE);
    if (n1) sc_neg(m1, m1);
    if (n2) sc_neg(m2, m2);
    sc_mul(t, m2, lambda);
    sc_add(r, m1, t);
    return memcmp(r.n, k.n, sizeof(r.n)) == 0;
}

void ecmult_plain(Gej& r, const Gej& a, const Scalar& na, const Scalar& ng);

void ecmult(Gej& r, const Gej& a, const Scalar& na, const Scalar& ng) {
    Gej acc;
    acc.inf = true;
    if (!a.inf && !sc_is_zero(na)) {
        // na * A = k1 * A + k2 * (lambda A): odd multiples A .. 15A, and lambda's with X * beta
        Gej pre_j[8], a2;
        pre_j[0] = a;
        gej_double(a2, a);
        for (int i = 1; i < 8; ++i) gej_add(pre_j[i], pre_j[i - 1], a2);
        Ge pre[2][8];
        batch_to_affine(pre[0], pre_j, 8);
        static const Fe beta = [] {
            Fe b;
            fe_set_b32(b, GLV_BETA_BE);
            return b;
        }();
        Scalar m[2];
        bool neg[2];
        glv_split(na, m[0], neg[0], m[1], neg[1]);
        for (int i = 0; i < 8; ++i) {
            pre[1][i] = pre[0][i];
            fe_mul(pre[1][i].x, pre[0][i].x, beta);
        }
        for (int h = 0; h < 2; ++h)
            if (neg[h])
                for (int i = 0; i < 8; ++i) fe_neg(pre[h][i].y, pre[h][i].y);
        int digits[2][140];
        int len[2];
        for (int h = 0; h < 2; ++h) len[h] = wnaf(digits[h], m[h], 5);
        for (int i = std::max(len[0], len[1]) - 1; i >= 0; --i) {
            gej_double(acc, acc);
            for (int h = 0; h < 2; ++h) {
                const int d = i < len[h] ? digits[h][i] : 0;
                if (d > 0) {
                    gej_add_ge(acc, acc, pre[h][(d - 1) / 2]);
                } else if (d < 0) {
                    Ge neg_p = pre[h][(-d - 1) / 2];
                    fe_neg(neg_p.y, neg_p.y);
                    gej_add_ge(acc, acc, neg_p);
                }
            }
        }
    }
    if (!sc_is_zero(ng)) {
        Gej g;
        ecmult_gen_var(g, ng);
        gej_add(acc, acc, g);
    }
    r = acc;
}

// The straightforward double-and-add over all 256 bits (kept as the differential reference).
void ecmult_plain(Gej& r, const Gej& a, const Scalar& na, const Scalar& ng) {
    Gej acc;
    acc.inf = true;
    if (!a.inf && !sc_is_zero(na)) {
        // odd multiples A, 3A, ..., 15A
        Gej pre_j[8], a2;
        pre_j[0] = a;
        gej_double(a2, a);
        for (int i = 1; i < 8; ++i) gej_add(pre_j[i], pre_j[i - 1], a2);
        Ge pre[8];
        batch_to_affine(pre, pre_j, 8);
        int digits[260];
        int len = wnaf(digits, na, 5);
        for (int i = len - 1; i >= 0; --i) {
            gej_double(acc, acc);
            int d = digits[i];
            if (d > 0) {
                gej_add_ge(acc, acc, pre[(d - 1) / 2]);
            } else if (d < 0) {
                Ge neg = pre[(-d - 1) / 2];
                fe_neg(neg.y, neg.y);
                gej_add_ge(acc, acc, neg);
            }
        }
    }
    if (!sc_is_zero(ng)) {
        Gej g;
        ecmult_gen_var(g, ng);
        gej_add(acc, acc, g);
    }
    r = acc;
}

// ---------------------------------------------------------------- keys
bool pubkey_parse(Ge& r, const unsigned char* in, size_t len) {
    r.inf = true;
    if (len == 33 && (in[0] == 0x02 || in[0] == 0x03)) {
        bool of;
        fe_set_b32(r.x, in + 1, &of);
        if (of) return false;
        Fe x3, seven, y;
        fe_sqr(x3, r.x);
        fe_mul(x3, x3, r.x);
        fe_set_int(seven, 7);
        fe_add(x3, x3, seven);
        if (!fe_sqrt(y, x3)) return false;
        if (fe_is_odd(y) != (in[0] == 0x03)) fe_neg(y, y);
        r.y = y;
        r.inf = false;
        return true;
    }
    if (len == 65 && (in[0] == 0x04 || in[0] == 0x06 || in[0] == 0x07)) {
        bool ofx, ofy;
        fe_set_b32(r.x, in + 1, &ofx);
        fe_set_b32(r.y, in + 33, &ofy);
        if (ofx || ofy) return false;
        r.inf = false;
        if ((in[0] == 0x06 || in[0] == 0x07) && fe_is_odd(r.y) != (in[0] == 0x07)) {
            r.inf = true;
            return false;
        }
        if (!ge_is_valid(r)) {
            r.inf = true;
            return false;
        }
        return true;
    }
    return false;
}

std::vector<unsigned char> pubkey_serialize(const Ge& p, bool compressed) {
    std::vector<unsigned char> out(compressed ? 33 : 65);
    fe_get_b32(&out[1], p.x);
    if (compressed) {
        out[0] = fe_is_odd(p.y) ? 0x03 : 0x02;
    } else {
        out[0] = 0x04;
        fe_get_b32(&out[33], p.y);
    }
    return out;
}

bool seckey_verify(const unsigned char* seckey32) {
    Scalar s;
    bool of;
    sc_set_b32(s, seckey32, &of);
    return !of && !sc_is_zero(s);
}

bool pubkey_create(Ge& r, const unsigned char* seckey32) {
    Scalar s;
    bool of;
    sc_set_b32(s, seckey32, &of);
    if (of || sc_is_zero(s)) return false;
    Gej pj;
    ecmult_gen(pj, s);
    ge_set_gej(r, pj);
    memory_cleanse(&s, sizeof(s));
    return true;
}

bool seckey_tweak_add(unsigned char* seckey32, const unsigned char* tweak32) {
    Scalar s, t;
    bool of1, of2;
    sc_set_b32(s, seckey32, &of1);
    sc_set_b32(t, tweak32, &of2);
    if (of1 || of2) return false;
    sc_add(s, s, t);
    if (sc_is_zero(s)) return false;
    sc_get_b32(seckey32, s);
    return true;
}

bool pubkey_tweak_add(Ge& p, const unsigned char* tweak32) {
    Scalar t;
    bool of;
    sc_set_b32(t, tweak32, &of);
    if (of) return false;
    Gej pj, tg;
    gej_set_ge(pj, p);
    ecmult_gen(tg, t);
    gej_add(pj, pj, tg);
    if (pj.inf) return false;
    ge_set_gej(p, pj);
    return true;
}

// ---------------------------------------------------------------- ECDSA
bool sig_parse_compact(Signature& sig, const unsigned char* in64) {
    bool of1, of2;
    sc_set_b32(sig.r, in64, &of1);
    sc_set_b32(sig.s, in64 + 32, &of2);
    if (of1 || of2) {
        memset(&sig, 0, sizeof(sig));
        return false;
    }
    return true;
}
void sig_serialize_compact(unsigned char* out64, const Signature& sig) {
    sc_get_b32(out64, sig.r);
    sc_get_b32(out64 + 32, sig.s);
}

bool sig_parse_der_lax(Signature& sig, const unsigned char* input, size_t inputlen) {
    size_t rpos, rlen, spos, slen, pos = 0, lenbyte;
    unsigned char tmp[64] = {0};
    memset(&sig, 0, sizeof(sig));
    if (pos == inputlen || input[pos] != 0x30) return false;
    pos++;
    if (pos == inputlen) return false;
    lenbyte = input[pos++];
    if (lenbyte & 0x80) {
        lenbyte -= 0x80;
        if (pos + lenbyte > inputlen) return false;
        pos += lenbyte;
    }
    auto read_int = [&](size_t& ipos, size_t& ilen) -> bool {
        if (pos == inputlen || input[pos] != 0x02) return false;
        pos++;
        if (pos == inputlen) return false;
        lenbyte = input[pos++];
        if (lenbyte & 0x80) {
            lenbyte -= 0x80;
            if (pos + lenbyte > inputlen) return false;
            while (lenbyte > 0 && input[pos] == 0) {
                pos++;
                lenbyte--;
            }
            if (lenbyte >= sizeof(size_t)) return false;
            ilen = 0;
            while (lenbyte > 0) {
                ilen = (ilen << 8) + input[pos];
                pos++;
                lenbyte--;
            }
        } else {
            ilen = lenbyte;
        }
        if (ilen > inputlen - pos) return false;
        ipos = pos;
        pos += ilen;
        return true;
    };
    if (!read_int(rpos, rlen)) return false;
    if (!read_int(spos, slen)) return false;
    bool overflow = false;
    while (rlen > 0 && input[rpos] == 0) {
        rlen--;
        rpos++;
    }
    if (rlen > 32) overflow = true;
    else memcpy(tmp + 32 - rlen, input + rpos, rlen);
    while (slen > 0 && input[spos] == 0) {
        slen--;
        spos++;
    }
    if (slen > 32) overflow = true;
    else memcpy(tmp + 64 - slen, input + spos, slen);
    if (!overflow) overflow = !sig_parse_compact(sig, tmp);
    if (overflow) memset(&sig, 0, sizeof(sig)); // parsed but invalid
    return true;
}

bool sig_parse_der_strict(Signature& sig, const unsigned char* in, size_t len) {
    // 0x30 [len] 0x02 [rlen] [r] 0x02 [slen] [s], minimal encodings
    if (len < 8 || len > 72 || in[0] != 0x30 || in[1] != len - 2) return false;
    size_t rlen = in[3];
    if (in[2] != 0x02 || rlen == 0 || 5 + rlen >= len) return false;
    size_t slen = in[5 + rlen];
    if (in[4 + rlen] != 0x02 || slen == 0 || rlen + slen + 6 != len) return false;
    if ((in[4] & 0x80) || (rlen > 1 && in[4] == 0 && !(in[5] & 0x80))) return false;
    if ((in[6 + rlen] & 0x80) || (slen > 1 && in[6 + rlen] == 0 && !(in[7 + rlen] & 0x80))) return false;
    return sig_parse_der_lax(sig, in, len) && !(sc_is_zero(sig.r) && sc_is_zero(sig.s));
}

std::vector<unsigned char> sig_serialize_der(const Signature& sig) {
    unsigned char r[33] = {0}, s[33] = {0};
    sc_get_b32(r + 1, sig.r);
    sc_get_b32(s + 1, sig.s);
    const unsigned char* rp = r;
    const unsigned char* sp = s;
    size_t lenR = 33, lenS = 33;
    while (lenR > 1 && rp[0] == 0 && rp[1] < 0x80) {
        lenR--;
        rp++;
    }
    while (lenS > 1 && sp[0] == 0 && sp[1] < 0x80) {
        lenS--;
        sp++;
    }
    std::vector<unsigned char> out;
    out.push_back(0x30);
    out.push_back((unsigned char)(4 + lenR + lenS));
    out.push_back(0x02);
    out.push_back((unsigned char)lenR);
    out.insert(out.end(), rp, rp + lenR);
    out.push_back(0x02);
    out.push_back((unsigned char)lenS);
    out.insert(out.end(), sp, sp + lenS);
    return out;
}

bool sig_normalize(Signature& sig) {
    if (sc_is_high(sig.s)) {
        sc_neg(sig.s, sig.s);
        return true;
    }
    return false;
}

bool ecdsa_verify(const Signature& sig, const unsigned char* msg32, const Ge& pub) {
    if (pub.inf || sc_is_zero(sig.r) || sc_is_zero(sig.s) || sc_is_high(sig.s)) return false;
    Scalar e, w, u1, u2;
    sc_set_b32(e, msg32);
    sc_inv(w, sig.s);
    sc_mul(u1, e, w);
    sc_mul(u2, sig.r, w);
    Gej pj, R;
    gej_set_ge(pj, pub);
    ecmult(R, pj, u2, u1);
    if (R.inf) return false;
    // x(R) mod n == r without leaving Jacobian coordinates: X == r * Z^2 (mod p), or, when
    // r + n < p, X == (r + n) * Z^2 (the affine x may exceed n)
    unsigned char rb[32];
    sc_get_b32(rb, sig.r);
    Fe rx, z2, t;
    fe_set_b32(rx, rb);
    fe_sqr(z2, R.z);
    fe_mul(t, rx, z2);
    if (fe_equal(t, R.x)) return true;
    static const uint64_t PMN[4] = {0x402DA1722FC9BAEEULL, 0x4551231950B75FC4ULL, 1, 0}; // p - n
    if (!geq4(rx.n, PMN)) { // r < p - n
        Fe nfe, rn;
        nfe.n[0] = N[0];
        nfe.n[1] = N[1];
        nfe.n[2] = N[2];
        nfe.n[3] = N[3];
        fe_add(rn, rx, nfe);
        fe_mul(t, rn, z2);
        if (fe_equal(t, R.x)) return true;
    }
    return false;
}

void rfc6979_nonce(unsigned char* out32, const unsigned char* msg32, const unsigned char* key32,
                   const unsigned char* extra32, unsigned int counter) {
    unsigned char keydata[96];
    size_t kl = 64;
    memcpy(keydata, key32, 32);
    memcpy(keydata + 32, msg32, 32);
    if (extra32) {
        memcpy(keydata + 64, extra32, 32);
        kl = 96;
    }
    unsigned char v[32], k[32];
    memset(v, 0x01, 32);
    memset(k, 0x00, 32);
    const unsigned char zero = 0x00, one = 0x01;
    CHMAC_SHA256(k, 32).Write(v, 32).Write(&zero, 1).Write(keydata, kl).Finalize(k);
    CHMAC_SHA256(k, 32).Write(v, 32).Finalize(v);
    CHMAC_SHA256(k, 32).Write(v, 32).Write(&one, 1).Write(keydata, kl).Finalize(k);
    CHMAC_SHA256(k, 32).Write(v, 32).Finalize(v);
    bool retry = false;
    for (unsigned int i = 0; i <= counter; ++i) {
        if (retry) {
            CHMAC_SHA256(k, 32).Write(v, 32).Write(&zero, 1).Finalize(k);
            CHMAC_SHA256(k, 32).Write(v, 32).Finalize(v);
        }
        CHMAC_SHA256(k, 32).Write(v, 32).Finalize(v);
        memcpy(out32, v, 32);
        retry = true;
    }
    memory_cleanse(k, 32);
    memory_cleanse(v, 32);
    memory_cleanse(keydata, sizeof(keydata));
}

bool ecdsa_sign(Signature& sig, int* recid, const unsigned char* msg32, const unsigned char* seckey32,
                const unsigned char* extra32) {
    Scalar d, e;
    bool of;
    sc_set_b32(d, seckey32, &of);
    if (of || sc_is_zero(d)) return false;
    sc_set_b32(e, msg32);
    bool ok = false;
    unsigned char nonce[32];
    Scalar k, n, kinv;
    for (unsigned int counter = 0; counter < 1000 && !ok; ++counter) {
        rfc6979_nonce(nonce, msg32, seckey32, extra32, counter);
        sc_set_b32(k, nonce, &of);
        if (of || sc_is_zero(k)) continue; // probability ~2^-128: a retry, not a timing signal
        Gej Rj;
        ecmult_gen(Rj, k); // constant-time, blinded
        Ge R;
        ge_set_gej(R, Rj);
        unsigned char xb[32];
        fe_get_b32(xb, R.x);
        bool xof;
        sc_set_b32(sig.r, xb, &xof);
        int rid = (xof ? 2 : 0) | (fe_is_odd(R.y) ? 1 : 0);
        sc_mul(n, sig.r, d);
        sc_add(n, n, e);
        sc_inv(kinv, k);
        sc_mul(sig.s, kinv, n);
        if (sc_is_zero(sig.r) || sc_is_zero(sig.s)) continue;
        if (sc_is_high(sig.s)) { // s is public output
            sc_neg(sig.s, sig.s);
            rid ^= 1;
        }
        if (recid) *recid = rid;
        ok = true;
    }
    memory_cleanse(nonce, sizeof(nonce));
    memory_cleanse(&k, sizeof(k));
    memory_cleanse(&kinv, sizeof(kinv));
    memory_cleanse(&n, sizeof(n));
    memory_cleanse(&d, sizeof(d));
    return ok;
}

bool ecdsa_recover(Ge& pub, const Signature& sig, int recid, const unsigned char* msg32) {
    if (sc_is_zero(sig.r) || sc_is_zero(sig.s) || recid < 0 || recid > 3) return false;
    unsigned char rb[32];
    sc_get_b32(rb, sig.r);
    Fe x;
    fe_set_b32(x, rb);
    if (recid & 2) {
        // x = r + n, must be < p
        static const uint64_t NN[4] = {0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL,
                                       0xFFFFFFFFFFFFFFFFULL};
        uint64_t t[4];
        if (add4(t, x.n, NN)) return false;
        if (geq4(t, P)) return false;
        memcpy(x.n, t, 32);
    }
    Fe x3, seven, y;
    fe_sqr(x3, x);
    fe_mul(x3, x3, x);
    fe_set_int(seven, 7);
    fe_add(x3, x3, seven);
    if (!fe_sqrt(y, x3)) return false;
    if (fe_is_odd(y) != (bool)(recid & 1)) fe_neg(y, y);
    Ge R;
    R.x = x;
    R.y = y;
    R.inf = false;
    Scalar e, rn, u1, u2;
    sc_set_b32(e, msg32);
    sc_inv(rn, sig.r);
    sc_mul(u1, rn, e);
    sc_neg(u1, u1);
    sc_mul(u2, rn, sig.s);
    Gej Rj, Q;
    gej_set_ge(Rj, R);
    ecmult(Q, Rj, u2, u1);
    if (Q.inf) return false;
    ge_set_gej(pub, Q);
    return true;
}

bool VerifySignature(const unsigned char* pub, size_t publen, const unsigned char* sig, size_t siglen,
                     const unsigned char* msg32) {
    Ge p;
    if (!pubkey_parse(p, pub, publen)) return false;
    if (siglen == 0) return false;
    Signature s;
    if (!sig_parse_der_lax(s, sig, siglen)) return false;
    sig_normalize(s);
    return ecdsa_verify(s, msg32, p);
}

} // namespace secp
} // namespace bcp
