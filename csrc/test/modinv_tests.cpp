// modinv_tests: the ECDSA kernels' binary-GCD inverse (csrc/kernels/modinv.h), run on the host.
// Checked against a * a^-1 == 1 (mod m) by an independent shift-and-add modular product, for the
// secp256k1 group order n and field prime p, over random and edge-case inputs.
// Parity: the reference's variable-time inverses, src/secp256k1/src/scalar_impl.h
// (secp256k1_scalar_inverse_var) and field_impl.h (secp256k1_fe_inv_var).
#include "test/unittest.h"

#include "kernels/modinv.h"

#include <random>

namespace {

const uint32_t N[8] = {0xD0364141, 0xBFD25E8C, 0xAF48A03B, 0xBAAEDCE6, 0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF};
const uint32_t P[8] = {0xFFFFFC2F, 0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF};

bool Less(const uint32_t* a, const uint32_t* b) {
    for (int i = 7; i >= 0; i--)
        if (a[i] != b[i]) return a[i] < b[i];
    return false;
}
// x = (x + y) mod m, for x, y < m
void AddMod(uint32_t* x, const uint32_t* y, const uint32_t* m) {
    uint64_t c = 0;
    uint32_t s[8];
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)x[i] + y[i];
        s[i] = (uint32_t)c;
        c >>= 32;
    }
    if (c || !Less(s, m)) {
        uint64_t bw = 0;
        for (int i = 0; i < 8; i++) {
            const uint64_t t = (uint64_t)s[i] - m[i] - bw;
            s[i] = (uint32_t)t;
            bw = (t >> 63) & 1;
        }
    }
    for (int i = 0; i < 8; i++) x[i] = s[i];
}
// a * b mod m by shift-and-add over b's bits (MSB first)
void MulMod(uint32_t* out, const uint32_t* a, const uint32_t* b, const uint32_t* m) {
    uint32_t acc[8] = {0};
    for (int bit = 255; bit >= 0; bit--) {
        uint32_t d[8];
        for (int i = 0; i < 8; i++) d[i] = acc[i];
        AddMod(acc, d, m);
        if ((b[bit / 32] >> (bit % 32)) & 1) AddMod(acc, a, m);
    }
    for (int i = 0; i < 8; i++) out[i] = acc[i];
}
bool IsOne(const uint32_t* x) {
    uint32_t r = x[0] ^ 1;
    for (int i = 1; i < 8; i++) r |= x[i];
    return r == 0;
}

} // namespace

TEST_CASE(modinv_tests, inverse_mod_n_and_p) {
    std::mt19937_64 rng(42);
    for (const uint32_t* m : {N, P}) {
        // edge cases: 1, 2, m - 1, m - 2, small powers of two, and random values below m
        std::vector<std::vector<uint32_t>> xs;
        xs.push_back({1, 0, 0, 0, 0, 0, 0, 0});
        xs.push_back({2, 0, 0, 0, 0, 0, 0, 0});
        std::vector<uint32_t> m1(m, m + 8), m2(m, m + 8);
        m1[0] -= 1;
        m2[0] -= 2;
        xs.push_back(m1);
        xs.push_back(m2);
        for (int k = 0; k < 256; k += 37) {
            std::vector<uint32_t> pw(8, 0);
            pw[k / 32] = 1u << (k % 32);
            xs.push_back(pw);
        }
        for (int t = 0; t < 400; t++) {
            std::vector<uint32_t> x(8);
            for (auto& w : x) w = (uint32_t)rng();
            if (!Less(x.data(), m)) x[7] &= 0x7fffffff;
            xs.push_back(x);
        }
        int bad = 0;
        for (const auto& x : xs) {
            uint32_t inv[8], prod[8];
            if (!bcpk::modinv256(inv, x.data(), m)) {
                bad++;
                continue;
            }
            if (!Less(inv, m)) bad++;
            MulMod(prod, x.data(), inv, m);
            if (!IsOne(prod)) bad++;
        }
        CHECK_EQ(bad, 0);
    }
    // zero has no inverse
    const uint32_t zero[8] = {0};
    uint32_t out[8];
    CHECK(!bcpk::modinv256(out, zero, N));
}
