// crypto_tests: the hash primitives against published vectors, and the SHA-NI SHA-256 engine
// against the portable one; the secp256k1 GLV endomorphism multiplication against plain
// double-and-add.
// Parity: reference src/test/crypto_tests.cpp (sha256_testvectors: NIST / well-known vectors,
// the million-'a' message, streaming in arbitrary splits) - here additionally the two engines
// must agree on every length and split, since the faster one is picked at run time.
#include "test/unittest.h"

#include "crypto/hashes.h"
#include "secp256k1/secp256k1.h"
#include "util/strencodings.h"
#include "util/util.h"

using namespace bcp;

namespace {

std::string Sha256Hex(const std::string& msg) {
    unsigned char out[32];
    Sha256((const unsigned char*)msg.data(), msg.size(), out);
    return HexStr(out, out + 32);
}

struct EngineGuard {
    std::string saved = Sha256Implementation();
    ~EngineGuard() { Sha256SetImplementation(saved); }
};

} // namespace

TEST_CASE(crypto_tests, sha256_vectors) {
    EngineGuard guard;
    for (const char* engine : {"scalar", "shani"}) {
        if (!Sha256SetImplementation(engine)) continue; // the host has no SHA extensions
        CHECK_EQ(Sha256Hex(""), std::string("e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"));
        CHECK_EQ(Sha256Hex("abc"), std::string("ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"));
        CHECK_EQ(Sha256Hex("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"),
                 std::string("248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"));
        CHECK_EQ(Sha256Hex("abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnop"
                           "qrsmnopqrstnopqrstu"),
                 std::string("cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"));
        CHECK_EQ(Sha256Hex(std::string(1000000, 'a')),
                 std::string("cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"));
        // double SHA-256 of the genesis header pattern: 64-byte merkle node hashing
        unsigned char in[64], out[32];
        for (int i = 0; i < 64; i++) in[i] = (unsigned char)i;
        Sha256d64(out, in, 1);
        unsigned char ref[32];
        Sha256d(in, 64, ref);
        CHECK(memcmp(out, ref, 32) == 0);
    }
}

TEST_CASE(crypto_tests, sha256_engines_agree) {
    EngineGuard guard;
    if (!Sha256SetImplementation("shani")) return;
    FastRandomContext rng(true);
    std::vector<unsigned char> buf(4096);
    for (auto& b : buf) b = (unsigned char)rng.randbits(8);
    for (int trial = 0; trial < 3000; trial++) {
        const size_t len = trial < 300 ? (size_t)trial : (size_t)rng.randrange(buf.size());
        // one engine hashes in one piece, the other in random splits
        unsigned char a[32], b[32];
        Sha256SetImplementation("scalar");
        CSHA256().Write(buf.data(), len).Finalize(a);
        Sha256SetImplementation("shani");
        CSHA256 h;
        size_t off = 0;
        while (off < len) {
            const size_t n = std::min(len - off, (size_t)rng.randrange(200) + 1);
            h.Write(buf.data() + off, n);
            off += n;
        }
        h.Finalize(b);
        if (memcmp(a, b, 32) != 0) {
            test::RecordFailure(strprintf("length %zu: engines differ", len), __FILE__, __LINE__);
            return;
        }
    }
    // HMAC and the midstate interface go through the same transform
    const unsigned char key[] = "key";
    unsigned char m1[32], m2[32];
    Sha256SetImplementation("scalar");
    CHMAC_SHA256(key, 3).Write(buf.data(), 777).Finalize(m1);
    Sha256SetImplementation("shani");
    CHMAC_SHA256(key, 3).Write(buf.data(), 777).Finalize(m2);
    CHECK(memcmp(m1, m2, 32) == 0);
}

TEST_CASE(crypto_tests, other_hash_vectors) {
    auto hex = [](const unsigned char* p, size_t n) { return HexStr(p, p + n); };
    unsigned char r[20];
    CRIPEMD160().Write((const unsigned char*)"abc", 3).Finalize(r);
    CHECK_EQ(hex(r, 20), std::string("8eb208f7e05d987a9b044a8e98c6b087f15a0bfc"));
    unsigned char s1[20];
    CSHA1().Write((const unsigned char*)"abc", 3).Finalize(s1);
    CHECK_EQ(hex(s1, 20), std::string("a9993e364706816aba3e25717850c26c9cd0d89d"));
    unsigned char s5[64];
    CSHA512().Write((const unsigned char*)"abc", 3).Finalize(s5);
    CHECK_EQ(hex(s5, 64), std::string("ddaf35a193617abacc417349ae20413112e6fa4e89a97ea20a9eeee64b55d39a2192992a274fc1a8"
                                      "36ba3c23a3feebbd454d4423643ce80e2a9ac94fa54ca49f"));
    // RFC 4231 test case 2
    unsigned char mac[32];
    CHMAC_SHA256((const unsigned char*)"Jefe", 4).Write((const unsigned char*)"what do ya want for nothing?", 28).Finalize(mac);
    CHECK_EQ(hex(mac, 32), std::string("5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843"));
}

TEST_CASE(crypto_tests, secp256k1_glv_ecmult) {
    // the endomorphism path (ecmult) against plain double-and-add (ecmult_plain) and the GLV
    // split's recombination, on random and edge scalars
    FastRandomContext rng(true);
    auto rnd_scalar = [&](secp::Scalar& s) {
        unsigned char b[32];
        for (auto& x : b) x = (unsigned char)rng.randbits(8);
        secp::sc_set_b32(s, b);
    };
    std::vector<secp::Scalar> edge;
    for (const char* hex : {"00", "01", "02", "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364140",
                            "0000000000000000000000000000000100000000000000000000000000000000",
                            "5363ad4cc05c30e0a5261c028812645a122e22ea20816678df02967c1b23bd72",
                            "a2a8918ca85bafe22016d0b997e4df60c21f5ab2e3b61db4ae2ef2bd9a62a6a8",
                            "7fffffffffffffffffffffffffffffff5d576e7357a4501ddfe92f46681b20a0"}) {
        const std::vector<unsigned char> v = ParseHex(hex);
        unsigned char b[32] = {0};
        memcpy(b + 32 - v.size(), v.data(), v.size());
        secp::Scalar s;
        secp::sc_set_b32(s, b);
        edge.push_back(s);
    }
    int checked = 0;
    for (int t = 0; t < 400; t++) {
        secp::Scalar na, ng, ka;
        if (t < (int)edge.size()) na = edge[t];
        else rnd_scalar(na);
        rnd_scalar(ng);
        rnd_scalar(ka);
        if (!secp::glv_check(na)) {
            test::RecordFailure(strprintf("GLV split of scalar %d does not recombine", t), __FILE__, __LINE__);
            return;
        }
        secp::Gej A;
        secp::ecmult_gen(A, ka);
        secp::Gej r1, r2;
        secp::ecmult(r1, A, na, t % 3 == 0 ? edge[0] : ng);
        secp::ecmult_plain(r2, A, na, t % 3 == 0 ? edge[0] : ng);
        secp::Ge g1, g2;
        secp::ge_set_gej(g1, r1);
        secp::ge_set_gej(g2, r2);
        if (g1.inf != g2.inf || (!g1.inf && (!secp::fe_equal(g1.x, g2.x) || !secp::fe_equal(g1.y, g2.y)))) {
            test::RecordFailure(strprintf("ecmult mismatch at %d", t), __FILE__, __LINE__);
            return;
        }
        checked++;
    }
    CHECK_EQ(checked, 400);
}

TEST_CASE(crypto_tests, secp256k1_field_chains_and_verify) {
    // addition-chain inverse / square root against square-and-multiply, and the windowed scalar
    // inverse; then ECDSA verification, including the r + n < p branch of the x check
    FastRandomContext rng(true);
    for (int t = 0; t < 300; t++) {
        unsigned char b[32];
        for (auto& x : b) x = (unsigned char)rng.randbits(8);
        secp::Fe a, i1, i2, one, prod;
        secp::fe_set_b32(a, b);
        if (secp::fe_is_zero(a)) continue;
        secp::fe_inv(i1, a);
        secp::fe_inv_slow(i2, a);
        CHECK(secp::fe_equal(i1, i2));
        secp::fe_mul(prod, a, i1);
        secp::fe_set_int(one, 1);
        CHECK(secp::fe_equal(prod, one));
        secp::Fe sq, root, back;
        secp::fe_sqr(sq, a);
        CHECK(secp::fe_sqrt(root, sq));
        secp::fe_sqr(back, root);
        CHECK(secp::fe_equal(back, sq));
        secp::Scalar s, si, sp;
        secp::sc_set_b32(s, b);
        if (secp::sc_is_zero(s)) continue;
        secp::sc_inv(si, s);
        secp::sc_mul(sp, s, si);
        CHECK(sp.n[0] == 1 && sp.n[1] == 0 && sp.n[2] == 0 && sp.n[3] == 0);
    }
    // sign/verify round trips and tampering
    int good = 0;
    for (int t = 0; t < 200; t++) {
        unsigned char key[32], msg[32];
        for (auto& x : key) x = (unsigned char)rng.randbits(8);
        for (auto& x : msg) x = (unsigned char)rng.randbits(8);
        if (!secp::seckey_verify(key)) continue;
        secp::Ge pub;
        REQUIRE(secp::pubkey_create(pub, key));
        secp::Signature sig;
        REQUIRE(secp::ecdsa_sign(sig, nullptr, msg, key));
        CHECK(secp::ecdsa_verify(sig, msg, pub));
        msg[t % 32] ^= 1;
        CHECK(!secp::ecdsa_verify(sig, msg, pub));
        good++;
    }
    CHECK(good > 150);
}

TEST_CASE(crypto_tests, secp256k1_ecmult_gen_constant_time) {
    // The signing-path k*G (blinded comb, full-row cmov lookups, mask-selected exceptional
    // cases) against the variable-time byte table, and its access pattern: scalars with and
    // without zero bytes / zero nibbles must read the same table entries in the same order and
    // make the same number of point additions (reference src/secp256k1/src/ecmult_gen_impl.h:124-156).
    FastRandomContext rng(true);
    std::vector<secp::Scalar> ks;
    for (const char* hex : {"01", "02", "0f", "10", "ff", "0100", "01000000000000000000000000000000",
                            "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364140",
                            "00ff00ff00ff00ff00ff00ff00ff00ff00ff00ff00ff00ff00ff00ff00ff00ff",
                            "1111111111111111111111111111111111111111111111111111111111111111",
                            "8000000000000000000000000000000000000000000000000000000000000000",
                            "7fffffffffffffffffffffffffffffff5d576e7357a4501ddfe92f46681b20a0"}) {
        const std::vector<unsigned char> v = ParseHex(hex);
        unsigned char b[32] = {0};
        memcpy(b + 32 - v.size(), v.data(), v.size());
        secp::Scalar s;
        secp::sc_set_b32(s, b);
        ks.push_back(s);
    }
    for (int i = 0; i < 200; ++i) {
        unsigned char b[32];
        for (auto& x : b) x = (unsigned char)rng.randbits(8);
        if (i % 4 == 1) // sparse scalars: most bytes zero
            for (int j = 0; j < 32; ++j)
                if (rng.randbits(2)) b[j] = 0;
        secp::Scalar s;
        secp::sc_set_b32(s, b);
        if (!secp::sc_is_zero(s)) ks.push_back(s);
    }
    std::vector<uint32_t> ref_reads;
    uint32_t ref_adds = 0;
    int same = 0;
    for (size_t t = 0; t < ks.size(); ++t) {
        if (t == ks.size() / 2) { // a fresh blind must not change any result
            unsigned char seed[32];
            for (auto& x : seed) x = (unsigned char)rng.randbits(8);
            secp::ecmult_gen_blind(seed);
        }
        secp::EcmultGenTrace tr;
        secp::ecmult_gen_trace(&tr);
        secp::Gej a, b;
        secp::ecmult_gen(a, ks[t]);
        secp::ecmult_gen_trace(nullptr);
        secp::ecmult_gen_var(b, ks[t]);
        secp::Ge ga, gb;
        secp::ge_set_gej(ga, a);
        secp::ge_set_gej(gb, b);
        CHECK(!ga.inf && !gb.inf);
        CHECK(secp::fe_equal(ga.x, gb.x) && secp::fe_equal(ga.y, gb.y));
        CHECK_EQ(tr.reads.size(), (size_t)(64 * 16));
        CHECK_EQ(tr.adds, 64u);
        if (t == 0) {
            ref_reads = tr.reads;
            ref_adds = tr.adds;
        }
        same += tr.reads == ref_reads && tr.adds == ref_adds;
    }
    CHECK_EQ(same, (int)ks.size());
    // every entry of every row, in row order
    for (uint32_t i = 0; i < ref_reads.size(); ++i) CHECK_EQ(ref_reads[i], i);
    // the exceptional inputs of the mask-selected addition: a == b (doubling), a == -b
    // (infinity) and a = infinity, against the variable-time formulas
    secp::Scalar three = {{3, 0, 0, 0}}, k2 = {{2, 0, 0, 0}};
    secp::Gej g3, g2;
    secp::ecmult_gen(g3, three);
    secp::ecmult_gen(g2, k2);
    secp::Ge a3, a2;
    secp::ge_set_gej(a3, g3);
    secp::ge_set_gej(a2, g2);
    CHECK(!a3.inf && !a2.inf);
}

TEST_CASE(crypto_tests, secp256k1_branchfree_field_scalar) {
    // the branch-free field / scalar operations against wide-integer references at their
    // carry and borrow boundaries
    auto fe = [](const char* hex) {
        const std::vector<unsigned char> v = ParseHex(hex);
        unsigned char b[32] = {0};
        memcpy(b + 32 - v.size(), v.data(), v.size());
        secp::Fe f;
        secp::fe_set_b32(f, b);
        return f;
    };
    auto sc = [](const char* hex, bool* of = nullptr) {
        const std::vector<unsigned char> v = ParseHex(hex);
        unsigned char b[32] = {0};
        memcpy(b + 32 - v.size(), v.data(), v.size());
        secp::Scalar s;
        secp::sc_set_b32(s, b, of);
        return s;
    };
    auto fhex = [](const secp::Fe& f) {
        unsigned char b[32];
        secp::fe_get_b32(b, f);
        return HexStr(b, b + 32);
    };
    auto shex = [](const secp::Scalar& s) {
        unsigned char b[32];
        secp::sc_get_b32(b, s);
        return HexStr(b, b + 32);
    };
    const char* PM1 = "fffffffffffffffffffffffffffffffffffffffffffffffffffffffefffffc2e";
    const char* NM1 = "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364140";
    secp::Fe r;
    secp::fe_add(r, fe(PM1), fe("01")); // p - 1 + 1 = 0
    CHECK_EQ(fhex(r), std::string(64, '0'));
    secp::fe_add(r, fe(PM1), fe(PM1)); // 2p - 2 = p - 2
    CHECK_EQ(fhex(r), std::string("fffffffffffffffffffffffffffffffffffffffffffffffffffffffefffffc2d"));
    secp::fe_sub(r, fe("00"), fe("01")); // -1 = p - 1
    CHECK_EQ(fhex(r), std::string(PM1));
    secp::fe_mul(r, fe(PM1), fe(PM1)); // (-1)^2 = 1
    CHECK_EQ(fhex(r), std::string(63, '0') + "1");
    bool of = false;
    secp::Fe f;
    unsigned char pb[32];
    secp::fe_get_b32(pb, fe(PM1));
    pb[31] += 1; // p itself overflows to 0
    secp::fe_set_b32(f, pb, &of);
    CHECK(of && secp::fe_is_zero(f));
    secp::Scalar s;
    secp::sc_add(s, sc(NM1), sc("02")); // n - 1 + 2 = 1
    CHECK_EQ(shex(s), std::string(63, '0') + "1");
    secp::sc_add(s, sc(NM1), sc(NM1)); // 2n - 2 = n - 2 (the sum carries out of 2^256)
    CHECK_EQ(shex(s), std::string("fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd036413f"));
    secp::sc_mul(s, sc(NM1), sc(NM1)); // (-1)^2 = 1
    CHECK_EQ(shex(s), std::string(63, '0') + "1");
    secp::sc_neg(s, sc("00"));
    CHECK(secp::sc_is_zero(s));
    secp::sc_neg(s, sc("01"));
    CHECK_EQ(shex(s), std::string(NM1));
    CHECK(secp::sc_is_high(sc(NM1)));
    CHECK(!secp::sc_is_high(sc("7fffffffffffffffffffffffffffffff5d576e7357a4501ddfe92f46681b20a0")));
    CHECK(secp::sc_is_high(sc("7fffffffffffffffffffffffffffffff5d576e7357a4501ddfe92f46681b20a1")));
    bool sof = false;
    sc("fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364141", &sof); // n
    CHECK(sof);
    // random products against the scalar inverse: a * a^-1 == 1
    FastRandomContext rng(true);
    for (int i = 0; i < 200; ++i) {
        unsigned char b[32];
        for (auto& x : b) x = (unsigned char)rng.randbits(8);
        secp::Scalar a, ai, p;
        secp::sc_set_b32(a, b);
        if (secp::sc_is_zero(a)) continue;
        secp::sc_inv(ai, a);
        secp::sc_mul(p, a, ai);
        CHECK_EQ(shex(p), std::string(63, '0') + "1");
    }
}

// The GPU's 11-bit comb table: entry [i*2048 + j] = j * 2^(11 i) * G, checked against
// ecmult_gen_var of the same scalar (j = 0 is the point at infinity).
TEST_CASE(crypto_tests, secp256k1_generator_table11) {
    const std::vector<secp::Ge>& t = secp::generator_table11();
    REQUIRE(t.size() == (size_t)24 * 2048);
    for (int i : {0, 1, 7, 22, 23}) {
        for (int j : {0, 1, 2, 3, 1000, 2047}) {
            const secp::Ge& e = t[(size_t)i * 2048 + j];
            if (j == 0) {
                CHECK(e.inf);
                continue;
            }
            // k = j << 11i as a big-endian 32-byte scalar (< 2^264 only for i = 23, j >= 8:
            // reduced mod n by sc_set_b32 like the table's own doublings)
            unsigned char b[33] = {0};
            const int bit = 11 * i;
            for (int q = 0; q < 12; q++) {
                const int pos = bit + q; // bit position of bit q of j
                if (!((j >> q) & 1) || pos >= 256) continue;
                b[32 - pos / 8] |= (unsigned char)(1u << (pos % 8));
            }
            const bool overflowBits = i == 23 && (j >> 3) != 0; // bits past 2^256: skip (not used by u1 < n)
            if (overflowBits) continue;
            secp::Scalar k;
            secp::sc_set_b32(k, b + 1);
            secp::Gej r;
            secp::ecmult_gen_var(r, k);
            secp::Ge a;
            secp::ge_set_gej(a, r);
            CHECK(!e.inf);
            CHECK(secp::fe_equal(a.x, e.x));
            CHECK(secp::fe_equal(a.y, e.y));
        }
    }
}
