// crypto_tests: the hash primitives against published vectors, and the SHA-NI SHA-256 engine
// against the portable one.
// Parity: reference src/test/crypto_tests.cpp (sha256_testvectors: NIST / well-known vectors,
// the million-'a' message, streaming in arbitrary splits) - here additionally the two engines
// must agree on every length and split, since the faster one is picked at run time.
#include "test/unittest.h"

#include "crypto/hashes.h"
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
