// wallet_crypto: CCrypter against OpenSSL's EVP interface, the way the reference wallet
// encrypted before it had its own AES: EVP_BytesToKey(AES-256-CBC, SHA-512) for the passphrase
// derivation (with the reference's known key/IV for "test" at 25000 rounds, and every suffix of
// a random passphrase at random rounds), and EVP AES-256-CBC for encrypt and decrypt (every
// suffix of the plaintext, 100 random 32-byte plaintexts, and corrupt-padding ciphertexts whose
// decrypt must fail the same way).
// Parity: reference src/wallet/test/crypto_tests.cpp (passphrase, encrypt, decrypt).
#include "test/unittest.h"

#include "util/strencodings.h"
#include "wallet/crypter.h"

#include <openssl/evp.h>

#include <cstring>

namespace bcp {

struct CrypterTestAccess {
    static const unsigned char* Key(const CCrypter& c) { return c.vchKey; }
    static const unsigned char* IV(const CCrypter& c) { return c.vchIV; }
};

} // namespace bcp

using namespace bcp;

namespace {

bool OldSetKeyFromPassphrase(const std::string& pass, const std::vector<unsigned char>& salt, unsigned rounds,
                             unsigned char* key, unsigned char* iv) {
    if (rounds < 1 || salt.size() != WALLET_CRYPTO_SALT_SIZE) return false;
    const int n = EVP_BytesToKey(EVP_aes_256_cbc(), EVP_sha512(), salt.data(),
                                 reinterpret_cast<const unsigned char*>(pass.data()), (int)pass.size(), (int)rounds, key,
                                 iv);
    return n == (int)WALLET_CRYPTO_KEY_SIZE;
}

bool OldCrypt(bool enc, const unsigned char* in, size_t n, std::vector<unsigned char>& out, const unsigned char* key,
              const unsigned char* iv) {
    out.assign(n + 16, 0);
    int len = 0, flen = 0;
    EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
    if (!ctx) return false;
    bool ok = EVP_CipherInit_ex(ctx, EVP_aes_256_cbc(), nullptr, key, iv, enc ? 1 : 0) != 0;
    ok = ok && EVP_CipherUpdate(ctx, out.data(), &len, in, (int)n) != 0;
    ok = ok && EVP_CipherFinal_ex(ctx, out.data() + len, &flen) != 0;
    EVP_CIPHER_CTX_free(ctx);
    if (!ok) return false;
    out.resize(len + flen);
    return true;
}

void TestPassphraseSingle(const std::vector<unsigned char>& salt, const std::string& pass, unsigned rounds,
                          const std::vector<unsigned char>& correctKey = {},
                          const std::vector<unsigned char>& correctIV = {}) {
    CCrypter crypt;
    CHECK(crypt.SetKeyFromPassphrase(pass, salt, rounds, 0));
    unsigned char key[WALLET_CRYPTO_KEY_SIZE], iv[WALLET_CRYPTO_IV_SIZE];
    CHECK(OldSetKeyFromPassphrase(pass, salt, rounds, key, iv));
    CHECK(memcmp(key, CrypterTestAccess::Key(crypt), sizeof(key)) == 0);
    CHECK(memcmp(iv, CrypterTestAccess::IV(crypt), sizeof(iv)) == 0);
    if (!correctKey.empty()) CHECK(memcmp(key, correctKey.data(), sizeof(key)) == 0);
    if (!correctIV.empty()) CHECK(memcmp(iv, correctIV.data(), sizeof(iv)) == 0);
}

void TestPassphrase(const std::vector<unsigned char>& salt, const std::string& pass, unsigned rounds,
                    const std::vector<unsigned char>& correctKey = {}, const std::vector<unsigned char>& correctIV = {}) {
    TestPassphraseSingle(salt, pass, rounds, correctKey, correctIV);
    for (size_t i = 0; i < pass.size(); i++) TestPassphraseSingle(salt, pass.substr(i), rounds);
}

void TestDecrypt(const CCrypter& crypt, const std::vector<unsigned char>& cipher,
                 const std::vector<unsigned char>& plain = {}) {
    CKeyingMaterial d1;
    std::vector<unsigned char> d2;
    const bool r1 = crypt.Decrypt(cipher, d1);
    const bool r2 = OldCrypt(false, cipher.data(), cipher.size(), d2, CrypterTestAccess::Key(crypt),
                             CrypterTestAccess::IV(crypt));
    CHECK_EQ(r1, r2);
    if (r1 && r2) CHECK(std::vector<unsigned char>(d1.begin(), d1.end()) == d2);
    if (!plain.empty()) CHECK(d2 == plain);
}

void TestEncryptSingle(const CCrypter& crypt, const CKeyingMaterial& plain) {
    std::vector<unsigned char> c1, c2;
    const bool r1 = crypt.Encrypt(plain, c1);
    const bool r2 = OldCrypt(true, plain.data(), plain.size(), c2, CrypterTestAccess::Key(crypt),
                             CrypterTestAccess::IV(crypt));
    CHECK_EQ(r1, r2);
    CHECK(c1 == c2);
    if (c1 == c2) TestDecrypt(crypt, c1, std::vector<unsigned char>(plain.begin(), plain.end()));
}

void TestEncrypt(const CCrypter& crypt, const std::vector<unsigned char>& plain) {
    TestEncryptSingle(crypt, CKeyingMaterial(plain.begin(), plain.end()));
    for (size_t i = 0; i < plain.size(); i++) TestEncryptSingle(crypt, CKeyingMaterial(plain.begin() + i, plain.end()));
}

} // namespace

TEST_CASE(wallet_crypto, passphrase) {
    TestPassphrase(ParseHex("0000deadbeef0000"), "test", 25000,
                   ParseHex("fc7aba077ad5f4c3a0988d8daa4810d0d4a0e3bcb53af662998898f33df0556a"),
                   ParseHex("cf2f2691526dd1aa220896fb8bf7c369"));
    FastRandomContext rng;
    const std::string pass = GetRandHash().ToString();
    std::vector<unsigned char> salt(8);
    GetRandBytes(salt.data(), salt.size());
    TestPassphrase(salt, pass, 1 + (unsigned)rng.randrange(30000));
}

TEST_CASE(wallet_crypto, encrypt) {
    const std::vector<unsigned char> salt = ParseHex("0000deadbeef0000");
    CHECK_EQ(salt.size(), (size_t)WALLET_CRYPTO_SALT_SIZE);
    CCrypter crypt;
    CHECK(crypt.SetKeyFromPassphrase("passphrase", salt, 25000, 0));
    TestEncrypt(crypt, ParseHex("22bcade09ac03ff6386914359cfe885cfeb5f77ff0d670f102f619687453b29d"));
    for (int i = 0; i < 100; i++) {
        const uint256 h = GetRandHash();
        TestEncrypt(crypt, std::vector<unsigned char>(h.begin(), h.end()));
    }
}

TEST_CASE(wallet_crypto, decrypt) {
    const std::vector<unsigned char> salt = ParseHex("0000deadbeef0000");
    CCrypter crypt;
    CHECK(crypt.SetKeyFromPassphrase("passphrase", salt, 25000, 0));
    // corner cases (mostly bad padding) from the reference
    for (const char* hex : {"795643ce39d736088367822cdc50535ec6f103715e3e48f4f3b1a60a08ef59ca",
                            "de096f4a8f9bd97db012aa9d90d74de8cdea779c3ee8bc7633d8b5d6da703486",
                            "32d0a8974e3afd9c6c3ebf4d66aa4e6419f8c173de25947f98cf8b7ace49449c",
                            "e7c055cca2faa78cb9ac22c9357a90b4778ded9b2cc220a14cea49f931e596ea",
                            "b88efddd668a6801d19516d6830da4ae9811988ccbaf40df8fbb72f3f4d335fd",
                            "8cae76aa6a43694e961ebcb28c8ca8f8540b84153d72865e8561ddd93fa7bfa9"})
        TestDecrypt(crypt, ParseHex(hex));
    for (int i = 0; i < 100; i++) {
        const uint256 h = GetRandHash();
        TestDecrypt(crypt, std::vector<unsigned char>(h.begin(), h.end()));
    }
}
