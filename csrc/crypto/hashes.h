// Streaming hash primitives used by the consensus core, wallet and P2P layer.
//
// Parity map (behaviour, not code):
//   CSHA256      <- reference src/crypto/sha256.{h,cpp}   (sha256::Transform, CSHA256)
//   CSHA512      <- reference src/crypto/sha512.{h,cpp}
//   CSHA1        <- reference src/crypto/sha1.{h,cpp}
//   CRIPEMD160   <- reference src/crypto/ripemd160.{h,cpp}
//   CHMAC_SHA256/CHMAC_SHA512 <- reference src/crypto/hmac_sha{256,512}.{h,cpp}
//   CBlake2b     <- libsodium crypto_generichash_blake2b_* as used by
//                   reference src/crypto/equihash.cpp:36-60 (personalised, unkeyed)
//   SipHash      <- reference src/hash.{h,cpp}:181-300 (CSipHasher, SipHashUint256[Extra])
//   ChaCha20     <- reference src/crypto/chacha20.{h,cpp}
//
// The CPU implementations are portable scalar code (SHA-256 on the x86 SHA extensions when the
// host has them, crypto/sha256_x86.cpp); the throughput paths
// (SHA-256d batches, BLAKE2b for Equihash) live in csrc/kernels/*.hip.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace bcp {

class CSHA256 {
public:
    static const size_t OUTPUT_SIZE = 32;
    CSHA256();
    CSHA256& Write(const unsigned char* data, size_t len);
    void Finalize(unsigned char hash[OUTPUT_SIZE]);
    CSHA256& Reset();
    // Midstate access (used to precompute header midstates for GPU nonce sweeps).
    const uint32_t* State() const { return s; }
    uint64_t BytesHashed() const { return bytes; }
    static void Transform(uint32_t* s, const unsigned char* chunk, size_t blocks);
private:
    uint32_t s[8];
    unsigned char buf[64];
    uint64_t bytes;
};

class CSHA512 {
public:
    static const size_t OUTPUT_SIZE = 64;
    CSHA512();
    CSHA512& Write(const unsigned char* data, size_t len);
    void Finalize(unsigned char hash[OUTPUT_SIZE]);
    CSHA512& Reset();
private:
    uint64_t s[8];
    unsigned char buf[128];
    uint64_t bytes;
};

class CSHA1 {
public:
    static const size_t OUTPUT_SIZE = 20;
    CSHA1();
    CSHA1& Write(const unsigned char* data, size_t len);
    void Finalize(unsigned char hash[OUTPUT_SIZE]);
    CSHA1& Reset();
private:
    uint32_t s[5];
    unsigned char buf[64];
    uint64_t bytes;
};

class CRIPEMD160 {
public:
    static const size_t OUTPUT_SIZE = 20;
    CRIPEMD160();
    CRIPEMD160& Write(const unsigned char* data, size_t len);
    void Finalize(unsigned char hash[OUTPUT_SIZE]);
    CRIPEMD160& Reset();
private:
    uint32_t s[5];
    unsigned char buf[64];
    uint64_t bytes;
};

class CHMAC_SHA256 {
public:
    static const size_t OUTPUT_SIZE = 32;
    CHMAC_SHA256(const unsigned char* key, size_t keylen);
    CHMAC_SHA256& Write(const unsigned char* data, size_t len) { inner.Write(data, len); return *this; }
    void Finalize(unsigned char hash[OUTPUT_SIZE]);
private:
    CSHA256 outer, inner;
};

class CHMAC_SHA512 {
public:
    static const size_t OUTPUT_SIZE = 64;
    CHMAC_SHA512(const unsigned char* key, size_t keylen);
    CHMAC_SHA512& Write(const unsigned char* data, size_t len) { inner.Write(data, len); return *this; }
    void Finalize(unsigned char hash[OUTPUT_SIZE]);
private:
    CSHA512 outer, inner;
};

// BLAKE2b (RFC 7693) with the full parameter block: digest length, key,
// salt and personalisation. The state is a plain POD so it can be copied
// byte-for-byte to the GPU (Equihash base state).
struct Blake2bState {
    uint64_t h[8];
    uint64_t t[2];
    uint64_t f[2];
    unsigned char buf[128];
    uint32_t buflen;
    uint32_t outlen;
};

class CBlake2b {
public:
    CBlake2b(size_t outlen, const unsigned char* key = nullptr, size_t keylen = 0,
             const unsigned char* salt16 = nullptr, const unsigned char* personal16 = nullptr);
    CBlake2b& Write(const unsigned char* data, size_t len);
    void Finalize(unsigned char* out); // writes outlen bytes
    const Blake2bState& GetState() const { return st; }
    Blake2bState& MutableState() { return st; }
    size_t OutLen() const { return st.outlen; }
    static void Compress(uint64_t h[8], const unsigned char block[128], uint64_t t0, uint64_t t1, bool last);
private:
    Blake2bState st;
};

// SipHash-2-4 (streaming, 8-byte words and raw bytes).
class CSipHasher {
public:
    CSipHasher(uint64_t k0, uint64_t k1);
    CSipHasher& Write(uint64_t data);
    CSipHasher& Write(const unsigned char* data, size_t size);
    uint64_t Finalize() const;
private:
    uint64_t v[4];
    uint64_t tmp;
    int count;
};
// Optimised SipHash of a 32-byte value (+ optional 32-bit extra), reference src/hash.cpp:181-300.
uint64_t SipHashUint256(uint64_t k0, uint64_t k1, const unsigned char val[32]);
uint64_t SipHashUint256Extra(uint64_t k0, uint64_t k1, const unsigned char val[32], uint32_t extra);

class ChaCha20 {
public:
    ChaCha20();
    ChaCha20(const unsigned char* key, size_t keylen);
    void SetKey(const unsigned char* key, size_t keylen);
    void SetIV(uint64_t iv);
    void Seek(uint64_t pos);
    void Output(unsigned char* output, size_t bytes);
private:
    uint32_t input[16];
};

// AES-256-CBC with PKCS7 padding (wallet encryption, reference src/crypto/aes.{h,cpp}).
class AES256CBCEncrypt {
public:
    AES256CBCEncrypt(const unsigned char key[32], const unsigned char iv[16], bool pad);
    ~AES256CBCEncrypt();
    int Encrypt(const unsigned char* data, int size, unsigned char* out) const;
private:
    uint32_t rk[60];
    unsigned char iv[16];
    bool pad;
};
class AES256CBCDecrypt {
public:
    AES256CBCDecrypt(const unsigned char key[32], const unsigned char iv[16], bool pad);
    ~AES256CBCDecrypt();
    int Decrypt(const unsigned char* data, int size, unsigned char* out) const;
private:
    uint32_t rk[60];
    unsigned char iv[16];
    bool pad;
};

// Convenience one-shots.
void Sha256(const unsigned char* data, size_t len, unsigned char out[32]);
void Sha256d(const unsigned char* data, size_t len, unsigned char out[32]);
void Sha256d64(unsigned char* out, const unsigned char* in, size_t blocks); // N x (64 B -> 32 B)
void Hash160(const unsigned char* data, size_t len, unsigned char out[20]);
// The SHA-256 compression engine in use: "shani" (x86 SHA extensions, chosen when the CPU has
// them) or "scalar". Setting is for tests and benchmarks; it is not thread-safe against hashing.
std::string Sha256Implementation();
bool Sha256SetImplementation(const std::string& name);

} // namespace bcp
