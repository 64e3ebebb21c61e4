// secp256k1 elliptic-curve arithmetic, ECDSA and public-key recovery (CPU reference).
//
// Replaces the reference's vendored libsecp256k1 (src/secp256k1/, used through
// CPubKey::Verify src/pubkey.cpp:170-193, CKey::Sign/SignCompact src/key.cpp,
// RecoverCompact src/pubkey.cpp) with a self-contained implementation:
//   field  : 4 x 64-bit limbs mod p = 2^256 - 2^32 - 977, products via unsigned __int128
//   scalar : 4 x 64-bit limbs mod n
//   points : Jacobian coordinates; u1*G from a 32 x 255 precomputed byte-window table,
//            u2*P by width-5 wNAF (Strauss-style verification)
//   signing: RFC 6979 HMAC-SHA256 nonces (optionally with 32 bytes of extra entropy,
//            exactly as libsecp256k1's nonce_function_rfc6979), low-S output.
// Verification semantics match CPubKey::Verify: lax-DER parse, low-S normalisation,
// r,s in [1, n-1], pubkeys in compressed/uncompressed/hybrid form.
// The throughput path is the batched GPU verifier (csrc/kernels/secp256k1.hip).
// Secret-scalar paths are constant-time: field and scalar arithmetic are branch-free, and
// ecmult_gen (signing nonces, pubkey_create, BIP32 private derivation) is a blinded comb whose
// table rows are scanned in full and whose additions select their exceptional cases by mask
// (reference src/secp256k1/src/ecmult_gen_impl.h:124-156). Verification and recovery work on
// public values and use the faster variable-time ecmult / ecmult_gen_var.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace bcp {
namespace secp {

struct Fe {
    uint64_t n[4]; // little-endian limbs, always fully reduced (< p)
};
struct Scalar {
    uint64_t n[4]; // little-endian limbs, always reduced (< n)
};
struct Ge { // affine point
    Fe x, y;
    bool inf = true;
};
struct Gej { // Jacobian point
    Fe x, y, z;
    bool inf = true;
};

// ---- field
void fe_set_b32(Fe& r, const unsigned char* b32, bool* overflow = nullptr);
void fe_get_b32(unsigned char* b32, const Fe& a);
void fe_set_int(Fe& r, uint64_t v);
bool fe_is_zero(const Fe& a);
bool fe_equal(const Fe& a, const Fe& b);
bool fe_is_odd(const Fe& a);
void fe_add(Fe& r, const Fe& a, const Fe& b);
void fe_sub(Fe& r, const Fe& a, const Fe& b);
void fe_neg(Fe& r, const Fe& a);
void fe_mul(Fe& r, const Fe& a, const Fe& b);
void fe_sqr(Fe& r, const Fe& a);
void fe_inv(Fe& r, const Fe& a);      // addition chain
void fe_inv_slow(Fe& r, const Fe& a); // plain square-and-multiply (tests)
bool fe_sqrt(Fe& r, const Fe& a); // false if a is not a square

// ---- scalar
void sc_set_b32(Scalar& r, const unsigned char* b32, bool* overflow = nullptr);
void sc_get_b32(unsigned char* b32, const Scalar& a);
bool sc_is_zero(const Scalar& a);
bool sc_is_high(const Scalar& a);
void sc_add(Scalar& r, const Scalar& a, const Scalar& b);
void sc_mul(Scalar& r, const Scalar& a, const Scalar& b);
void sc_neg(Scalar& r, const Scalar& a);
void sc_inv(Scalar& r, const Scalar& a);

// ---- group
const Ge& generator();
void gej_set_ge(Gej& r, const Ge& a);
void gej_double(Gej& r, const Gej& a);
void gej_add_ge(Gej& r, const Gej& a, const Ge& b);
void gej_add(Gej& r, const Gej& a, const Gej& b);
void ge_set_gej(Ge& r, const Gej& a);
bool ge_is_valid(const Ge& a);
void ecmult_gen(Gej& r, const Scalar& k);     // constant-time, blinded (secret k)
void ecmult_gen_var(Gej& r, const Scalar& k); // variable-time (public k only)
// Re-randomise the signing blind (libsecp256k1's context_randomize); nullptr = /dev/urandom.
// A blind is drawn from /dev/urandom on first use anyway.
void ecmult_gen_blind(const unsigned char* seed32);
// Test instrumentation: while set (per thread), ecmult_gen appends the index (row * 16 + entry) of
// every table entry it reads and counts its point additions.
struct EcmultGenTrace {
    std::vector<uint32_t> reads;
    uint32_t adds = 0;
};
void ecmult_gen_trace(EcmultGenTrace* t);
// Affine comb table, entry [i*256 + j] = j * 256^i * G (j = 0 is the point at infinity).
const std::vector<Ge>& generator_table();                                  // k*G
// Entry [i*2048 + j] = j * 2^(11 i) * G, i < 24 (the GPU's 11-bit comb; j = 0 is infinity).
const std::vector<Ge>& generator_table11();
void ecmult(Gej& r, const Gej& a, const Scalar& na, const Scalar& ng);     // na*A + ng*G (GLV)
void ecmult_plain(Gej& r, const Gej& a, const Scalar& na, const Scalar& ng); // same, no endomorphism
bool glv_check(const Scalar& k); // the GLV split of k recombines to k with halves < 2^130 (tests)

// ---- keys / serialization
bool pubkey_parse(Ge& r, const unsigned char* in, size_t len);
std::vector<unsigned char> pubkey_serialize(const Ge& p, bool compressed);
bool seckey_verify(const unsigned char* seckey32);
bool pubkey_create(Ge& r, const unsigned char* seckey32);
bool seckey_tweak_add(unsigned char* seckey32, const unsigned char* tweak32);
bool pubkey_tweak_add(Ge& p, const unsigned char* tweak32);

// ---- ECDSA
struct Signature {
    Scalar r, s;
};
bool sig_parse_compact(Signature& sig, const unsigned char* in64); // false on overflow
void sig_serialize_compact(unsigned char* out64, const Signature& sig);
// Lax DER as used by CPubKey::Verify (reference src/pubkey.cpp ecdsa_signature_parse_der_lax).
bool sig_parse_der_lax(Signature& sig, const unsigned char* in, size_t len);
bool sig_parse_der_strict(Signature& sig, const unsigned char* in, size_t len);
std::vector<unsigned char> sig_serialize_der(const Signature& sig);
bool sig_normalize(Signature& sig); // returns true if it was high-S
bool ecdsa_verify(const Signature& sig, const unsigned char* msg32, const Ge& pub); // requires low-S
// Sign; extra32 may be null. recid receives the recovery id. Result is low-S.
bool ecdsa_sign(Signature& sig, int* recid, const unsigned char* msg32, const unsigned char* seckey32,
                const unsigned char* extra32 = nullptr);
bool ecdsa_recover(Ge& pub, const Signature& sig, int recid, const unsigned char* msg32);

// RFC 6979 nonce generation (HMAC-DRBG over SHA-256), exposed for tests.
void rfc6979_nonce(unsigned char* out32, const unsigned char* msg32, const unsigned char* key32,
                   const unsigned char* extra32, unsigned int counter);

// Full CPubKey::Verify semantics on serialized inputs.
bool VerifySignature(const unsigned char* pub, size_t publen, const unsigned char* sig, size_t siglen,
                     const unsigned char* msg32);

} // namespace secp
} // namespace bcp
