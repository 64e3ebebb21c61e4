// SHA-256 / SHA-512 / SHA-1 / RIPEMD-160 / HMAC — portable scalar CPU versions.
// Behaviour parity: reference src/crypto/{sha256,sha512,sha1,ripemd160,hmac_sha256,hmac_sha512}.cpp
#include "crypto/hashes.h"
#include "crypto/common.h"

#include <atomic>
#include <cstring>

namespace bcp {

// memory_cleanse lives in util/lockedpool.cpp

// ---------------------------------------------------------------- SHA-256
namespace {
const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

const uint32_t H256[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                          0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
} // namespace

namespace sha256_x86 {
bool Available();
void Transform(uint32_t* s, const unsigned char* chunk, size_t blocks);
} // namespace sha256_x86

namespace {
void TransformScalar(uint32_t* st, const unsigned char* chunk, size_t blocks);
void TransformResolve(uint32_t* st, const unsigned char* chunk, size_t blocks);
using TransformFn = void (*)(uint32_t*, const unsigned char*, size_t);
// constant-initialised, so hashing during other translation units' static initialisation works;
// the first call picks the engine
std::atomic<TransformFn> g_transform{TransformResolve};

void TransformResolve(uint32_t* st, const unsigned char* chunk, size_t blocks) {
    const TransformFn f = sha256_x86::Available() ? sha256_x86::Transform : TransformScalar;
    g_transform.store(f, std::memory_order_relaxed);
    f(st, chunk, blocks);
}
} // namespace

void CSHA256::Transform(uint32_t* st, const unsigned char* chunk, size_t blocks) {
    g_transform.load(std::memory_order_relaxed)(st, chunk, blocks);
}

std::string Sha256Implementation() {
    TransformFn f = g_transform.load();
    if (f == TransformResolve) f = sha256_x86::Available() ? sha256_x86::Transform : TransformScalar;
    return f == TransformScalar ? "scalar" : "shani";
}

bool Sha256SetImplementation(const std::string& name) {
    if (name == "scalar") g_transform = TransformScalar;
    else if (name == "shani" && sha256_x86::Available()) g_transform = sha256_x86::Transform;
    else return false;
    return true;
}

namespace {
void TransformScalar(uint32_t* st, const unsigned char* chunk, size_t blocks) {
    while (blocks--) {
        uint32_t w[64];
        for (int i = 0; i < 16; ++i) w[i] = ReadBE32(chunk + 4 * i);
        for (int i = 16; i < 64; ++i) {
            uint32_t s0 = Rotr32(w[i - 15], 7) ^ Rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = Rotr32(w[i - 2], 17) ^ Rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
        for (int i = 0; i < 64; ++i) {
            uint32_t S1 = Rotr32(e, 6) ^ Rotr32(e, 11) ^ Rotr32(e, 25);
            uint32_t ch = (e & f) ^ (~e & g);
            uint32_t t1 = h + S1 + ch + K256[i] + w[i];
            uint32_t S0 = Rotr32(a, 2) ^ Rotr32(a, 13) ^ Rotr32(a, 22);
            uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
            uint32_t t2 = S0 + mj;
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
        chunk += 64;
    }
}
} // namespace

CSHA256::CSHA256() : bytes(0) { memcpy(s, H256, sizeof(s)); }

CSHA256& CSHA256::Reset() { bytes = 0; memcpy(s, H256, sizeof(s)); return *this; }

CSHA256& CSHA256::Write(const unsigned char* data, size_t len) {
    const unsigned char* end = data + len;
    size_t bufsize = bytes % 64;
    if (bufsize && bufsize + len >= 64) {
        memcpy(buf + bufsize, data, 64 - bufsize);
        bytes += 64 - bufsize;
        data += 64 - bufsize;
        Transform(s, buf, 1);
        bufsize = 0;
    }
    if (end - data >= 64) {
        size_t blocks = (end - data) / 64;
        Transform(s, data, blocks);
        data += 64 * blocks;
        bytes += 64 * blocks;
    }
    if (end > data) {
        memcpy(buf + bufsize, data, end - data);
        bytes += end - data;
    }
    return *this;
}

void CSHA256::Finalize(unsigned char hash[OUTPUT_SIZE]) {
    static const unsigned char pad[64] = {0x80};
    unsigned char sizedesc[8];
    WriteBE64(sizedesc, bytes << 3);
    Write(pad, 1 + ((119 - (bytes % 64)) % 64));
    Write(sizedesc, 8);
    for (int i = 0; i < 8; ++i) WriteBE32(hash + 4 * i, s[i]);
}

void Sha256(const unsigned char* data, size_t len, unsigned char out[32]) {
    CSHA256().Write(data, len).Finalize(out);
}

void Sha256d(const unsigned char* data, size_t len, unsigned char out[32]) {
    unsigned char t[32];
    CSHA256().Write(data, len).Finalize(t);
    CSHA256().Write(t, 32).Finalize(out);
}

void Sha256d64(unsigned char* out, const unsigned char* in, size_t blocks) {
    for (size_t i = 0; i < blocks; ++i) Sha256d(in + 64 * i, 64, out + 32 * i);
}

// ---------------------------------------------------------------- SHA-512
namespace {
const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

void Sha512Transform(uint64_t* st, const unsigned char* chunk) {
    uint64_t w[80];
    for (int i = 0; i < 16; ++i) w[i] = ReadBE64(chunk + 8 * i);
    for (int i = 16; i < 80; ++i) {
        uint64_t s0 = Rotr64(w[i - 15], 1) ^ Rotr64(w[i - 15], 8) ^ (w[i - 15] >> 7);
        uint64_t s1 = Rotr64(w[i - 2], 19) ^ Rotr64(w[i - 2], 61) ^ (w[i - 2] >> 6);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 80; ++i) {
        uint64_t S1 = Rotr64(e, 14) ^ Rotr64(e, 18) ^ Rotr64(e, 41);
        uint64_t ch = (e & f) ^ (~e & g);
        uint64_t t1 = h + S1 + ch + K512[i] + w[i];
        uint64_t S0 = Rotr64(a, 28) ^ Rotr64(a, 34) ^ Rotr64(a, 39);
        uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
} // namespace

CSHA512::CSHA512() : bytes(0) { Reset(); }

CSHA512& CSHA512::Reset() {
    static const uint64_t H[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                  0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                  0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    memcpy(s, H, sizeof(s));
    bytes = 0;
    return *this;
}

CSHA512& CSHA512::Write(const unsigned char* data, size_t len) {
    const unsigned char* end = data + len;
    size_t bufsize = bytes % 128;
    if (bufsize && bufsize + len >= 128) {
        memcpy(buf + bufsize, data, 128 - bufsize);
        bytes += 128 - bufsize;
        data += 128 - bufsize;
        Sha512Transform(s, buf);
        bufsize = 0;
    }
    while (end - data >= 128) {
        Sha512Transform(s, data);
        data += 128;
        bytes += 128;
    }
    if (end > data) {
        memcpy(buf + bufsize, data, end - data);
        bytes += end - data;
    }
    return *this;
}

void CSHA512::Finalize(unsigned char hash[OUTPUT_SIZE]) {
    static const unsigned char pad[128] = {0x80};
    unsigned char sizedesc[16] = {0};
    WriteBE64(sizedesc + 8, bytes << 3);
    Write(pad, 1 + ((239 - (bytes % 128)) % 128));
    Write(sizedesc, 16);
    for (int i = 0; i < 8; ++i) WriteBE64(hash + 8 * i, s[i]);
}

// ---------------------------------------------------------------- SHA-1
namespace {
void Sha1Transform(uint32_t* st, const unsigned char* chunk) {
    uint32_t w[80];
    for (int i = 0; i < 16; ++i) w[i] = ReadBE32(chunk + 4 * i);
    for (int i = 16; i < 80; ++i) w[i] = Rotl32(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
    for (int i = 0; i < 80; ++i) {
        uint32_t f, k;
        if (i < 20) { f = (b & c) | (~b & d); k = 0x5a827999; }
        else if (i < 40) { f = b ^ c ^ d; k = 0x6ed9eba1; }
        else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdc; }
        else { f = b ^ c ^ d; k = 0xca62c1d6; }
        uint32_t t = Rotl32(a, 5) + f + e + k + w[i];
        e = d; d = c; c = Rotl32(b, 30); b = a; a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}
} // namespace

CSHA1::CSHA1() { Reset(); }
CSHA1& CSHA1::Reset() {
    s[0] = 0x67452301; s[1] = 0xEFCDAB89; s[2] = 0x98BADCFE; s[3] = 0x10325476; s[4] = 0xC3D2E1F0;
    bytes = 0;
    return *this;
}
CSHA1& CSHA1::Write(const unsigned char* data, size_t len) {
    const unsigned char* end = data + len;
    size_t bufsize = bytes % 64;
    if (bufsize && bufsize + len >= 64) {
        memcpy(buf + bufsize, data, 64 - bufsize);
        bytes += 64 - bufsize; data += 64 - bufsize;
        Sha1Transform(s, buf);
        bufsize = 0;
    }
    while (end - data >= 64) { Sha1Transform(s, data); data += 64; bytes += 64; }
    if (end > data) { memcpy(buf + bufsize, data, end - data); bytes += end - data; }
    return *this;
}
void CSHA1::Finalize(unsigned char hash[OUTPUT_SIZE]) {
    static const unsigned char pad[64] = {0x80};
    unsigned char sizedesc[8];
    WriteBE64(sizedesc, bytes << 3);
    Write(pad, 1 + ((119 - (bytes % 64)) % 64));
    Write(sizedesc, 8);
    for (int i = 0; i < 5; ++i) WriteBE32(hash + 4 * i, s[i]);
}

// ---------------------------------------------------------------- RIPEMD-160
namespace {
inline uint32_t rf1(uint32_t x, uint32_t y, uint32_t z) { return x ^ y ^ z; }
inline uint32_t rf2(uint32_t x, uint32_t y, uint32_t z) { return (x & y) | (~x & z); }
inline uint32_t rf3(uint32_t x, uint32_t y, uint32_t z) { return (x | ~y) ^ z; }
inline uint32_t rf4(uint32_t x, uint32_t y, uint32_t z) { return (x & z) | (y & ~z); }
inline uint32_t rf5(uint32_t x, uint32_t y, uint32_t z) { return x ^ (y | ~z); }

const int RL[80] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
                    7, 4, 13, 1, 10, 6, 15, 3, 12, 0, 9, 5, 2, 14, 11, 8,
                    3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12,
                    1, 9, 11, 10, 0, 8, 12, 4, 13, 3, 7, 15, 14, 5, 6, 2,
                    4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13};
const int RR[80] = {5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12,
                    6, 11, 3, 7, 0, 13, 5, 10, 14, 15, 8, 12, 4, 9, 1, 2,
                    15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13,
                    8, 6, 4, 1, 3, 11, 15, 0, 5, 12, 2, 13, 9, 7, 10, 14,
                    12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11};
const int SL[80] = {11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8,
                    7, 6, 8, 13, 11, 9, 7, 15, 7, 12, 15, 9, 11, 7, 13, 12,
                    11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5,
                    11, 12, 14, 15, 14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12,
                    9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8, 5, 6};
const int SR[80] = {8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6,
                    9, 13, 15, 7, 12, 8, 9, 11, 7, 7, 12, 7, 6, 15, 13, 11,
                    9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5,
                    15, 5, 8, 11, 14, 14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8,
                    8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11, 11};
const uint32_t KL[5] = {0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E};
const uint32_t KR[5] = {0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000};

inline uint32_t rfunc(int j, uint32_t x, uint32_t y, uint32_t z) {
    switch (j / 16) {
    case 0: return rf1(x, y, z);
    case 1: return rf2(x, y, z);
    case 2: return rf3(x, y, z);
    case 3: return rf4(x, y, z);
    default: return rf5(x, y, z);
    }
}

void RipemdTransform(uint32_t* st, const unsigned char* chunk) {
    uint32_t X[16];
    for (int i = 0; i < 16; ++i) X[i] = ReadLE32(chunk + 4 * i);
    uint32_t al = st[0], bl = st[1], cl = st[2], dl = st[3], el = st[4];
    uint32_t ar = al, br = bl, cr = cl, dr = dl, er = el;
    for (int j = 0; j < 80; ++j) {
        uint32_t t = Rotl32(al + rfunc(j, bl, cl, dl) + X[RL[j]] + KL[j / 16], SL[j]) + el;
        al = el; el = dl; dl = Rotl32(cl, 10); cl = bl; bl = t;
        t = Rotl32(ar + rfunc(79 - j, br, cr, dr) + X[RR[j]] + KR[j / 16], SR[j]) + er;
        ar = er; er = dr; dr = Rotl32(cr, 10); cr = br; br = t;
    }
    uint32_t t = st[1] + cl + dr;
    st[1] = st[2] + dl + er;
    st[2] = st[3] + el + ar;
    st[3] = st[4] + al + br;
    st[4] = st[0] + bl + cr;
    st[0] = t;
}
} // namespace

CRIPEMD160::CRIPEMD160() { Reset(); }
CRIPEMD160& CRIPEMD160::Reset() {
    s[0] = 0x67452301; s[1] = 0xEFCDAB89; s[2] = 0x98BADCFE; s[3] = 0x10325476; s[4] = 0xC3D2E1F0;
    bytes = 0;
    return *this;
}
CRIPEMD160& CRIPEMD160::Write(const unsigned char* data, size_t len) {
    const unsigned char* end = data + len;
    size_t bufsize = bytes % 64;
    if (bufsize && bufsize + len >= 64) {
        memcpy(buf + bufsize, data, 64 - bufsize);
        bytes += 64 - bufsize; data += 64 - bufsize;
        RipemdTransform(s, buf);
        bufsize = 0;
    }
    while (end - data >= 64) { RipemdTransform(s, data); data += 64; bytes += 64; }
    if (end > data) { memcpy(buf + bufsize, data, end - data); bytes += end - data; }
    return *this;
}
void CRIPEMD160::Finalize(unsigned char hash[OUTPUT_SIZE]) {
    static const unsigned char pad[64] = {0x80};
    unsigned char sizedesc[8];
    WriteLE64(sizedesc, bytes << 3);
    Write(pad, 1 + ((119 - (bytes % 64)) % 64));
    Write(sizedesc, 8);
    for (int i = 0; i < 5; ++i) WriteLE32(hash + 4 * i, s[i]);
}

void Hash160(const unsigned char* data, size_t len, unsigned char out[20]) {
    unsigned char t[32];
    CSHA256().Write(data, len).Finalize(t);
    CRIPEMD160().Write(t, 32).Finalize(out);
}

// ---------------------------------------------------------------- HMAC
CHMAC_SHA256::CHMAC_SHA256(const unsigned char* key, size_t keylen) {
    unsigned char rkey[64];
    if (keylen <= 64) {
        memcpy(rkey, key, keylen);
        memset(rkey + keylen, 0, 64 - keylen);
    } else {
        CSHA256().Write(key, keylen).Finalize(rkey);
        memset(rkey + 32, 0, 32);
    }
    for (int n = 0; n < 64; n++) rkey[n] ^= 0x5c;
    outer.Write(rkey, 64);
    for (int n = 0; n < 64; n++) rkey[n] ^= 0x5c ^ 0x36;
    inner.Write(rkey, 64);
}
void CHMAC_SHA256::Finalize(unsigned char hash[OUTPUT_SIZE]) {
    unsigned char temp[32];
    inner.Finalize(temp);
    outer.Write(temp, 32).Finalize(hash);
}

CHMAC_SHA512::CHMAC_SHA512(const unsigned char* key, size_t keylen) {
    unsigned char rkey[128];
    if (keylen <= 128) {
        memcpy(rkey, key, keylen);
        memset(rkey + keylen, 0, 128 - keylen);
    } else {
        CSHA512().Write(key, keylen).Finalize(rkey);
        memset(rkey + 64, 0, 64);
    }
    for (int n = 0; n < 128; n++) rkey[n] ^= 0x5c;
    outer.Write(rkey, 128);
    for (int n = 0; n < 128; n++) rkey[n] ^= 0x5c ^ 0x36;
    inner.Write(rkey, 128);
}
void CHMAC_SHA512::Finalize(unsigned char hash[OUTPUT_SIZE]) {
    unsigned char temp[64];
    inner.Finalize(temp);
    outer.Write(temp, 64).Finalize(hash);
}

} // namespace bcp
