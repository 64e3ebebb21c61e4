// BLAKE2b (RFC 7693), SipHash-2-4, ChaCha20, AES-256-CBC.
// BLAKE2b replaces the libsodium dependency of reference src/crypto/equihash.h:13,24
// (crypto_generichash_blake2b_init_salt_personal / _update / _final).
#include "crypto/hashes.h"
#include "crypto/common.h"

#include <cstring>
#include <stdexcept>

namespace bcp {

// ---------------------------------------------------------------- BLAKE2b
namespace {
const uint64_t B2B_IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                            0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                            0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
const uint8_t B2B_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
} // namespace

void CBlake2b::Compress(uint64_t h[8], const unsigned char block[128], uint64_t t0, uint64_t t1, bool last) {
    uint64_t m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = ReadLE64(block + 8 * i);
    for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = B2B_IV[i]; }
    v[12] ^= t0;
    v[13] ^= t1;
    if (last) v[14] = ~v[14];
#define B2G(a, b, c, d, x, y)             \
    v[a] = v[a] + v[b] + x;               \
    v[d] = Rotr64(v[d] ^ v[a], 32);       \
    v[c] = v[c] + v[d];                   \
    v[b] = Rotr64(v[b] ^ v[c], 24);       \
    v[a] = v[a] + v[b] + y;               \
    v[d] = Rotr64(v[d] ^ v[a], 16);       \
    v[c] = v[c] + v[d];                   \
    v[b] = Rotr64(v[b] ^ v[c], 63);
    for (int r = 0; r < 12; ++r) {
        const uint8_t* s = B2B_SIGMA[r];
        B2G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        B2G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        B2G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        B2G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        B2G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        B2G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        B2G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        B2G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef B2G
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

CBlake2b::CBlake2b(size_t outlen, const unsigned char* key, size_t keylen,
                   const unsigned char* salt16, const unsigned char* personal16) {
    if (outlen == 0 || outlen > 64 || keylen > 64) throw std::invalid_argument("blake2b params");
    memset(&st, 0, sizeof(st));
    unsigned char param[64] = {0};
    param[0] = (unsigned char)outlen;
    param[1] = (unsigned char)keylen;
    param[2] = 1; // fanout
    param[3] = 1; // depth
    if (salt16) memcpy(param + 32, salt16, 16);
    if (personal16) memcpy(param + 48, personal16, 16);
    for (int i = 0; i < 8; ++i) st.h[i] = B2B_IV[i] ^ ReadLE64(param + 8 * i);
    st.outlen = (uint32_t)outlen;
    if (keylen) {
        unsigned char block[128] = {0};
        memcpy(block, key, keylen);
        Write(block, 128);
        memory_cleanse(block, sizeof(block));
    }
}

CBlake2b& CBlake2b::Write(const unsigned char* in, size_t inlen) {
    while (inlen > 0) {
        // Keep the final block buffered: compress only when more input follows.
        if (st.buflen == 128) {
            st.t[0] += 128;
            if (st.t[0] < 128) st.t[1]++;
            Compress(st.h, st.buf, st.t[0], st.t[1], false);
            st.buflen = 0;
        }
        size_t take = 128 - st.buflen;
        if (take > inlen) take = inlen;
        memcpy(st.buf + st.buflen, in, take);
        st.buflen += (uint32_t)take;
        in += take;
        inlen -= take;
    }
    return *this;
}

void CBlake2b::Finalize(unsigned char* out) {
    uint64_t h[8];
    memcpy(h, st.h, sizeof(h));
    uint64_t t0 = st.t[0] + st.buflen, t1 = st.t[1] + (t0 < st.t[0] ? 1 : 0);
    unsigned char block[128] = {0};
    memcpy(block, st.buf, st.buflen);
    Compress(h, block, t0, t1, true);
    unsigned char full[64];
    for (int i = 0; i < 8; ++i) WriteLE64(full + 8 * i, h[i]);
    memcpy(out, full, st.outlen);
}

// ---------------------------------------------------------------- SipHash
#define SIPROUND                                                      \
    do {                                                              \
        v0 += v1; v1 = Rotl64(v1, 13); v1 ^= v0; v0 = Rotl64(v0, 32); \
        v2 += v3; v3 = Rotl64(v3, 16); v3 ^= v2;                      \
        v0 += v3; v3 = Rotl64(v3, 21); v3 ^= v0;                      \
        v2 += v1; v1 = Rotl64(v1, 17); v1 ^= v2; v2 = Rotl64(v2, 32); \
    } while (0)

CSipHasher::CSipHasher(uint64_t k0, uint64_t k1) {
    v[0] = 0x736f6d6570736575ULL ^ k0;
    v[1] = 0x646f72616e646f6dULL ^ k1;
    v[2] = 0x6c7967656e657261ULL ^ k0;
    v[3] = 0x7465646279746573ULL ^ k1;
    count = 0;
    tmp = 0;
}

CSipHasher& CSipHasher::Write(uint64_t data) {
    uint64_t v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3];
    // Only valid when count is a multiple of 8 (as in the reference).
    v3 ^= data;
    SIPROUND; SIPROUND;
    v0 ^= data;
    v[0] = v0; v[1] = v1; v[2] = v2; v[3] = v3;
    count += 8;
    return *this;
}

CSipHasher& CSipHasher::Write(const unsigned char* data, size_t size) {
    uint64_t v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3];
    uint64_t t = tmp;
    int c = count;
    while (size--) {
        t |= ((uint64_t)(*(data++))) << (8 * (c % 8));
        c++;
        if ((c & 7) == 0) {
            v3 ^= t;
            SIPROUND; SIPROUND;
            v0 ^= t;
            t = 0;
        }
    }
    v[0] = v0; v[1] = v1; v[2] = v2; v[3] = v3;
    count = c;
    tmp = t;
    return *this;
}

uint64_t CSipHasher::Finalize() const {
    uint64_t v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3];
    uint64_t t = tmp | (((uint64_t)count) << 56);
    v3 ^= t;
    SIPROUND; SIPROUND;
    v0 ^= t;
    v2 ^= 0xFF;
    SIPROUND; SIPROUND; SIPROUND; SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

uint64_t SipHashUint256(uint64_t k0, uint64_t k1, const unsigned char val[32]) {
    CSipHasher h(k0, k1);
    for (int i = 0; i < 4; ++i) h.Write(ReadLE64(val + 8 * i));
    return h.Finalize();
}

uint64_t SipHashUint256Extra(uint64_t k0, uint64_t k1, const unsigned char val[32], uint32_t extra) {
    uint64_t v0 = 0x736f6d6570736575ULL ^ k0;
    uint64_t v1 = 0x646f72616e646f6dULL ^ k1;
    uint64_t v2 = 0x6c7967656e657261ULL ^ k0;
    uint64_t v3 = 0x7465646279746573ULL ^ k1;
    for (int i = 0; i < 4; ++i) {
        uint64_t d = ReadLE64(val + 8 * i);
        v3 ^= d; SIPROUND; SIPROUND; v0 ^= d;
    }
    uint64_t d = (((uint64_t)36) << 56) | extra;
    v3 ^= d; SIPROUND; SIPROUND; v0 ^= d;
    v2 ^= 0xFF;
    SIPROUND; SIPROUND; SIPROUND; SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}
#undef SIPROUND

// ---------------------------------------------------------------- ChaCha20
#define QR(a, b, c, d)                       \
    a += b; d = Rotl32(d ^ a, 16);           \
    c += d; b = Rotl32(b ^ c, 12);           \
    a += b; d = Rotl32(d ^ a, 8);            \
    c += d; b = Rotl32(b ^ c, 7);

ChaCha20::ChaCha20() { memset(input, 0, sizeof(input)); }
ChaCha20::ChaCha20(const unsigned char* k, size_t keylen) { SetKey(k, keylen); }

void ChaCha20::SetKey(const unsigned char* k, size_t keylen) {
    static const char sigma[] = "expand 32-byte k";
    static const char tau[] = "expand 16-byte k";
    const char* constants;
    input[4] = ReadLE32(k + 0); input[5] = ReadLE32(k + 4);
    input[6] = ReadLE32(k + 8); input[7] = ReadLE32(k + 12);
    if (keylen == 32) { k += 16; constants = sigma; } else { constants = tau; }
    input[8] = ReadLE32(k + 0); input[9] = ReadLE32(k + 4);
    input[10] = ReadLE32(k + 8); input[11] = ReadLE32(k + 12);
    input[0] = ReadLE32((const unsigned char*)constants + 0);
    input[1] = ReadLE32((const unsigned char*)constants + 4);
    input[2] = ReadLE32((const unsigned char*)constants + 8);
    input[3] = ReadLE32((const unsigned char*)constants + 12);
    input[12] = input[13] = input[14] = input[15] = 0;
}
void ChaCha20::SetIV(uint64_t iv) { input[14] = (uint32_t)iv; input[15] = (uint32_t)(iv >> 32); }
void ChaCha20::Seek(uint64_t pos) { input[12] = (uint32_t)pos; input[13] = (uint32_t)(pos >> 32); }

void ChaCha20::Output(unsigned char* c, size_t bytes) {
    while (bytes) {
        uint32_t x[16];
        memcpy(x, input, sizeof(x));
        for (int i = 0; i < 10; ++i) {
            QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
            QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
            QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
            QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
        }
        unsigned char blk[64];
        for (int i = 0; i < 16; ++i) WriteLE32(blk + 4 * i, x[i] + input[i]);
        if (++input[12] == 0) ++input[13];
        size_t n = bytes < 64 ? bytes : 64;
        memcpy(c, blk, n);
        c += n;
        bytes -= n;
    }
}
#undef QR

// ---------------------------------------------------------------- AES-256
namespace {
uint8_t SBOX[256], INV_SBOX[256];
bool aes_tables_ready = false;

inline uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) { if (b & 1) p ^= a; a = xtime(a); b >>= 1; }
    return p;
}
void aes_init_tables() {
    if (aes_tables_ready) return;
    // Build the S-box from the multiplicative inverse in GF(2^8) and the affine map.
    uint8_t p = 1, q = 1;
    do {
        p = p ^ (uint8_t)(p << 1) ^ (uint8_t)((p & 0x80) ? 0x1B : 0);
        q ^= q << 1; q ^= q << 2; q ^= q << 4;
        if (q & 0x80) q ^= 0x09;
        uint8_t x = q ^ (uint8_t)((q << 1) | (q >> 7)) ^ (uint8_t)((q << 2) | (q >> 6)) ^
                    (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4));
        SBOX[p] = x ^ 0x63;
    } while (p != 1);
    SBOX[0] = 0x63;
    for (int i = 0; i < 256; ++i) INV_SBOX[SBOX[i]] = (uint8_t)i;
    aes_tables_ready = true;
}

void key_expand(const unsigned char key[32], uint32_t rk[60]) {
    aes_init_tables();
    for (int i = 0; i < 8; ++i) rk[i] = ReadBE32(key + 4 * i);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint32_t t = rk[i - 1];
        if (i % 8 == 0) {
            t = (t << 8) | (t >> 24);
            t = ((uint32_t)SBOX[t >> 24] << 24) | ((uint32_t)SBOX[(t >> 16) & 0xff] << 16) |
                ((uint32_t)SBOX[(t >> 8) & 0xff] << 8) | SBOX[t & 0xff];
            t ^= (uint32_t)rcon << 24;
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            t = ((uint32_t)SBOX[t >> 24] << 24) | ((uint32_t)SBOX[(t >> 16) & 0xff] << 16) |
                ((uint32_t)SBOX[(t >> 8) & 0xff] << 8) | SBOX[t & 0xff];
        }
        rk[i] = rk[i - 8] ^ t;
    }
}

void add_round_key(uint8_t s[16], const uint32_t* rk) {
    for (int c = 0; c < 4; ++c) {
        s[4 * c + 0] ^= (uint8_t)(rk[c] >> 24);
        s[4 * c + 1] ^= (uint8_t)(rk[c] >> 16);
        s[4 * c + 2] ^= (uint8_t)(rk[c] >> 8);
        s[4 * c + 3] ^= (uint8_t)rk[c];
    }
}

void aes_encrypt_block(const uint32_t rk[60], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    memcpy(s, in, 16);
    add_round_key(s, rk);
    for (int round = 1; round <= 14; ++round) {
        for (int i = 0; i < 16; ++i) s[i] = SBOX[s[i]];
        uint8_t t[16];
        for (int c = 0; c < 4; ++c)
            for (int r = 0; r < 4; ++r) t[4 * c + r] = s[4 * ((c + r) % 4) + r];
        memcpy(s, t, 16);
        if (round != 14) {
            for (int c = 0; c < 4; ++c) {
                uint8_t* col = s + 4 * c;
                uint8_t a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3];
                col[0] = gmul(a0, 2) ^ gmul(a1, 3) ^ a2 ^ a3;
                col[1] = a0 ^ gmul(a1, 2) ^ gmul(a2, 3) ^ a3;
                col[2] = a0 ^ a1 ^ gmul(a2, 2) ^ gmul(a3, 3);
                col[3] = gmul(a0, 3) ^ a1 ^ a2 ^ gmul(a3, 2);
            }
        }
        add_round_key(s, rk + 4 * round);
    }
    memcpy(out, s, 16);
}

void aes_decrypt_block(const uint32_t rk[60], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    memcpy(s, in, 16);
    add_round_key(s, rk + 56);
    for (int round = 13; round >= 0; --round) {
        uint8_t t[16];
        for (int c = 0; c < 4; ++c)
            for (int r = 0; r < 4; ++r) t[4 * ((c + r) % 4) + r] = s[4 * c + r];
        for (int i = 0; i < 16; ++i) s[i] = INV_SBOX[t[i]];
        add_round_key(s, rk + 4 * round);
        if (round != 0) {
            for (int c = 0; c < 4; ++c) {
                uint8_t* col = s + 4 * c;
                uint8_t a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3];
                col[0] = gmul(a0, 14) ^ gmul(a1, 11) ^ gmul(a2, 13) ^ gmul(a3, 9);
                col[1] = gmul(a0, 9) ^ gmul(a1, 14) ^ gmul(a2, 11) ^ gmul(a3, 13);
                col[2] = gmul(a0, 13) ^ gmul(a1, 9) ^ gmul(a2, 14) ^ gmul(a3, 11);
                col[3] = gmul(a0, 11) ^ gmul(a1, 13) ^ gmul(a2, 9) ^ gmul(a3, 14);
            }
        }
    }
    memcpy(out, s, 16);
}
} // namespace

AES256CBCEncrypt::AES256CBCEncrypt(const unsigned char key[32], const unsigned char ivIn[16], bool padIn)
    : pad(padIn) {
    key_expand(key, rk);
    memcpy(iv, ivIn, 16);
}
AES256CBCEncrypt::~AES256CBCEncrypt() { memory_cleanse(rk, sizeof(rk)); memory_cleanse(iv, sizeof(iv)); }

int AES256CBCEncrypt::Encrypt(const unsigned char* data, int size, unsigned char* out) const {
    if (!data || !size || !out) return 0;
    int padsize = pad ? 16 - (size % 16) : 0;
    if (!pad && size % 16) return 0;
    int written = 0;
    uint8_t mixed[16], prev[16];
    memcpy(prev, iv, 16);
    int total = size + padsize;
    for (int off = 0; off < total; off += 16) {
        for (int i = 0; i < 16; ++i) {
            int idx = off + i;
            uint8_t b = idx < size ? data[idx] : (uint8_t)padsize;
            mixed[i] = b ^ prev[i];
        }
        aes_encrypt_block(rk, mixed, out + off);
        memcpy(prev, out + off, 16);
        written += 16;
    }
    return written;
}

AES256CBCDecrypt::AES256CBCDecrypt(const unsigned char key[32], const unsigned char ivIn[16], bool padIn)
    : pad(padIn) {
    key_expand(key, rk);
    memcpy(iv, ivIn, 16);
}
AES256CBCDecrypt::~AES256CBCDecrypt() { memory_cleanse(rk, sizeof(rk)); memory_cleanse(iv, sizeof(iv)); }

int AES256CBCDecrypt::Decrypt(const unsigned char* data, int size, unsigned char* out) const {
    if (!data || !size || !out || size % 16) return 0;
    uint8_t prev[16];
    memcpy(prev, iv, 16);
    for (int off = 0; off < size; off += 16) {
        uint8_t blk[16];
        aes_decrypt_block(rk, data + off, blk);
        for (int i = 0; i < 16; ++i) out[off + i] = blk[i] ^ prev[i];
        memcpy(prev, data + off, 16);
    }
    if (!pad) return size;
    uint8_t padsize = out[size - 1];
    if (padsize == 0 || padsize > 16) return 0;
    bool fail = false;
    for (int i = size - padsize; i < size; ++i) fail |= out[i] != padsize;
    return fail ? 0 : size - padsize;
}

} // namespace bcp
