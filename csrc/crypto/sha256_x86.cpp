// SHA-256 compression on the x86 SHA extensions (SHA-NI: sha256rnds2 / sha256msg1 / sha256msg2),
// selected at run time by CSHA256::Transform when the host CPU has them (EPYC hosts of MI355X
// nodes do). The hashing the block-connect path does on the CPU - txids, BIP143-style sighash
// preimages, script-cache keys, HASH160 of public keys, merkle trees - is a few hundred thousand
// compressions per 8 MB block; the scalar transform made it one of the largest CPU costs.
// Parity: reference src/crypto/sha256.cpp (the portable transform) - same function, other engine.
//
// Register layout the instructions use: one vector holds (A,B,E,F) with F in lane 0, the other
// (C,D,G,H) with H in lane 0. sha256rnds2 runs two rounds with the W+K words of lanes 0 and 1.
#include <cpuid.h>
#include <immintrin.h>

#include <cstddef>
#include <cstdint>

namespace bcp {
namespace sha256_x86 {

namespace {
alignas(16) const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
} // namespace

bool Available() {
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
    const bool ssse3 = c & (1u << 9), sse41 = c & (1u << 19);
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    const bool sha = b & (1u << 29);
    return ssse3 && sse41 && sha;
}

__attribute__((target("sha,sse4.1"))) void Transform(uint32_t* s, const unsigned char* chunk, size_t blocks) {
    // big-endian words: reverse the bytes of each 32-bit lane
    const __m128i bswap = _mm_set_epi8(12, 13, 14, 15, 8, 9, 10, 11, 4, 5, 6, 7, 0, 1, 2, 3);
    __m128i abef = _mm_set_epi32((int)s[0], (int)s[1], (int)s[4], (int)s[5]);
    __m128i cdgh = _mm_set_epi32((int)s[2], (int)s[3], (int)s[6], (int)s[7]);
    while (blocks--) {
        const __m128i abef0 = abef, cdgh0 = cdgh;
        __m128i m[4];
        for (int i = 0; i < 4; i++)
            m[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(chunk + 16 * i)), bswap);
#pragma GCC unroll 16
        for (int g = 0; g < 16; g++) {
            // four rounds on W[4g..4g+3]
            __m128i wk = _mm_add_epi32(m[g & 3], _mm_load_si128((const __m128i*)&K[4 * g]));
            cdgh = _mm_sha256rnds2_epu32(cdgh, abef, wk);
            wk = _mm_shuffle_epi32(wk, 0x0E);
            abef = _mm_sha256rnds2_epu32(abef, cdgh, wk); // each call's old (A,B,E,F) is the new (C,D,G,H)
            // schedule W[4g+16..4g+19] from W[4g..4g+15] into the slot just consumed
            if (g < 12) {
                __m128i w = _mm_sha256msg1_epu32(m[g & 3], m[(g + 1) & 3]);
                w = _mm_add_epi32(w, _mm_alignr_epi8(m[(g + 3) & 3], m[(g + 2) & 3], 4));
                m[g & 3] = _mm_sha256msg2_epu32(w, m[(g + 3) & 3]);
            }
        }
        abef = _mm_add_epi32(abef, abef0);
        cdgh = _mm_add_epi32(cdgh, cdgh0);
        chunk += 64;
    }
    s[0] = (uint32_t)_mm_extract_epi32(abef, 3);
    s[1] = (uint32_t)_mm_extract_epi32(abef, 2);
    s[4] = (uint32_t)_mm_extract_epi32(abef, 1);
    s[5] = (uint32_t)_mm_extract_epi32(abef, 0);
    s[2] = (uint32_t)_mm_extract_epi32(cdgh, 3);
    s[3] = (uint32_t)_mm_extract_epi32(cdgh, 2);
    s[6] = (uint32_t)_mm_extract_epi32(cdgh, 1);
    s[7] = (uint32_t)_mm_extract_epi32(cdgh, 0);
}

} // namespace sha256_x86
} // namespace bcp
