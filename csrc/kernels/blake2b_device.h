// Device BLAKE2b for Equihash on CDNA4.
//
// One work-item runs one full 12-round compression on 64-bit lanes. The 64-bit
// rotations by 32/24/16/63 lower to v_alignbit_b32 pairs / register swaps, the
// adds to v_add_co/v_addc pairs; the base state (chaining value after the
// 128-byte header block plus the g-independent message words) is
// wave-uniform, so it sits in SGPRs and only the message word that carries
// le32(g) is per-lane.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace bcpk {

// Host-prepared, g-independent part of H(I||V||le32(g)): chaining value after all
// full blocks, the final (partial) block with the g slot zeroed, byte counter.
struct EhBaseState {
    uint64_t h[8];
    uint64_t m[16];
    uint64_t t0;        // total bytes hashed including the 4-byte g
    uint32_t g_byte;    // byte offset of le32(g) within the final block
    uint32_t outlen;    // digest bytes (HashOutput)
};

__device__ __constant__ static const uint8_t kB2Sigma[12][16] = {
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

// 64-bit rotate right as two 32-bit funnel shifts (v_alignbit_b32): the generic shift/or form
// compiles to two 64-bit shifts plus two ORs. n is a compile-time constant at every call site
// (32 is a plain half swap).
// a ^ b ^ c in one gfx950 three-input bit operation per 32-bit half (v_bitop3_b32, truth table
// 0x96) instead of two xors: the digest words of every hash (h ^ v[i] ^ v[i + 8]).
__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    uint32_t rlo, rhi;
    if (n == 32) {
        rlo = hi;
        rhi = lo;
    } else if (n < 32) {
        rlo = __builtin_amdgcn_alignbit(hi, lo, n);
        rhi = __builtin_amdgcn_alignbit(lo, hi, n);
    } else {
        rlo = __builtin_amdgcn_alignbit(lo, hi, n - 32);
        rhi = __builtin_amdgcn_alignbit(hi, lo, n - 32);
    }
    return ((uint64_t)rhi << 32) | rlo;
}

// 64-bit add. BCP_B2_ADDC=1 spells it as a full-rate v_add_co/v_addc pair instead of the
// single 64-bit v_lshl_add_u64 the compiler picks for gfx950 (A/B builds).
#ifndef BCP_B2_ADDC
#define BCP_B2_ADDC 0
#endif
__device__ __forceinline__ uint64_t add64(uint64_t a, uint64_t b) {
#if BCP_B2_ADDC
    uint32_t lo, hi;
    asm("v_add_co_u32_e32 %0, vcc, %2, %3\n\tv_addc_co_u32_e32 %1, vcc, %4, %5, vcc"
        : "=&v"(lo), "=v"(hi)
        : "v"((uint32_t)a), "v"((uint32_t)b), "v"((uint32_t)(a >> 32)), "v"((uint32_t)(b >> 32))
        : "vcc");
    return ((uint64_t)hi << 32) | lo;
#else
    return a + b;
#endif
}
// a + m, where m is a compile-time zero for most message words of the header specialisation
#define BCPK_ADDM(a, x) ((__builtin_constant_p(x) && (x) == 0) ? (a) : add64((a), (x)))

#define BCPK_B2G(a, b, c, d, x, y)       \
    a = BCPK_ADDM(add64(a, b), (x));     \
    d = rotr64(d ^ a, 32);               \
    c = add64(c, d);                     \
    b = rotr64(b ^ c, 24);               \
    a = BCPK_ADDM(add64(a, b), (y));     \
    d = rotr64(d ^ a, 16);               \
    c = add64(c, d);                     \
    b = rotr64(b ^ c, 63);

// Final-block compression with message m; writes the new chaining value to out.
__device__ __forceinline__ void blake2b_compress_final(const uint64_t hin[8], const uint64_t m[16], uint64_t t0,
                                                       uint64_t out[8]) {
    const uint64_t IV0 = 0x6a09e667f3bcc908ULL, IV1 = 0xbb67ae8584caa73bULL, IV2 = 0x3c6ef372fe94f82bULL,
                   IV3 = 0xa54ff53a5f1d36f1ULL, IV4 = 0x510e527fade682d1ULL, IV5 = 0x9b05688c2b3e6c1fULL,
                   IV6 = 0x1f83d9abfb41bd6bULL, IV7 = 0x5be0cd19137e2179ULL;
    uint64_t v0 = hin[0], v1 = hin[1], v2 = hin[2], v3 = hin[3], v4 = hin[4], v5 = hin[5], v6 = hin[6],
             v7 = hin[7];
    uint64_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3, v12 = IV4 ^ t0, v13 = IV5, v14 = ~IV6, v15 = IV7;
#pragma unroll
    for (int r = 0; r < 12; ++r) {
        BCPK_B2G(v0, v4, v8, v12, m[kB2Sigma[r][0]], m[kB2Sigma[r][1]]);
        BCPK_B2G(v1, v5, v9, v13, m[kB2Sigma[r][2]], m[kB2Sigma[r][3]]);
        BCPK_B2G(v2, v6, v10, v14, m[kB2Sigma[r][4]], m[kB2Sigma[r][5]]);
        BCPK_B2G(v3, v7, v11, v15, m[kB2Sigma[r][6]], m[kB2Sigma[r][7]]);
        BCPK_B2G(v0, v5, v10, v15, m[kB2Sigma[r][8]], m[kB2Sigma[r][9]]);
        BCPK_B2G(v1, v6, v11, v12, m[kB2Sigma[r][10]], m[kB2Sigma[r][11]]);
        BCPK_B2G(v2, v7, v8, v13, m[kB2Sigma[r][12]], m[kB2Sigma[r][13]]);
        BCPK_B2G(v3, v4, v9, v14, m[kB2Sigma[r][14]], m[kB2Sigma[r][15]]);
    }
    out[0] = xor3_64(hin[0], v0, v8);
    out[1] = xor3_64(hin[1], v1, v9);
    out[2] = xor3_64(hin[2], v2, v10);
    out[3] = xor3_64(hin[3], v3, v11);
    out[4] = xor3_64(hin[4], v4, v12);
    out[5] = xor3_64(hin[5], v5, v13);
    out[6] = xor3_64(hin[6], v6, v14);
    out[7] = xor3_64(hin[7], v7, v15);
}

// One compression of a full, non-final 128-byte block (t0 = bytes hashed so far, this block
// included): the chaining value h is updated in place.
__device__ __forceinline__ void blake2b_compress_block(uint64_t h[8], const uint64_t m[16], uint64_t t0) {
    const uint64_t IV0 = 0x6a09e667f3bcc908ULL, IV1 = 0xbb67ae8584caa73bULL, IV2 = 0x3c6ef372fe94f82bULL,
                   IV3 = 0xa54ff53a5f1d36f1ULL, IV4 = 0x510e527fade682d1ULL, IV5 = 0x9b05688c2b3e6c1fULL,
                   IV6 = 0x1f83d9abfb41bd6bULL, IV7 = 0x5be0cd19137e2179ULL;
    uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
    uint64_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3, v12 = IV4 ^ t0, v13 = IV5, v14 = IV6, v15 = IV7;
    for (int r = 0; r < 12; ++r) { // not unrolled: one compression per header, code size matters more
        BCPK_B2G(v0, v4, v8, v12, m[kB2Sigma[r][0]], m[kB2Sigma[r][1]]);
        BCPK_B2G(v1, v5, v9, v13, m[kB2Sigma[r][2]], m[kB2Sigma[r][3]]);
        BCPK_B2G(v2, v6, v10, v14, m[kB2Sigma[r][4]], m[kB2Sigma[r][5]]);
        BCPK_B2G(v3, v7, v11, v15, m[kB2Sigma[r][6]], m[kB2Sigma[r][7]]);
        BCPK_B2G(v0, v5, v10, v15, m[kB2Sigma[r][8]], m[kB2Sigma[r][9]]);
        BCPK_B2G(v1, v6, v11, v12, m[kB2Sigma[r][10]], m[kB2Sigma[r][11]]);
        BCPK_B2G(v2, v7, v8, v13, m[kB2Sigma[r][12]], m[kB2Sigma[r][13]]);
        BCPK_B2G(v3, v4, v9, v14, m[kB2Sigma[r][14]], m[kB2Sigma[r][15]]);
    }
    h[0] = xor3_64(h[0], v0, v8);
    h[1] = xor3_64(h[1], v1, v9);
    h[2] = xor3_64(h[2], v2, v10);
    h[3] = xor3_64(h[3], v3, v11);
    h[4] = xor3_64(h[4], v4, v12);
    h[5] = xor3_64(h[5], v5, v13);
    h[6] = xor3_64(h[6], v6, v14);
    h[7] = xor3_64(h[7], v7, v15);
}

// The base state of a block header's Equihash input, built on the device from the raw 140 bytes
// (CEquihashInput 108 B || nNonce 32 B): BLAKE2b with digest length (512/N)*N/8 and personal
// "ZcashPoW" || le32(N) || le32(K) (reference src/crypto/equihash.cpp:26-36 InitialiseState),
// the first 128 bytes compressed, the last 12 left in the final block ahead of le32(g).
// The same state the host builds with MakeEhBaseState(EquihashStateFor(header)).
__device__ __forceinline__ void eh_header_state(const uint8_t* in140, uint32_t N, uint32_t K, EhBaseState& bs) {
    const uint32_t outlen = (512 / N) * N / 8;
    uint64_t h[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                     0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    h[0] ^= (uint64_t)outlen | (1ULL << 16) | (1ULL << 24); // digest length, key 0, fanout 1, depth 1
    h[6] ^= 0x576f50687361635aULL;                           // "ZcashPoW" (little-endian)
    h[7] ^= (uint64_t)N | ((uint64_t)K << 32);
    uint64_t m[16];
    for (int i = 0; i < 16; ++i) {
        uint64_t w = 0;
        for (int b = 7; b >= 0; --b) w = (w << 8) | in140[8 * i + b];
        m[i] = w;
    }
    blake2b_compress_block(h, m, 128);
    for (int i = 0; i < 8; ++i) bs.h[i] = h[i];
    uint64_t w0 = 0, w1 = 0;
    for (int b = 7; b >= 0; --b) w0 = (w0 << 8) | in140[128 + b];
    for (int b = 3; b >= 0; --b) w1 = (w1 << 8) | in140[136 + b];
    bs.m[0] = w0;
    bs.m[1] = w1;
    for (int i = 2; i < 16; ++i) bs.m[i] = 0;
    bs.t0 = 144;
    bs.g_byte = 12;
    bs.outlen = outlen;
}

// H(base || le32(g)) -> 8 chaining words (digest = first outlen bytes, little-endian).
__device__ __forceinline__ void eh_hash_g(const EhBaseState& bs, uint32_t g, uint64_t out[8]) {
    uint64_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = bs.m[i];
    // Insert le32(g) at byte g_byte (may straddle two 64-bit words).
    const uint32_t w = bs.g_byte >> 3, sh = (bs.g_byte & 7) * 8;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i == (int)w) m[i] |= (uint64_t)g << sh;
        if (sh > 32 && i == (int)w + 1) m[i] |= (uint64_t)g >> (64 - sh);
    }
    blake2b_compress_final(bs.h, m, bs.t0, out);
}

// Specialisation for the block-header input (CEquihashInput 108 B || nonce 32 B): the final
// block holds 12 bytes of nonce then le32(g), so m[0] is wave-uniform, m[1] = uniform |
// g << 32 and m[2..15] are zero — the 168 zero-word additions fold away at compile time.
__device__ __forceinline__ void eh_hash_g_hdr(const EhBaseState& bs, uint32_t g, uint64_t out[8]) {
    uint64_t m[16];
    m[0] = bs.m[0];
    m[1] = bs.m[1] | ((uint64_t)g << 32);
#pragma unroll
    for (int i = 2; i < 16; ++i) m[i] = 0;
    blake2b_compress_final(bs.h, m, bs.t0, out);
}

// The header specialisation split at its first g-dependent operation. In round 0 only G0's
// second half reads m[1] (which carries g << 32); G1..G3 and G0's first half depend on the
// base state alone. eh_hdr_round0_uniform computes that g-independent prefix once (per
// workgroup) - the 16 state words with v0 already holding a + b + (m[1] without g) - and
// eh_hash_g_hdr_from finishes each hash from it: the add of g << 32 only touches the high word.
__device__ __forceinline__ void eh_hdr_round0_uniform(const EhBaseState& bs, uint64_t P[16]) {
    const uint64_t IV0 = 0x6a09e667f3bcc908ULL, IV1 = 0xbb67ae8584caa73bULL, IV2 = 0x3c6ef372fe94f82bULL,
                   IV3 = 0xa54ff53a5f1d36f1ULL, IV4 = 0x510e527fade682d1ULL, IV5 = 0x9b05688c2b3e6c1fULL,
                   IV6 = 0x1f83d9abfb41bd6bULL, IV7 = 0x5be0cd19137e2179ULL;
    uint64_t v0 = bs.h[0], v1 = bs.h[1], v2 = bs.h[2], v3 = bs.h[3], v4 = bs.h[4], v5 = bs.h[5], v6 = bs.h[6],
             v7 = bs.h[7];
    uint64_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3, v12 = IV4 ^ bs.t0, v13 = IV5, v14 = ~IV6, v15 = IV7;
    // G0, first half (message word m[0])
    v0 = v0 + v4 + bs.m[0];
    v12 = rotr64(v12 ^ v0, 32);
    v8 = v8 + v12;
    v4 = rotr64(v4 ^ v8, 24);
    v0 = v0 + v4 + bs.m[1]; // the g-independent part of G0's second add
    // G1..G3 (message words 2..7 are zero)
    BCPK_B2G(v1, v5, v9, v13, 0, 0);
    BCPK_B2G(v2, v6, v10, v14, 0, 0);
    BCPK_B2G(v3, v7, v11, v15, 0, 0);
    P[0] = v0, P[1] = v1, P[2] = v2, P[3] = v3, P[4] = v4, P[5] = v5, P[6] = v6, P[7] = v7;
    P[8] = v8, P[9] = v9, P[10] = v10, P[11] = v11, P[12] = v12, P[13] = v13, P[14] = v14, P[15] = v15;
}

__device__ __forceinline__ void eh_hash_g_hdr_from(const uint64_t P[16], const EhBaseState& bs, uint32_t g,
                                                   uint64_t out[8]) {
    uint64_t v0 = P[0], v1 = P[1], v2 = P[2], v3 = P[3], v4 = P[4], v5 = P[5], v6 = P[6], v7 = P[7];
    uint64_t v8 = P[8], v9 = P[9], v10 = P[10], v11 = P[11], v12 = P[12], v13 = P[13], v14 = P[14], v15 = P[15];
    const uint64_t m0 = bs.m[0], m1 = bs.m[1] | ((uint64_t)g << 32);
    // G0, second half: a += g << 32 (high word only), then the rest of the G
    v0 = ((uint64_t)((uint32_t)(v0 >> 32) + g) << 32) | (uint32_t)v0;
    v12 = rotr64(v12 ^ v0, 16);
    v8 = add64(v8, v12);
    v4 = rotr64(v4 ^ v8, 63);
    // round 0, diagonal step (message words 8..15 are zero)
    BCPK_B2G(v0, v5, v10, v15, 0, 0);
    BCPK_B2G(v1, v6, v11, v12, 0, 0);
    BCPK_B2G(v2, v7, v8, v13, 0, 0);
    BCPK_B2G(v3, v4, v9, v14, 0, 0);
    uint64_t m[16];
    m[0] = m0;
    m[1] = m1;
#pragma unroll
    for (int i = 2; i < 16; ++i) m[i] = 0;
#pragma unroll
    for (int r = 1; r < 12; ++r) {
        BCPK_B2G(v0, v4, v8, v12, m[kB2Sigma[r][0]], m[kB2Sigma[r][1]]);
        BCPK_B2G(v1, v5, v9, v13, m[kB2Sigma[r][2]], m[kB2Sigma[r][3]]);
        BCPK_B2G(v2, v6, v10, v14, m[kB2Sigma[r][4]], m[kB2Sigma[r][5]]);
        BCPK_B2G(v3, v7, v11, v15, m[kB2Sigma[r][6]], m[kB2Sigma[r][7]]);
        BCPK_B2G(v0, v5, v10, v15, m[kB2Sigma[r][8]], m[kB2Sigma[r][9]]);
        BCPK_B2G(v1, v6, v11, v12, m[kB2Sigma[r][10]], m[kB2Sigma[r][11]]);
        BCPK_B2G(v2, v7, v8, v13, m[kB2Sigma[r][12]], m[kB2Sigma[r][13]]);
        BCPK_B2G(v3, v4, v9, v14, m[kB2Sigma[r][14]], m[kB2Sigma[r][15]]);
    }
    out[0] = xor3_64(bs.h[0], v0, v8);
    out[1] = xor3_64(bs.h[1], v1, v9);
    out[2] = xor3_64(bs.h[2], v2, v10);
    out[3] = xor3_64(bs.h[3], v3, v11);
    out[4] = xor3_64(bs.h[4], v4, v12);
    out[5] = xor3_64(bs.h[5], v5, v13);
    out[6] = xor3_64(bs.h[6], v6, v14);
    out[7] = xor3_64(bs.h[7], v7, v15);
}

// Byte k (0-based) of the digest held in 8 little-endian words.
__device__ __forceinline__ uint32_t digest_byte(const uint64_t h[8], int k) {
    return (uint32_t)(h[k >> 3] >> ((k & 7) * 8)) & 0xff;
}

} // namespace bcpk
