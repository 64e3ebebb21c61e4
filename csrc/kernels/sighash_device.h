// Device FORKID signature hash (K7): the SIGHASH_FORKID digest of reference
// src/script/interpreter.cpp:1354-1404, computed from host-built recipes (gpu_api.h
// SighashTx / SighashJob). One lane per check. The preimage is never materialised: each
// 64-byte SHA-256 block is gathered straight from the recipe regions
//   [0,4) version  [4,36) hashPrevouts  [36,68) hashSequence  [68,104) outpoint
//   [104,104+cs) compactsize(L)  [.., +L) script code  then amount(8) nSequence(4)
//   hashOutputs(32) nLockTime(4) nHashType(4)
// and the digest is written as raw bytes, which is the ECDSA message the verify kernels read.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels/gpu_api.h"
#include "kernels/sha256_device.h"

namespace bcpk {

struct SighashView {
    const uint8_t* tx;   // SighashTx bytes
    const uint8_t* job;  // SighashJob bytes
    const uint8_t* code; // script code
    uint32_t flags, L, cs, tailAt, len;
};

__device__ __forceinline__ uint32_t sighash_byte(const SighashView& v, uint32_t p) {
    if (p < 4) return v.tx[p];
    if (p < 36) return (v.flags & bcp::gpu::SIGHASH_JOB_ZERO_PREVOUTS) ? 0u : v.tx[p];      // tx +4
    if (p < 68) return (v.flags & bcp::gpu::SIGHASH_JOB_ZERO_SEQUENCE) ? 0u : v.tx[p];      // tx +36
    if (p < 104) return v.job[20 + (p - 68)];                                               // outpoint
    if (p < 104 + v.cs) {
        const uint32_t q = p - 104;
        if (v.cs == 1) return v.L;
        if (q == 0) return v.cs == 3 ? 0xfdu : 0xfeu;
        return (v.L >> (8 * (q - 1))) & 0xffu;
    }
    if (p < v.tailAt) return v.code[p - 104 - v.cs];
    const uint32_t q = p - v.tailAt;
    if (q < 8) return v.job[56 + q];                                                        // amount
    if (q < 12) return v.job[64 + (q - 8)];                                                 // nSequence
    if (q < 44) return (v.flags & bcp::gpu::SIGHASH_JOB_ZERO_OUTPUTS) ? 0u : v.tx[68 + (q - 12)];
    if (q < 48) return v.tx[100 + (q - 44)];                                                // nLockTime
    if (q < 52) return v.job[16 + (q - 48)];                                                // nHashType LE
    return 0u;
}

// digests[i] (32 bytes) = the recipe's SHA256d, unless the job is PRECOMPUTED (left as is).
static __global__ __launch_bounds__(256) void sighash_forkid_kernel(const uint8_t* __restrict__ txs,
                                                                    const uint8_t* __restrict__ jobs,
                                                                    const uint8_t* __restrict__ code,
                                                                    uint8_t* __restrict__ digests, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* job = jobs + (size_t)i * sizeof(bcp::gpu::SighashJob);
    const uint32_t* jw = reinterpret_cast<const uint32_t*>(job);
    SighashView v;
    v.flags = jw[1];
    if (v.flags & bcp::gpu::SIGHASH_JOB_PRECOMPUTED) return;
    v.tx = txs + (size_t)jw[0] * sizeof(bcp::gpu::SighashTx);
    v.job = job;
    v.code = code + jw[2];
    v.L = jw[3];
    v.cs = v.L < 253 ? 1u : (v.L <= 0xffffu ? 3u : 5u);
    v.tailAt = 104 + v.cs + v.L;
    v.len = v.tailAt + 52;
    uint32_t s[8];
    sha256_init(s);
    const uint32_t nblocks = (v.len + 9 + 63) / 64;
    for (uint32_t blk = 0; blk < nblocks; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            uint32_t x = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t p = blk * 64 + q * 4 + t;
                const uint32_t b = p < v.len ? sighash_byte(v, p) : (p == v.len ? 0x80u : 0u);
                x = (x << 8) | b;
            }
            w[q] = x;
        }
        if (blk == nblocks - 1) {
            const uint64_t bits = (uint64_t)v.len * 8;
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha256_transform(s, w);
    }
    uint32_t d[8];
    sha256_32(s, d);
    uint4* o = reinterpret_cast<uint4*>(digests + (size_t)i * 32);
    o[0] = make_uint4(bswap32d(d[0]), bswap32d(d[1]), bswap32d(d[2]), bswap32d(d[3]));
    o[1] = make_uint4(bswap32d(d[4]), bswap32d(d[5]), bswap32d(d[6]), bswap32d(d[7]));
}

} // namespace bcpk
