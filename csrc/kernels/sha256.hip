// SHA-256d batch kernels for CDNA4: the GPU side of the reference's hashing hot
// paths —
//   txids            CTransaction::ComputeHash      (src/primitives/transaction.cpp:75)
//   merkle levels    MerkleComputation              (src/consensus/merkle.cpp:47-144)
//   legacy PoW sweep generateBlocks nonce loop      (src/rpc/mining.cpp:154-160),
//                    CheckProofOfWork               (src/pow.cpp:141)
// One lane per message / pair / nonce; all inputs staged with 16-byte loads.
#include <hip/hip_runtime.h>

#include "crypto/common.h"
#include "crypto/hashes.h"

#include <algorithm>
#include "kernels/gpu_api.h"
#include "kernels/hip_util.h"
#include "kernels/sha256_device.h"

#include <cstring>
#include <mutex>
#include <stdexcept>

namespace bcpk {

__device__ __forceinline__ void store_digest_bytes(uint8_t* out, const uint32_t s[8]) {
    uint4* o = reinterpret_cast<uint4*>(out);
    o[0] = make_uint4(bswap32d(s[0]), bswap32d(s[1]), bswap32d(s[2]), bswap32d(s[3]));
    o[1] = make_uint4(bswap32d(s[4]), bswap32d(s[5]), bswap32d(s[6]), bswap32d(s[7]));
}

// SHA256d of 64-byte inputs (merkle pairs, or any 64-byte preimage).
__global__ __launch_bounds__(256) void sha256d_64(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* src = reinterpret_cast<const uint4*>(in + 64 * i);
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = src[q];
        w[4 * q + 0] = bswap32d(v.x);
        w[4 * q + 1] = bswap32d(v.y);
        w[4 * q + 2] = bswap32d(v.z);
        w[4 * q + 3] = bswap32d(v.w);
    }
    uint32_t s[8];
    sha256_init(s);
    sha256_transform(s, w);
    uint32_t pad[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 512};
    sha256_transform(s, pad);
    uint32_t d[8];
    sha256_32(s, d);
    store_digest_bytes(out + 32 * i, d);
}

// One merkle level: out[i] = SHA256d(in[2i] || in[min(2i+1, n-1)]).
// Mutation (CVE-2012-2459) is flagged only for pairs of complete subtrees,
// matching the reference's constant-space MerkleComputation: the last pair is
// skipped when its right child descends from an odd-level duplication.
__global__ __launch_bounds__(256) void merkle_level(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                    uint32_t n, int last_impure, uint32_t* __restrict__ mutated) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t m = (n + 1) / 2;
    if (i >= m) return;
    const uint32_t a = 2 * i, b = (2 * i + 1 < n) ? 2 * i + 1 : 2 * i;
    const uint4* pa = reinterpret_cast<const uint4*>(in + 32 * (size_t)a);
    const uint4* pb = reinterpret_cast<const uint4*>(in + 32 * (size_t)b);
    const uint4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
    if (b != a && !(b == n - 1 && last_impure)) {
        const bool eq = a0.x == b0.x && a0.y == b0.y && a0.z == b0.z && a0.w == b0.w && a1.x == b1.x && a1.y == b1.y &&
                        a1.z == b1.z && a1.w == b1.w;
        if (eq) atomicOr(mutated, 1u);
    }
    uint32_t w[16] = {bswap32d(a0.x), bswap32d(a0.y), bswap32d(a0.z), bswap32d(a0.w),
                      bswap32d(a1.x), bswap32d(a1.y), bswap32d(a1.z), bswap32d(a1.w),
                      bswap32d(b0.x), bswap32d(b0.y), bswap32d(b0.z), bswap32d(b0.w),
                      bswap32d(b1.x), bswap32d(b1.y), bswap32d(b1.z), bswap32d(b1.w)};
    uint32_t s[8];
    sha256_init(s);
    sha256_transform(s, w);
    uint32_t pad[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 512};
    sha256_transform(s, pad);
    uint32_t d[8];
    sha256_32(s, d);
    store_digest_bytes(out + 32 * (size_t)i, d);
}

// The last levels of a merkle tree (n <= MERKLE_TAIL leaves) in one workgroup: the level lives
// in LDS, one barrier per level, the root and the mutation flag leave once. Same pair rule as
// merkle_level.
constexpr int MERKLE_TAIL = 1024;
__global__ __launch_bounds__(MERKLE_TAIL / 2) void merkle_tail(const uint8_t* __restrict__ in, uint32_t n,
                                                                 int last_impure, uint32_t* __restrict__ mutated,
                                                                 uint8_t* __restrict__ root) {
    __shared__ uint4 lv[2][MERKLE_TAIL][2];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < n; i += blockDim.x) {
        const uint4* p = reinterpret_cast<const uint4*>(in + 32 * (size_t)i);
        lv[0][i][0] = p[0];
        lv[0][i][1] = p[1];
    }
    __syncthreads();
    int cur = 0, impure = last_impure;
    bool mut = false;
    while (n > 1) {
        const uint32_t m = (n + 1) / 2;
        for (uint32_t i = t; i < m; i += blockDim.x) {
            const uint32_t a = 2 * i, b = (2 * i + 1 < n) ? 2 * i + 1 : 2 * i;
            const uint4 a0 = lv[cur][a][0], a1 = lv[cur][a][1], b0 = lv[cur][b][0], b1 = lv[cur][b][1];
            if (b != a && !(b == n - 1 && impure))
                mut |= a0.x == b0.x && a0.y == b0.y && a0.z == b0.z && a0.w == b0.w && a1.x == b1.x &&
                       a1.y == b1.y && a1.z == b1.z && a1.w == b1.w;
            uint32_t w[16] = {bswap32d(a0.x), bswap32d(a0.y), bswap32d(a0.z), bswap32d(a0.w),
                              bswap32d(a1.x), bswap32d(a1.y), bswap32d(a1.z), bswap32d(a1.w),
                              bswap32d(b0.x), bswap32d(b0.y), bswap32d(b0.z), bswap32d(b0.w),
                              bswap32d(b1.x), bswap32d(b1.y), bswap32d(b1.z), bswap32d(b1.w)};
            uint32_t st[8];
            sha256_init(st);
            sha256_transform(st, w);
            uint32_t pad[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 512};
            sha256_transform(st, pad);
            uint32_t d[8];
            sha256_32(st, d);
            lv[cur ^ 1][i][0] = make_uint4(bswap32d(d[0]), bswap32d(d[1]), bswap32d(d[2]), bswap32d(d[3]));
            lv[cur ^ 1][i][1] = make_uint4(bswap32d(d[4]), bswap32d(d[5]), bswap32d(d[6]), bswap32d(d[7]));
        }
        __syncthreads();
        impure = (n & 1) || impure;
        n = m;
        cur ^= 1;
    }
    if (mut) atomicOr(mutated, 1u);
    if (t == 0) {
        uint4* o = reinterpret_cast<uint4*>(root);
        o[0] = lv[cur][0][0];
        o[1] = lv[cur][0][1];
    }
}

// Variable-length SHA256d (txids). Lane per message; byte-gathered input.
__global__ __launch_bounds__(256) void sha256d_var(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ lens, uint8_t* __restrict__ out,
                                                   size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = data + offs[i];
    const uint32_t len = lens[i];
    uint32_t s[8];
    sha256_init(s);
    const uint32_t nblocks = (len + 9 + 63) / 64;
    for (uint32_t blk = 0; blk < nblocks; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            uint32_t v = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t pos = blk * 64 + q * 4 + t;
                uint32_t byte;
                if (pos < len) byte = p[pos];
                else if (pos == len) byte = 0x80;
                else byte = 0;
                v = (v << 8) | byte;
            }
            w[q] = v;
        }
        if (blk == nblocks - 1) {
            const uint64_t bits = (uint64_t)len * 8;
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha256_transform(s, w);
    }
    uint32_t d[8];
    sha256_32(s, d);
    store_digest_bytes(out + 32 * i, d);
}

// Legacy 80-byte header nonce sweep from a host-computed midstate.
__global__ __launch_bounds__(256) void sha256d_scan(const uint32_t* __restrict__ mid, uint32_t t0, uint32_t t1,
                                                    uint32_t t2, const uint32_t* __restrict__ target, uint32_t start,
                                                    uint64_t count, uint64_t* __restrict__ found) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t ms[8], tg[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        ms[q] = mid[q];
        tg[q] = target[q];
    }
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += stride) {
        const uint32_t nonce = start + (uint32_t)k;
        uint32_t w[16] = {t0, t1, t2, bswap32d(nonce), 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 640};
        uint32_t s[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] = ms[q];
        sha256_transform(s, w);
        uint32_t d[8];
        sha256_32(s, d);
        // uint256 limbs (little-endian) are byte-swapped digest words; compare from the top limb.
        int cmp = 0;
#pragma unroll
        for (int q = 7; q >= 0; --q) {
            const uint32_t hv = bswap32d(d[q]);
            if (cmp == 0) cmp = (hv < tg[q]) ? -1 : (hv > tg[q] ? 1 : 0);
        }
        if (cmp <= 0) atomicMin((unsigned long long*)found, (unsigned long long)k);
    }
}

} // namespace bcpk

namespace bcp {
namespace gpu {

namespace {
unsigned grid_for(size_t n, unsigned bs = 256) { return (unsigned)((n + bs - 1) / bs); }

template <typename T> void grow(DevBuf<T>& b, size_t n) {
    if (b.n < n) b.alloc(std::max(n, 2 * b.n));
}
template <typename T> void grow(HostBuf<T>& b, size_t n) {
    if (b.n < n) b.alloc(std::max(n, 2 * b.n));
}

// Per-device state of the SHA-256d entry points: one stream, device buffers and pinned staging
// buffers kept across calls (a per-call hipMalloc/stream/pageable copy cost ~5 ms, more than the
// whole merkle root of an 8 MB block). Calls on one device are serialised by its mutex.
struct ShaCtx {
    std::mutex m;
    int device = -1;
    hipStream_t s = nullptr;
    DevBuf<uint8_t> a, b, misc;
    DevBuf<uint64_t> offs;
    DevBuf<uint32_t> lens;
    HostBuf<uint8_t> hin, hout;
};
ShaCtx& Ctx(int device) {
    static ShaCtx ctx[64];
    if (device < 0 || device >= 64) throw std::runtime_error("sha256 GPU context: device index out of range");
    return ctx[device];
}
// Locks and (first use) initialises the context of `device` (already current).
std::unique_lock<std::mutex> Lock(ShaCtx& c, int device) {
    std::unique_lock<std::mutex> l(c.m);
    if (!c.s) {
        BCP_HIP_CHECK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
        c.device = device;
        c.misc.alloc(64);
    }
    return l;
}
} // namespace

std::vector<unsigned char> Sha256d64Batch(const std::vector<unsigned char>& data, int device) {
    if (data.size() % 64) throw std::invalid_argument("Sha256d64Batch: input not a multiple of 64 bytes");
    device = UseDevice(device);
    const size_t n = data.size() / 64;
    std::vector<unsigned char> out(n * 32);
    if (!n) return out;
    ShaCtx& c = Ctx(device);
    auto l = Lock(c, device);
    grow(c.a, data.size());
    grow(c.b, out.size());
    grow(c.hin, data.size());
    grow(c.hout, out.size());
    memcpy(c.hin.p, data.data(), data.size());
    BCP_HIP_CHECK(hipMemcpyAsync(c.a.p, c.hin.p, data.size(), hipMemcpyHostToDevice, c.s));
    hipLaunchKernelGGL(bcpk::sha256d_64, dim3(grid_for(n)), dim3(256), 0, c.s, c.a.p, c.b.p, n);
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipMemcpyAsync(c.hout.p, c.b.p, out.size(), hipMemcpyDeviceToHost, c.s));
    BCP_HIP_CHECK(hipStreamSynchronize(c.s));
    memcpy(out.data(), c.hout.p, out.size());
    return out;
}

void Sha256d64Device(const void* in64, void* out32, size_t n, int device, uintptr_t stream) {
    if (!n) return;
    DeviceScope ds(device);
    hipLaunchKernelGGL(bcpk::sha256d_64, dim3(grid_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       static_cast<const uint8_t*>(in64), static_cast<uint8_t*>(out32), n);
    BCP_HIP_CHECK(hipGetLastError());
}

std::vector<unsigned char> Sha256dBatch(const std::vector<unsigned char>& data, const std::vector<uint64_t>& offs,
                                        const std::vector<uint32_t>& lens, int device) {
    if (offs.size() != lens.size()) throw std::invalid_argument("Sha256dBatch: offs/lens mismatch");
    for (size_t i = 0; i < offs.size(); ++i)
        if (offs[i] + lens[i] > data.size()) throw std::invalid_argument("Sha256dBatch: message out of range");
    device = UseDevice(device);
    const size_t n = offs.size();
    std::vector<unsigned char> out(n * 32);
    if (!n) return out;
    ShaCtx& c = Ctx(device);
    auto l = Lock(c, device);
    const size_t bytes = data.size() + n * 12;
    grow(c.a, std::max<size_t>(data.size(), 1));
    grow(c.b, out.size());
    grow(c.offs, n);
    grow(c.lens, n);
    grow(c.hin, bytes);
    grow(c.hout, out.size());
    memcpy(c.hin.p, data.data(), data.size());
    memcpy(c.hin.p + data.size(), offs.data(), n * 8);
    memcpy(c.hin.p + data.size() + n * 8, lens.data(), n * 4);
    if (!data.empty()) BCP_HIP_CHECK(hipMemcpyAsync(c.a.p, c.hin.p, data.size(), hipMemcpyHostToDevice, c.s));
    BCP_HIP_CHECK(hipMemcpyAsync(c.offs.p, c.hin.p + data.size(), n * 8, hipMemcpyHostToDevice, c.s));
    BCP_HIP_CHECK(hipMemcpyAsync(c.lens.p, c.hin.p + data.size() + n * 8, n * 4, hipMemcpyHostToDevice, c.s));
    hipLaunchKernelGGL(bcpk::sha256d_var, dim3(grid_for(n)), dim3(256), 0, c.s, c.a.p, c.offs.p, c.lens.p, c.b.p, n);
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipMemcpyAsync(c.hout.p, c.b.p, out.size(), hipMemcpyDeviceToHost, c.s));
    BCP_HIP_CHECK(hipStreamSynchronize(c.s));
    memcpy(out.data(), c.hout.p, out.size());
    return out;
}

std::vector<unsigned char> MerkleRoot(const std::vector<unsigned char>& leaves, bool* mutated, int device) {
    if (leaves.size() % 32) throw std::invalid_argument("MerkleRoot: leaves must be 32-byte hashes");
    size_t n = leaves.size() / 32;
    if (mutated) *mutated = false;
    if (n == 0) return std::vector<unsigned char>(32, 0);
    if (n == 1) return leaves;
    if (n > 0xffffffffu) throw std::invalid_argument("MerkleRoot: too many leaves");
    device = UseDevice(device);
    ShaCtx& c = Ctx(device);
    auto l = Lock(c, device);
    grow(c.a, n * 32);
    grow(c.b, (n + 1) / 2 * 32);
    grow(c.hin, n * 32);
    grow(c.hout, 64);
    memcpy(c.hin.p, leaves.data(), leaves.size());
    BCP_HIP_CHECK(hipMemcpyAsync(c.a.p, c.hin.p, leaves.size(), hipMemcpyHostToDevice, c.s));
    uint32_t* dmut = reinterpret_cast<uint32_t*>(c.misc.p + 32);
    BCP_HIP_CHECK(hipMemsetAsync(dmut, 0, 4, c.s));
    uint8_t* cur = c.a.p;
    uint8_t* nxt = c.b.p;
    int impure = 0;
    // wide levels: one launch each, lane per pair; the last <= MERKLE_TAIL leaves in one workgroup
    while (n > (size_t)bcpk::MERKLE_TAIL) {
        const uint32_t m = (uint32_t)((n + 1) / 2);
        hipLaunchKernelGGL(bcpk::merkle_level, dim3(grid_for(m)), dim3(256), 0, c.s, cur, nxt, (uint32_t)n, impure,
                           dmut);
        BCP_HIP_CHECK(hipGetLastError());
        impure = (n & 1) || impure;
        n = m;
        std::swap(cur, nxt);
    }
    hipLaunchKernelGGL(bcpk::merkle_tail, dim3(1), dim3(bcpk::MERKLE_TAIL / 2), 0, c.s, cur, (uint32_t)n, impure, dmut,
                       c.misc.p);
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipMemcpyAsync(c.hout.p, c.misc.p, 36, hipMemcpyDeviceToHost, c.s));
    BCP_HIP_CHECK(hipStreamSynchronize(c.s));
    std::vector<unsigned char> root(c.hout.p, c.hout.p + 32);
    uint32_t mut = 0;
    memcpy(&mut, c.hout.p + 32, 4);
    if (mutated) *mutated = mut != 0;
    return root;
}

int64_t Sha256dScanNonces(const unsigned char header80[80], const unsigned char target_le[32], uint32_t start,
                          uint64_t count, int device) {
    device = UseDevice(device);
    if (count == 0) return -1;
    if (count > (1ULL << 32)) count = 1ULL << 32;
    CSHA256 h;
    h.Write(header80, 64);
    uint32_t t0 = ReadBE32(header80 + 64), t1 = ReadBE32(header80 + 68), t2 = ReadBE32(header80 + 72);
    ShaCtx& c = Ctx(device);
    auto l = Lock(c, device);
    grow(c.hin, 72);
    grow(c.hout, 8);
    uint32_t* mid = reinterpret_cast<uint32_t*>(c.hin.p);
    memcpy(mid, h.State(), 32);
    for (int q = 0; q < 8; ++q) memcpy(&mid[8 + q], target_le + 4 * q, 4);
    const uint64_t init = ~0ULL;
    memcpy(c.hin.p + 64, &init, 8);
    uint32_t* dmid = reinterpret_cast<uint32_t*>(c.misc.p);   // midstate (32 B) + target (32 B)
    grow(c.b, 8);
    uint64_t* dfound = reinterpret_cast<uint64_t*>(c.b.p);
    BCP_HIP_CHECK(hipMemcpyAsync(dmid, c.hin.p, 64, hipMemcpyHostToDevice, c.s));
    BCP_HIP_CHECK(hipMemcpyAsync(dfound, c.hin.p + 64, 8, hipMemcpyHostToDevice, c.s));
    const unsigned grid = (unsigned)std::min<uint64_t>(grid_for(count), 256 * 64);
    hipLaunchKernelGGL(bcpk::sha256d_scan, dim3(grid), dim3(256), 0, c.s, dmid, t0, t1, t2, dmid + 8, start, count,
                       dfound);
    BCP_HIP_CHECK(hipGetLastError());
    BCP_HIP_CHECK(hipMemcpyAsync(c.hout.p, dfound, 8, hipMemcpyDeviceToHost, c.s));
    BCP_HIP_CHECK(hipStreamSynchronize(c.s));
    uint64_t found;
    memcpy(&found, c.hout.p, 8);
    if (found == ~0ULL) return -1;
    return (int64_t)(uint32_t)(start + (uint32_t)found);
}

} // namespace gpu
} // namespace bcp
