// Level-wise merkle computation with the reference's mutation semantics.
#include "consensus/merkle.h"
#include "kernels/gpu_api.h"

#include <atomic>
#include <cstring>

namespace bcp {

// Blocks with at least this many transactions hash their merkle tree on the GPU when one is
// visible. With SHA-256 on the SHA extensions the CPU matches the GPU at 21k leaves (0.21 vs
// 0.19 ms on MI355X) and is 5x slower at 1M (10.2 vs 1.9 ms), profiles/connect_r3.md: the GPU
// path is kept for blocks of 32k+ transactions (it was 2048 with the scalar CPU hash).
static std::atomic<size_t> g_gpu_merkle_threshold{32768};
void SetGpuMerkleThreshold(size_t n) { g_gpu_merkle_threshold = n; }

// One level: pairs (2i, 2i+1), odd tail duplicated. The tail pair is "impure" if its right
// child descends from an odd-level duplication: the reference's constant-space walk never
// compares such pairs, so neither do we.
static uint256 MerkleLevels(std::vector<uint256> level, bool* mutated) {
    bool mut = false, impure_last = false;
    while (level.size() > 1) {
        const size_t n = level.size();
        std::vector<uint256> next((n + 1) / 2);
        for (size_t i = 0; i < next.size(); ++i) {
            const uint256& a = level[2 * i];
            const bool has_b = 2 * i + 1 < n;
            const uint256& b = has_b ? level[2 * i + 1] : a;
            if (has_b && !(2 * i + 1 == n - 1 && impure_last) && a == b) mut = true;
            next[i] = Hash256Concat(a, b);
        }
        impure_last = (n & 1) || impure_last;
        level.swap(next);
    }
    if (mutated) *mutated = mut;
    return level.empty() ? uint256() : level[0];
}

uint256 ComputeMerkleRoot(const std::vector<uint256>& leaves, bool* mutated) {
    if (leaves.empty()) {
        if (mutated) *mutated = false;
        return uint256();
    }
    if (leaves.size() >= g_gpu_merkle_threshold && gpu::GpuAvailable()) {
        std::vector<unsigned char> flat(leaves.size() * 32);
        for (size_t i = 0; i < leaves.size(); ++i) memcpy(&flat[32 * i], leaves[i].begin(), 32);
        bool mut = false;
        try {
            std::vector<unsigned char> root = gpu::MerkleRoot(flat, &mut);
            if (mutated) *mutated = mut;
            return uint256(root);
        } catch (const std::exception&) {
            // a device error must not decide validity: recompute on the CPU
        }
    }
    return MerkleLevels(leaves, mutated);
}

std::vector<uint256> ComputeMerkleBranch(const std::vector<uint256>& leaves, uint32_t position) {
    std::vector<uint256> branch;
    std::vector<uint256> level = leaves;
    uint32_t pos = position;
    while (level.size() > 1) {
        const size_t n = level.size();
        const uint32_t sib = pos ^ 1;
        branch.push_back(sib < n ? level[sib] : level[pos]);
        std::vector<uint256> next((n + 1) / 2);
        for (size_t i = 0; i < next.size(); ++i) {
            const uint256& a = level[2 * i];
            const uint256& b = 2 * i + 1 < n ? level[2 * i + 1] : a;
            next[i] = Hash256Concat(a, b);
        }
        level.swap(next);
        pos >>= 1;
    }
    return branch;
}

uint256 ComputeMerkleRootFromBranch(const uint256& leaf, const std::vector<uint256>& branch, uint32_t nIndex) {
    uint256 hash = leaf;
    for (const uint256& b : branch) {
        hash = (nIndex & 1) ? Hash256Concat(b, hash) : Hash256Concat(hash, b);
        nIndex >>= 1;
    }
    return hash;
}

uint256 BlockMerkleRoot(const CBlock& block, bool* mutated) {
    std::vector<uint256> leaves(block.vtx.size());
    for (size_t s = 0; s < block.vtx.size(); s++) leaves[s] = block.vtx[s]->GetId();
    return ComputeMerkleRoot(leaves, mutated);
}

std::vector<uint256> BlockMerkleBranch(const CBlock& block, uint32_t position) {
    std::vector<uint256> leaves(block.vtx.size());
    for (size_t s = 0; s < block.vtx.size(); s++) leaves[s] = block.vtx[s]->GetId();
    return ComputeMerkleBranch(leaves, position);
}

} // namespace bcp
