// Merkle roots and branches. Parity: reference src/consensus/merkle.{h,cpp}:47-175
// (Bitcoin odd-level duplication, CVE-2012-2459 mutation flag only for pairs of
// complete subtrees). Large blocks are hashed level-wise on the GPU
// (csrc/kernels/sha256.hip merkle_level) when one is available.
#pragma once
#include "primitives/block.h"
#include "primitives/uint256.h"

#include <vector>

namespace bcp {

uint256 ComputeMerkleRoot(const std::vector<uint256>& leaves, bool* mutated = nullptr);
std::vector<uint256> ComputeMerkleBranch(const std::vector<uint256>& leaves, uint32_t position);
uint256 ComputeMerkleRootFromBranch(const uint256& leaf, const std::vector<uint256>& branch, uint32_t nIndex);
uint256 BlockMerkleRoot(const CBlock& block, bool* mutated = nullptr);
std::vector<uint256> BlockMerkleBranch(const CBlock& block, uint32_t position);

// Leaves at or above this count go to the GPU kernel if a device is present.
void SetGpuMerkleThreshold(size_t nLeaves);

} // namespace bcp
