// Equihash proof-of-work: parameters, BLAKE2b base state, bit packing, the
// consensus verifier and a CPU reference solver.
//
// Behaviour parity with reference src/crypto/equihash.{h,cpp,tcc}:
//   InitialiseState      equihash.cpp:36   (personal "ZcashPoW"||le32 N||le32 K, outlen (512/N)*N/8)
//   GenerateHash         equihash.cpp:51   (H(state || le32(g)))
//   ExpandArray/CompressArray equihash.cpp:62-142 (big-endian bit groups)
//   GetIndicesFromMinimal / GetMinimalFromIndices equihash.cpp:176-207
//   IsValidSolution      equihash.cpp:725  (collision, ordering, distinctness, final zero)
//   BasicSolve           equihash.cpp:332  (any valid solution is acceptable to the verifier)
// Design differences: parameters are runtime values (one code path for
// (200,9)/(96,5)/(96,3)/(48,5)), and the solver stores parent references per
// round instead of ever-growing index lists (same design as the GPU kernel in
// csrc/kernels/equihash_solver.hip), expanding and canonicalising the index
// tree only for final candidates.
#pragma once
#include "crypto/hashes.h"

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace bcp {

struct EquihashParams {
    unsigned N = 200, K = 9;
    EquihashParams() {}
    EquihashParams(unsigned n, unsigned k) : N(n), K(k) {}
    unsigned IndicesPerHashOutput() const { return 512 / N; }
    unsigned HashOutput() const { return IndicesPerHashOutput() * N / 8; }
    unsigned CollisionBitLength() const { return N / (K + 1); }
    unsigned CollisionByteLength() const { return (CollisionBitLength() + 7) / 8; }
    unsigned HashLength() const { return (K + 1) * CollisionByteLength(); }
    unsigned SolutionWidth() const { return (1u << K) * (CollisionBitLength() + 1) / 8; }
    uint32_t InitSize() const { return 1u << (CollisionBitLength() + 1); }
    bool Valid() const;
    std::string ToString() const;
};

// The parameter sets the reference instantiates (equihash.h:197-200).
bool EquihashParamsSupported(unsigned n, unsigned k);

// Personalised BLAKE2b base state for (N,K); callers then absorb the 108-byte
// CEquihashInput and the 32-byte nonce.
CBlake2b EhInitialiseState(const EquihashParams& p);
void EhGenerateHash(const CBlake2b& base, uint32_t g, unsigned char* out /* HashOutput bytes */);

void ExpandArray(const unsigned char* in, size_t in_len, unsigned char* out, size_t out_len,
                 size_t bit_len, size_t byte_pad = 0);
void CompressArray(const unsigned char* in, size_t in_len, unsigned char* out, size_t out_len,
                   size_t bit_len, size_t byte_pad = 0);
std::vector<uint32_t> GetIndicesFromMinimal(const std::vector<unsigned char>& minimal, size_t cBitLen);
std::vector<unsigned char> GetMinimalFromIndices(const std::vector<uint32_t>& indices, size_t cBitLen);

// Consensus verifier; `reason` (optional) receives the first failure.
bool EhIsValidSolution(const EquihashParams& p, const CBlake2b& base, const std::vector<unsigned char>& soln,
                       std::string* reason = nullptr);

// Reorders the index list so every merge has its lexicographically-smaller
// subtree on the left, and reports whether all indices are distinct.
bool EhCanonicaliseIndices(std::vector<uint32_t>& idx, unsigned K);

struct EhSolveStats {
    uint64_t candidates = 0;
    uint64_t duplicates = 0;
    uint64_t solutions = 0;
};

// CPU reference solver. Calls validBlock(minimal) for each valid solution;
// stops early when it returns true. Returns true if validBlock accepted one.
bool EhBasicSolve(const EquihashParams& p, const CBlake2b& base,
                  const std::function<bool(const std::vector<unsigned char>&)>& validBlock,
                  const std::function<bool()>& cancelled = nullptr, EhSolveStats* stats = nullptr);

// All solutions for a state (convenience for tests/benchmarks).
std::vector<std::vector<unsigned char>> EhSolveAll(const EquihashParams& p, const CBlake2b& base,
                                                   EhSolveStats* stats = nullptr);

} // namespace bcp
