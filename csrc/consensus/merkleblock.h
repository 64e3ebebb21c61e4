// Partial merkle trees / merkle blocks (SPV proofs) and BIP37 bloom filters.
// Parity: reference src/merkleblock.{h,cpp} (CPartialMerkleTree traversal with
// depth-first flag bits, CVE-2012-2459 guard, CMerkleBlock from a bloom filter or a
// txid set) and src/bloom.{h,cpp} (CBloomFilter with MurmurHash3 and BLOOM_UPDATE_*
// flags, CRollingBloomFilter).
#pragma once
#include "primitives/block.h"

#include <set>
#include <vector>

namespace bcp {

uint32_t MurmurHash3(uint32_t nHashSeed, const unsigned char* data, size_t len);

enum bloomflags { BLOOM_UPDATE_NONE = 0, BLOOM_UPDATE_ALL = 1, BLOOM_UPDATE_P2PUBKEY_ONLY = 2, BLOOM_UPDATE_MASK = 3 };

class CBloomFilter {
public:
    static constexpr unsigned int MAX_BLOOM_FILTER_SIZE = 36000; // bytes
    static constexpr unsigned int MAX_HASH_FUNCS = 50;
    CBloomFilter() : isFull(true), isEmpty(false), nHashFuncs(0), nTweak(0), nFlags(0) {}
    CBloomFilter(unsigned nElements, double nFPRate, unsigned nTweak, unsigned char nFlags);
    void insert(const std::vector<unsigned char>& vKey);
    void insert(const COutPoint& outpoint);
    void insert(const uint256& hash);
    bool contains(const std::vector<unsigned char>& vKey) const;
    bool contains(const COutPoint& outpoint) const;
    bool contains(const uint256& hash) const;
    void clear();
    void reset(unsigned nNewTweak);
    bool IsWithinSizeConstraints() const;
    bool IsRelevantAndUpdate(const CTransaction& tx);
    void UpdateEmptyFull();
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, vData);
        ::bcp::Serialize(s, nHashFuncs);
        ::bcp::Serialize(s, nTweak);
        ::bcp::Serialize(s, nFlags);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, vData);
        ::bcp::Unserialize(s, nHashFuncs);
        ::bcp::Unserialize(s, nTweak);
        ::bcp::Unserialize(s, nFlags);
        isFull = false;
        isEmpty = false;
    }

private:
    unsigned Hash(unsigned nHashNum, const std::vector<unsigned char>& vDataToHash) const;
    std::vector<unsigned char> vData;
    bool isFull, isEmpty;
    unsigned nHashFuncs, nTweak;
    unsigned char nFlags;
};

// Probabilistic "recently seen" set with bounded memory (three generations).
class CRollingBloomFilter {
public:
    CRollingBloomFilter(unsigned nElements, double nFPRate);
    void insert(const std::vector<unsigned char>& vKey);
    void insert(const uint256& hash);
    bool contains(const std::vector<unsigned char>& vKey) const;
    bool contains(const uint256& hash) const;
    void reset();

private:
    int nEntriesPerGeneration, nEntriesThisGeneration, nGeneration;
    std::vector<uint64_t> data;
    unsigned nTweak;
    int nHashFuncs;
};

class CPartialMerkleTree {
public:
    CPartialMerkleTree(const std::vector<uint256>& vTxid, const std::vector<bool>& vMatch);
    CPartialMerkleTree();
    // returns the root, or 0 on failure; fills the matched txids/indices
    uint256 ExtractMatches(std::vector<uint256>& vMatch, std::vector<unsigned>& vnIndex);
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, nTransactions);
        ::bcp::Serialize(s, vHash);
        std::vector<unsigned char> vBytes((vBits.size() + 7) / 8);
        for (unsigned p = 0; p < vBits.size(); p++) vBytes[p / 8] |= vBits[p] << (p % 8);
        ::bcp::Serialize(s, vBytes);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, nTransactions);
        ::bcp::Unserialize(s, vHash);
        std::vector<unsigned char> vBytes;
        ::bcp::Unserialize(s, vBytes);
        vBits.resize(vBytes.size() * 8);
        for (unsigned p = 0; p < vBits.size(); p++) vBits[p] = (vBytes[p / 8] & (1 << (p % 8))) != 0;
        fBad = false;
    }
    unsigned GetNumTransactions() const { return nTransactions; }

protected:
    unsigned CalcTreeWidth(int height) const { return (nTransactions + (1 << height) - 1) >> height; }
    uint256 CalcHash(int height, unsigned pos, const std::vector<uint256>& vTxid);
    void TraverseAndBuild(int height, unsigned pos, const std::vector<uint256>& vTxid, const std::vector<bool>& vMatch);
    uint256 TraverseAndExtract(int height, unsigned pos, unsigned& nBitsUsed, unsigned& nHashUsed,
                               std::vector<uint256>& vMatch, std::vector<unsigned>& vnIndex);
    unsigned nTransactions = 0;
    std::vector<bool> vBits;
    std::vector<uint256> vHash;
    bool fBad = false;
};

class CMerkleBlock {
public:
    CBlockHeader header;
    CPartialMerkleTree txn;
    std::vector<std::pair<unsigned, uint256>> vMatchedTxn;
    CMerkleBlock() {}
    CMerkleBlock(const CBlock& block, CBloomFilter& filter);
    CMerkleBlock(const CBlock& block, const std::set<uint256>& txids);
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, header);
        ::bcp::Serialize(s, txn);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, header);
        ::bcp::Unserialize(s, txn);
    }
};

// A gettxoutproof proof (a serialized CMerkleBlock). The header inside is the legacy 80-byte form
// below the fork height and the new form above it, and nothing in the bytes says which: both are
// tried and the one that consumes the proof exactly wins (verifytxoutproof, importprunedfunds).
bool DecodeTxOutProof(const std::vector<unsigned char>& data, CMerkleBlock& mb);

} // namespace bcp
