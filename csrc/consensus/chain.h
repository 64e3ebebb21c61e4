// Block index tree and the active chain. Parity: reference src/chain.{h,cpp}
// (BlockStatus bits, CBlockIndex incl. BCP header fields, skip list GetAncestor/BuildSkip,
// median-time-past over 11 blocks, GetBlockProof, CChain locator/fork search,
// CDiskBlockIndex on-disk form).
#pragma once
#include "primitives/block.h"
#include "primitives/uint256.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace bcp {

namespace Consensus { struct Params; }

struct CDiskBlockPos {
    int nFile = -1;
    unsigned int nPos = 0;
    CDiskBlockPos() {}
    CDiskBlockPos(int f, unsigned int p) : nFile(f), nPos(p) {}
    bool IsNull() const { return nFile == -1; }
    void SetNull() { nFile = -1; nPos = 0; }
    friend bool operator==(const CDiskBlockPos& a, const CDiskBlockPos& b) { return a.nFile == b.nFile && a.nPos == b.nPos; }
    friend bool operator!=(const CDiskBlockPos& a, const CDiskBlockPos& b) { return !(a == b); }
    template <typename S> void Serialize(S& s) const { WriteVarInt(s, (uint64_t)(int64_t)nFile); WriteVarInt(s, nPos); }
    template <typename S> void Unserialize(S& s) { nFile = (int)(int64_t)ReadVarInt(s); nPos = (unsigned)ReadVarInt(s); }
};

enum BlockStatus : uint32_t {
    BLOCK_VALID_UNKNOWN = 0,
    BLOCK_VALID_HEADER = 1,
    BLOCK_VALID_TREE = 2,
    BLOCK_VALID_TRANSACTIONS = 3,
    BLOCK_VALID_CHAIN = 4,
    BLOCK_VALID_SCRIPTS = 5,
    BLOCK_VALID_MASK = BLOCK_VALID_HEADER | BLOCK_VALID_TREE | BLOCK_VALID_TRANSACTIONS | BLOCK_VALID_CHAIN |
                       BLOCK_VALID_SCRIPTS,
    BLOCK_HAVE_DATA = 8,
    BLOCK_HAVE_UNDO = 16,
    BLOCK_HAVE_MASK = BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO,
    BLOCK_FAILED_VALID = 32,
    BLOCK_FAILED_CHILD = 64,
    BLOCK_FAILED_MASK = BLOCK_FAILED_VALID | BLOCK_FAILED_CHILD,
};

class CBlockIndex {
public:
    const uint256* phashBlock = nullptr;
    CBlockIndex* pprev = nullptr;
    CBlockIndex* pskip = nullptr;
    int nHeight = 0;
    int nFile = 0;
    unsigned int nDataPos = 0;
    unsigned int nUndoPos = 0;
    arith_uint256 nChainWork;
    unsigned int nTx = 0;
    unsigned int nChainTx = 0;
    uint32_t nStatus = 0;
    // header
    int32_t nVersion = 0;
    uint256 hashMerkleRoot;
    uint32_t nReserved[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t nTime = 0;
    uint32_t nBits = 0;
    uint256 nNonce;
    std::vector<unsigned char> nSolution;
    int32_t nSequenceId = 0;
    unsigned int nTimeMax = 0;

    CBlockIndex() {}
    explicit CBlockIndex(const CBlockHeader& block)
        : nVersion(block.nVersion), hashMerkleRoot(block.hashMerkleRoot), nTime(block.nTime), nBits(block.nBits),
          nNonce(block.nNonce), nSolution(block.nSolution) {
        memcpy(nReserved, block.nReserved, sizeof(nReserved));
    }

    CDiskBlockPos GetBlockPos() const {
        CDiskBlockPos ret;
        if (nStatus & BLOCK_HAVE_DATA) { ret.nFile = nFile; ret.nPos = nDataPos; }
        return ret;
    }
    CDiskBlockPos GetUndoPos() const {
        CDiskBlockPos ret;
        if (nStatus & BLOCK_HAVE_UNDO) { ret.nFile = nFile; ret.nPos = nUndoPos; }
        return ret;
    }
    CBlockHeader GetBlockHeader() const;
    uint256 GetBlockHash() const { return *phashBlock; }
    int64_t GetBlockTime() const { return (int64_t)nTime; }
    int64_t GetBlockTimeMax() const { return (int64_t)nTimeMax; }
    enum { nMedianTimeSpan = 11 };
    int64_t GetMedianTimePast() const;
    std::string ToString() const;
    bool IsValid(BlockStatus nUpTo = BLOCK_VALID_TRANSACTIONS) const {
        if (nStatus & BLOCK_FAILED_MASK) return false;
        return (nStatus & BLOCK_VALID_MASK) >= (uint32_t)nUpTo;
    }
    bool RaiseValidity(BlockStatus nUpTo) {
        if (nStatus & BLOCK_FAILED_MASK) return false;
        if ((nStatus & BLOCK_VALID_MASK) < (uint32_t)nUpTo) {
            nStatus = (nStatus & ~BLOCK_VALID_MASK) | nUpTo;
            return true;
        }
        return false;
    }
    void BuildSkip();
    CBlockIndex* GetAncestor(int height);
    const CBlockIndex* GetAncestor(int height) const;
};

arith_uint256 GetBlockProof(const CBlockIndex& block);
int64_t GetBlockProofEquivalentTime(const CBlockIndex& to, const CBlockIndex& from, const CBlockIndex& tip,
                                    const Consensus::Params& params);
const CBlockIndex* LastCommonAncestor(const CBlockIndex* pa, const CBlockIndex* pb);

typedef std::unordered_map<uint256, CBlockIndex*, Uint256Hasher> BlockMap;

// On-disk form of a block index entry (reference src/chain.h:390-457).
class CDiskBlockIndex : public CBlockIndex {
public:
    uint256 hashPrev;
    CDiskBlockIndex() {}
    explicit CDiskBlockIndex(const CBlockIndex* pindex) : CBlockIndex(*pindex) {
        hashPrev = pprev ? pprev->GetBlockHash() : uint256();
    }
    template <typename S> void Serialize(S& s) const {
        int nVersionS = s.GetVersion();
        if (!(s.GetType() & SER_GETHASH)) WriteVarInt(s, (uint64_t)nVersionS);
        WriteVarInt(s, (uint64_t)nHeight);
        WriteVarInt(s, nStatus);
        WriteVarInt(s, nTx);
        if (nStatus & (BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)) WriteVarInt(s, (uint64_t)nFile);
        if (nStatus & BLOCK_HAVE_DATA) WriteVarInt(s, nDataPos);
        if (nStatus & BLOCK_HAVE_UNDO) WriteVarInt(s, nUndoPos);
        ::bcp::Serialize(s, nVersion);
        ::bcp::Serialize(s, hashPrev);
        ::bcp::Serialize(s, hashMerkleRoot);
        for (int i = 0; i < 7; ++i) ::bcp::Serialize(s, nReserved[i]);
        ::bcp::Serialize(s, nTime);
        ::bcp::Serialize(s, nBits);
        ::bcp::Serialize(s, nNonce);
        ::bcp::Serialize(s, nSolution);
    }
    template <typename S> void Unserialize(S& s) {
        if (!(s.GetType() & SER_GETHASH)) (void)ReadVarInt(s);
        nHeight = (int)ReadVarInt(s);
        nStatus = (uint32_t)ReadVarInt(s);
        nTx = (unsigned)ReadVarInt(s);
        if (nStatus & (BLOCK_HAVE_DATA | BLOCK_HAVE_UNDO)) nFile = (int)ReadVarInt(s);
        if (nStatus & BLOCK_HAVE_DATA) nDataPos = (unsigned)ReadVarInt(s);
        if (nStatus & BLOCK_HAVE_UNDO) nUndoPos = (unsigned)ReadVarInt(s);
        ::bcp::Unserialize(s, nVersion);
        ::bcp::Unserialize(s, hashPrev);
        ::bcp::Unserialize(s, hashMerkleRoot);
        for (int i = 0; i < 7; ++i) ::bcp::Unserialize(s, nReserved[i]);
        ::bcp::Unserialize(s, nTime);
        ::bcp::Unserialize(s, nBits);
        ::bcp::Unserialize(s, nNonce);
        ::bcp::Unserialize(s, nSolution);
    }
    CBlockHeader GetHeader() const;
    // hash of the stored header (reference CDiskBlockIndex::GetBlockHash, chain.h:441): a
    // freshly read entry has no phashBlock yet
    uint256 GetBlockHash() const { return GetHeader().GetHash(); }
};

class CChain {
    std::vector<CBlockIndex*> vChain;
public:
    CBlockIndex* Genesis() const { return vChain.size() > 0 ? vChain[0] : nullptr; }
    CBlockIndex* Tip() const { return vChain.size() > 0 ? vChain[vChain.size() - 1] : nullptr; }
    CBlockIndex* operator[](int nHeight) const {
        if (nHeight < 0 || nHeight >= (int)vChain.size()) return nullptr;
        return vChain[nHeight];
    }
    friend bool operator==(const CChain& a, const CChain& b) {
        return a.vChain.size() == b.vChain.size() && a.vChain[a.vChain.size() - 1] == b.vChain[b.vChain.size() - 1];
    }
    bool Contains(const CBlockIndex* pindex) const { return (*this)[pindex->nHeight] == pindex; }
    CBlockIndex* Next(const CBlockIndex* pindex) const {
        if (Contains(pindex)) return (*this)[pindex->nHeight + 1];
        return nullptr;
    }
    int Height() const { return (int)vChain.size() - 1; }
    void SetTip(CBlockIndex* pindex);
    CBlockLocator GetLocator(const CBlockIndex* pindex = nullptr) const;
    const CBlockIndex* FindFork(const CBlockIndex* pindex) const;
    CBlockIndex* FindEarliestAtLeast(int64_t nTime) const;
};

} // namespace bcp
