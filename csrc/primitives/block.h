// Block header / block with the BCP dual header format.
// Parity: reference src/primitives/block.{h,cpp}:
//   new format (Zcash-compatible): nVersion | hashPrevBlock | hashMerkleRoot | nHeight |
//     nReserved[7] | nTime | nBits | nNonce(uint256) | nSolution (compact-size vector)  = 140 B + solution
//   legacy format (stream version & SERIALIZE_BLOCK_LEGACY): 80-byte Bitcoin header with the
//     low 32 bits of nNonce
//   GetHash(params): the header's own nHeight >= BCPHeight selects the new format.
//   CEquihashInput: the first 108 bytes of the new format (no nonce/solution).
#pragma once
#include "primitives/serialize.h"
#include "primitives/transaction.h"
#include "primitives/uint256.h"

#include <cstring>
#include <string>
#include <vector>

namespace bcp {

namespace Consensus { struct Params; }

class CBlockHeader {
public:
    int32_t nVersion;
    uint256 hashPrevBlock;
    uint256 hashMerkleRoot;
    uint32_t nHeight;
    uint32_t nReserved[7];
    uint32_t nTime;
    uint32_t nBits;
    uint256 nNonce;
    std::vector<unsigned char> nSolution;

    CBlockHeader() { SetNull(); }

    template <typename S> void Serialize(S& s) const {
        const bool legacy = (s.GetVersion() & SERIALIZE_BLOCK_LEGACY) != 0;
        ::bcp::Serialize(s, nVersion);
        ::bcp::Serialize(s, hashPrevBlock);
        ::bcp::Serialize(s, hashMerkleRoot);
        if (!legacy) {
            ::bcp::Serialize(s, nHeight);
            for (int i = 0; i < 7; ++i) ::bcp::Serialize(s, nReserved[i]);
        }
        ::bcp::Serialize(s, nTime);
        ::bcp::Serialize(s, nBits);
        if (!legacy) {
            ::bcp::Serialize(s, nNonce);
            ::bcp::Serialize(s, nSolution);
        } else {
            ::bcp::Serialize(s, (uint32_t)nNonce.GetUint64(0));
        }
    }
    template <typename S> void Unserialize(S& s) {
        const bool legacy = (s.GetVersion() & SERIALIZE_BLOCK_LEGACY) != 0;
        ::bcp::Unserialize(s, nVersion);
        ::bcp::Unserialize(s, hashPrevBlock);
        ::bcp::Unserialize(s, hashMerkleRoot);
        if (!legacy) {
            ::bcp::Unserialize(s, nHeight);
            for (int i = 0; i < 7; ++i) ::bcp::Unserialize(s, nReserved[i]);
        } else {
            nHeight = 0;
            memset(nReserved, 0, sizeof(nReserved));
        }
        ::bcp::Unserialize(s, nTime);
        ::bcp::Unserialize(s, nBits);
        if (!legacy) {
            ::bcp::Unserialize(s, nNonce);
            ::bcp::Unserialize(s, nSolution);
        } else {
            uint32_t n32;
            ::bcp::Unserialize(s, n32);
            nNonce.SetNull();
            memcpy(nNonce.begin(), &n32, 4);
            nSolution.clear();
        }
    }

    void SetNull() {
        nVersion = 0;
        hashPrevBlock.SetNull();
        hashMerkleRoot.SetNull();
        nHeight = 0;
        memset(nReserved, 0, sizeof(nReserved));
        nTime = 0;
        nBits = 0;
        nNonce.SetNull();
        nSolution.clear();
    }
    bool IsNull() const { return nBits == 0; }
    // Hash in the format the header's own nHeight selects.
    uint256 GetHash(const Consensus::Params& params) const;
    uint256 GetHash() const; // uses the active chain parameters
    // Explicit-format hashes.
    uint256 GetHashLegacy() const;
    uint256 GetHashNew() const;
    int64_t GetBlockTime() const { return (int64_t)nTime; }
    // 108-byte CEquihashInput serialization (reference src/primitives/block.h:147)
    std::vector<unsigned char> EquihashInput() const;
};

class CBlock : public CBlockHeader {
public:
    std::vector<CTransactionRef> vtx;
    mutable bool fChecked = false;

    CBlock() { SetNull(); }
    CBlock(const CBlockHeader& header) {
        SetNull();
        *(CBlockHeader*)this = header;
    }
    template <typename S> void Serialize(S& s) const {
        CBlockHeader::Serialize(s);
        ::bcp::Serialize(s, vtx);
    }
    template <typename S> void Unserialize(S& s) {
        CBlockHeader::Unserialize(s);
        ::bcp::Unserialize(s, vtx);
    }
    void SetNull() {
        CBlockHeader::SetNull();
        vtx.clear();
        fChecked = false;
    }
    CBlockHeader GetBlockHeader() const { return *(const CBlockHeader*)this; }
    std::string ToString() const;
};

struct CBlockLocator {
    std::vector<uint256> vHave;
    CBlockLocator() {}
    explicit CBlockLocator(const std::vector<uint256>& v) : vHave(v) {}
    template <typename S> void Serialize(S& s) const {
        int nVersion = s.GetVersion();
        if (!(s.GetType() & SER_GETHASH)) ::bcp::Serialize(s, nVersion);
        ::bcp::Serialize(s, vHave);
    }
    template <typename S> void Unserialize(S& s) {
        int nVersion = 0;
        if (!(s.GetType() & SER_GETHASH)) ::bcp::Unserialize(s, nVersion);
        ::bcp::Unserialize(s, vHave);
    }
    void SetNull() { vHave.clear(); }
    bool IsNull() const { return vHave.empty(); }
};

} // namespace bcp
