// BIP152 compact blocks.
// Parity: reference src/blockencodings.{h,cpp}: CBlockHeaderAndShortTxIDs (header,
// 64-bit nonce, 6-byte SipHash-2-4 short ids keyed by SHA256(header || nonce),
// differentially-encoded prefilled transactions), BlockTransactionsRequest /
// BlockTransactions (getblocktxn / blocktxn), PartiallyDownloadedBlock (InitData
// from the mempool + extra txn pool, IsTxAvailable, FillBlock with merkle re-check).
#pragma once
#include "primitives/block.h"

#include <memory>
#include <vector>

namespace bcp {

class CTxMemPool;
class CValidationState;

// Upper bound on transactions a compact block can reference (16-bit indexes).
static const size_t MAX_BLOCK_TX_COUNT_CMPCT = 0xFFFF;


struct PrefilledTransaction {
    uint16_t index = 0; // absolute when in memory; differential on the wire
    CTransactionRef tx;
};

class CBlockHeaderAndShortTxIDs {
public:
    static const int SHORTTXIDS_LENGTH = 6;
    CBlockHeaderAndShortTxIDs() {}
    CBlockHeaderAndShortTxIDs(const CBlock& block, uint64_t nonce);
    uint64_t GetShortID(const uint256& txhash) const;
    size_t BlockTxCount() const { return shorttxids.size() + prefilledtxn.size(); }

    CBlockHeader header;
    uint64_t nonce = 0;
    std::vector<uint64_t> shorttxids;
    std::vector<PrefilledTransaction> prefilledtxn;

    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, header);
        ::bcp::Serialize(s, nonce);
        WriteCompactSize(s, shorttxids.size());
        for (uint64_t id : shorttxids) {
            unsigned char b[6];
            for (int i = 0; i < 6; i++) b[i] = (unsigned char)(id >> (8 * i));
            s.write((const char*)b, 6);
        }
        WriteCompactSize(s, prefilledtxn.size());
        uint64_t prev = 0;
        for (size_t i = 0; i < prefilledtxn.size(); i++) {
            const uint64_t diff = prefilledtxn[i].index - (i ? prev + 1 : 0);
            WriteCompactSize(s, diff);
            prev = prefilledtxn[i].index;
            ::bcp::Serialize(s, *prefilledtxn[i].tx);
        }
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, header);
        ::bcp::Unserialize(s, nonce);
        const uint64_t n = ReadCompactSize(s);
        shorttxids.resize(n);
        for (uint64_t i = 0; i < n; i++) {
            unsigned char b[6];
            s.read((char*)b, 6);
            uint64_t id = 0;
            for (int k = 0; k < 6; k++) id |= (uint64_t)b[k] << (8 * k);
            shorttxids[i] = id;
        }
        const uint64_t np = ReadCompactSize(s);
        prefilledtxn.resize(np);
        uint64_t idx = 0;
        for (uint64_t i = 0; i < np; i++) {
            const uint64_t diff = ReadCompactSize(s);
            idx = (i ? idx + 1 : 0) + diff;
            if (idx > 0xFFFF) throw ser_error("indexes overflowed 16 bits");
            prefilledtxn[i].index = (uint16_t)idx;
            CMutableTransaction mtx;
            ::bcp::Unserialize(s, mtx);
            prefilledtxn[i].tx = MakeTransactionRef(std::move(mtx));
        }
        FillShortTxIDSelector();
        if (BlockTxCount() > 0xFFFF) throw ser_error("indexes overflowed 16 bits");
    }

    // SipHash key (k0, k1) of the short ids (keyed on first use)
    uint64_t Key0() const { if (!keyed) FillShortTxIDSelector(); return k0; }
    uint64_t Key1() const { if (!keyed) FillShortTxIDSelector(); return k1; }

private:
    void FillShortTxIDSelector() const;
    mutable uint64_t k0 = 0, k1 = 0;
    mutable bool keyed = false;
};

// Short ids of many transactions under one compact block's key: on the GPU (K9, relay.hip) for
// at least -gpushortidthreshold transactions when a device is visible, else on the CPU.
std::vector<uint64_t> ShortTxIds(const CBlockHeaderAndShortTxIDs& cmpct, const std::vector<CTransactionRef>& txs);
void SetGpuShortIdThreshold(size_t n);
size_t GetGpuShortIdThreshold();

class BlockTransactionsRequest {
public:
    uint256 blockhash;
    std::vector<uint16_t> indexes; // absolute
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, blockhash);
        WriteCompactSize(s, indexes.size());
        for (size_t i = 0; i < indexes.size(); i++) WriteCompactSize(s, indexes[i] - (i ? indexes[i - 1] + 1 : 0));
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, blockhash);
        const uint64_t n = ReadCompactSize(s);
        if (n > 0xFFFF) throw ser_error("too many indexes");
        indexes.resize(n);
        uint64_t idx = 0;
        for (uint64_t i = 0; i < n; i++) {
            idx = (i ? idx + 1 : 0) + ReadCompactSize(s);
            if (idx > 0xFFFF) throw ser_error("index overflowed 16 bits");
            indexes[i] = (uint16_t)idx;
        }
    }
};

class BlockTransactions {
public:
    uint256 blockhash;
    std::vector<CTransactionRef> txn;
    BlockTransactions() {}
    explicit BlockTransactions(const BlockTransactionsRequest& req) : blockhash(req.blockhash), txn(req.indexes.size()) {}
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, blockhash);
        ::bcp::Serialize(s, txn);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, blockhash);
        ::bcp::Unserialize(s, txn);
    }
};

enum ReadStatus { READ_STATUS_OK, READ_STATUS_INVALID, READ_STATUS_FAILED, READ_STATUS_CHECKBLOCK_FAILED };

class PartiallyDownloadedBlock {
public:
    explicit PartiallyDownloadedBlock(CTxMemPool* pool) : pool(pool) {}
    ReadStatus InitData(const CBlockHeaderAndShortTxIDs& cmpctblock,
                        const std::vector<std::pair<uint256, CTransactionRef>>& extra_txn);
    bool IsTxAvailable(size_t index) const;
    ReadStatus FillBlock(CBlock& block, const std::vector<CTransactionRef>& vtx_missing);
    size_t prefilled_count = 0, mempool_count = 0, extra_count = 0;
    CBlockHeader header;

private:
    std::vector<CTransactionRef> txn_available;
    CTxMemPool* pool;
};

} // namespace bcp
