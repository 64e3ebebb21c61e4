#include "net/blockencodings.h"
#include "consensus/merkle.h"
#include "crypto/hashes.h"
#include "node/txmempool.h"
#include "util/util.h"
#include "kernels/gpu_api.h"

#include <atomic>
#include <cstring>

#include <unordered_map>

namespace bcp {

CBlockHeaderAndShortTxIDs::CBlockHeaderAndShortTxIDs(const CBlock& block, uint64_t n)
    : header(block), nonce(n), shorttxids(block.vtx.size() - 1) {
    FillShortTxIDSelector();
    // the coinbase is always prefilled
    prefilledtxn.push_back({0, block.vtx[0]});
    for (size_t i = 1; i < block.vtx.size(); i++) shorttxids[i - 1] = GetShortID(block.vtx[i]->GetHash());
}

void CBlockHeaderAndShortTxIDs::FillShortTxIDSelector() const {
    HashWriter hw(SER_NETWORK, PROTOCOL_VERSION);
    hw << header << nonce;
    const uint256 h = hw.GetSHA256();
    k0 = h.GetUint64(0);
    k1 = h.GetUint64(1);
    keyed = true;
}

uint64_t CBlockHeaderAndShortTxIDs::GetShortID(const uint256& txhash) const {
    if (!keyed) FillShortTxIDSelector();
    return SipHashUint256(k0, k1, txhash.begin()) & 0xffffffffffffULL;
}

static std::atomic<size_t> g_gpuShortIdThreshold{16384};
void SetGpuShortIdThreshold(size_t n) { g_gpuShortIdThreshold = n; }
size_t GetGpuShortIdThreshold() { return g_gpuShortIdThreshold.load(); }

std::vector<uint64_t> ShortTxIds(const CBlockHeaderAndShortTxIDs& cmpct, const std::vector<CTransactionRef>& txs) {
    std::vector<uint64_t> ids(txs.size());
    if (txs.size() >= g_gpuShortIdThreshold.load() && gpu::GpuAvailable()) {
        std::vector<unsigned char> flat(txs.size() * 32);
        for (size_t i = 0; i < txs.size(); i++) memcpy(&flat[32 * i], txs[i]->GetHash().begin(), 32);
        try {
            ids = gpu::ShortTxIdBatch(cmpct.Key0(), cmpct.Key1(), flat.data(), txs.size());
            return ids;
        } catch (const std::exception& e) {
            // a device error must not lose the reconstruction: hash on the CPU
            LogPrint(BCLog::CMPCTBLOCK, "GPU short ids failed (%s); computing them on the CPU\n", e.what());
        }
    }
    for (size_t i = 0; i < txs.size(); i++) ids[i] = cmpct.GetShortID(txs[i]->GetHash());
    return ids;
}

ReadStatus PartiallyDownloadedBlock::InitData(const CBlockHeaderAndShortTxIDs& cmpct,
                                              const std::vector<std::pair<uint256, CTransactionRef>>& extra_txn) {
    if (cmpct.header.IsNull() || (cmpct.shorttxids.empty() && cmpct.prefilledtxn.empty())) return READ_STATUS_INVALID;
    if (cmpct.BlockTxCount() > MAX_BLOCK_TX_COUNT_CMPCT) return READ_STATUS_INVALID;
    header = cmpct.header;
    txn_available.assign(cmpct.BlockTxCount(), nullptr);

    int32_t lastprefilled = -1;
    for (const PrefilledTransaction& p : cmpct.prefilledtxn) {
        if (!p.tx || p.tx->IsNull()) return READ_STATUS_INVALID;
        if ((int32_t)p.index <= lastprefilled || p.index >= txn_available.size()) return READ_STATUS_INVALID;
        lastprefilled = p.index;
        txn_available[p.index] = p.tx;
    }
    prefilled_count = cmpct.prefilledtxn.size();

    // short id -> slot
    std::unordered_map<uint64_t, uint16_t> idmap;
    idmap.reserve(cmpct.shorttxids.size());
    uint16_t slot = 0;
    for (size_t i = 0; i < cmpct.shorttxids.size(); i++) {
        while (txn_available[slot]) slot++;
        if (!idmap.emplace(cmpct.shorttxids[i], slot).second) return READ_STATUS_FAILED; // short id collision
        slot++;
    }
    // bucket-size sanity (reference: fail if the table degenerates)
    std::vector<bool> haveDup(txn_available.size(), false);
    auto offer = [&](const uint256& h, uint64_t shortid, const CTransactionRef& tx, size_t& counter) {
        auto it = idmap.find(shortid);
        if (it == idmap.end()) return;
        const uint16_t idx = it->second;
        if (!haveDup[idx]) {
            if (!txn_available[idx]) {
                txn_available[idx] = tx;
                counter++;
            }
            haveDup[idx] = true;
        } else if (txn_available[idx] && txn_available[idx]->GetHash() != h) {
            // two candidates for one short id: request it instead
            txn_available[idx].reset();
            counter--;
        }
    };
    if (pool) {
        const std::vector<CTransactionRef> all = pool->AllTransactions();
        const std::vector<uint64_t> ids = ShortTxIds(cmpct, all);
        for (size_t i = 0; i < all.size(); i++) offer(all[i]->GetHash(), ids[i], all[i], mempool_count);
    }
    for (const auto& e : extra_txn) {
        if (!e.second) continue;
        offer(e.first, cmpct.GetShortID(e.first), e.second, extra_count);
    }
    LogPrint(BCLog::CMPCTBLOCK, "Initialized PartiallyDownloadedBlock for block %s using a cmpctblock of size %zu\n",
             cmpct.header.GetHash().ToString().c_str(), GetSerializeSize(cmpct));
    return READ_STATUS_OK;
}

bool PartiallyDownloadedBlock::IsTxAvailable(size_t index) const {
    return index < txn_available.size() && txn_available[index] != nullptr;
}

ReadStatus PartiallyDownloadedBlock::FillBlock(CBlock& block, const std::vector<CTransactionRef>& vtx_missing) {
    if (header.IsNull()) return READ_STATUS_INVALID;
    block = CBlock(header);
    block.vtx.resize(txn_available.size());
    size_t tx_missing_offset = 0;
    for (size_t i = 0; i < txn_available.size(); i++) {
        if (!txn_available[i]) {
            if (tx_missing_offset >= vtx_missing.size()) return READ_STATUS_INVALID;
            block.vtx[i] = vtx_missing[tx_missing_offset++];
        } else {
            block.vtx[i] = std::move(txn_available[i]);
        }
    }
    header.SetNull();
    txn_available.clear();
    if (vtx_missing.size() != tx_missing_offset) return READ_STATUS_INVALID;
    // A wrong short-id match shows up as a merkle mismatch or a duplicated transaction: corruption
    // is possible, so the read failed rather than the block being invalid (reference
    // blockencodings.cpp FillBlock: CheckBlock + CorruptionPossible -> READ_STATUS_FAILED).
    bool mutated = false;
    if (BlockMerkleRoot(block, &mutated) != block.hashMerkleRoot || mutated) return READ_STATUS_FAILED;
    LogPrint(BCLog::CMPCTBLOCK, "Successfully reconstructed block %s with %zu txn prefilled, %zu txn from mempool "
                                "(incl at least %zu from extra pool) and %zu txn requested\n",
             block.GetHash().ToString().c_str(), prefilled_count, mempool_count, extra_count, vtx_missing.size());
    return READ_STATUS_OK;
}

} // namespace bcp
