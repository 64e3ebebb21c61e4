// P2P protocol logic.
// Parity: reference src/net_processing.{h,cpp}: per-peer CNodeState (best known block,
// blocks in flight, sync/stall state, misbehaviour score, header/cmpct preferences),
// ProcessMessage handlers for every NetMsgType (version/verack handshake with
// BCP_HARD_FORK_VERSION legacy-header negotiation, addr, inv/getdata, getblocks,
// getheaders/headers (headers-first sync, unconnecting-header handling), tx with the
// orphan pool, block, BIP152 cmpctblock/getblocktxn/blocktxn, BIP37 filterload/add/clear
// and merkleblock, mempool, ping/pong, feefilter, reject, notfound), SendMessages
// (pings, addr trickle, block announcements via headers/cmpct/inv, tx inventory
// trickle with fee/bloom filters, block download scheduling with a 1024-block window
// and 16 in flight per peer, stall/timeout eviction, feefilter), and the validation
// callbacks (UpdatedBlockTip, BlockConnected, NewPoWValidBlock, BlockChecked).
#pragma once
#include "net/net.h"
#include "node/signals.h"

namespace bcp {

class Chainstate;
class CTxMemPool;

struct CNodeStateStats {
    int nMisbehavior = 0;
    int nSyncHeight = -1;
    int nCommonHeight = -1;
    std::vector<int> vHeightInFlight;
};

class PeerLogicValidation : public CValidationInterface, public NetEventsInterface {
public:
    PeerLogicValidation(CConnman* connman, Chainstate* chainstate, CTxMemPool* mempool);
    ~PeerLogicValidation();

    // NetEventsInterface
    void InitializeNode(CNode* pnode) override;
    void FinalizeNode(NodeId id, bool& fUpdateConnectionTime) override;
    bool ProcessMessages(CNode* pnode, std::atomic<bool>& interrupt) override;
    bool SendMessages(CNode* pnode, std::atomic<bool>& interrupt) override;

    // CValidationInterface
    void UpdatedBlockTip(const CBlockIndex* pindexNew, const CBlockIndex* pindexFork, bool fInitialDownload) override;
    void BlockConnected(const std::shared_ptr<const CBlock>& block, const CBlockIndex* pindex,
                        const std::vector<CTransactionRef>& txnConflicted) override;
    void NewPoWValidBlock(const CBlockIndex* pindex, const std::shared_ptr<const CBlock>& block) override;
    void BlockChecked(const CBlock& block, const CValidationState& state) override;
    void TransactionAddedToMempool(const CTransactionRef& tx) override;

    bool GetNodeStateStats(NodeId id, CNodeStateStats& stats);
    void Misbehaving(NodeId id, int howmuch, const std::string& reason = "");
    size_t OrphanCount();
    // The orphan pool (reference net_processing.cpp AddOrphanTx / EraseOrphansFor /
    // LimitOrphanTxSize, also exercised directly by DoS_tests): returns whether the tx was kept,
    // and how many orphans the limit evicted.
    bool AddOrphanTx(const CTransactionRef& tx, NodeId peer);
    void EraseOrphansFor(NodeId peer);
    unsigned LimitOrphanTxSize(unsigned nMaxOrphans);
    // relay a locally-submitted transaction (sendrawtransaction / wallet)
    void RelayTransaction(const CTransaction& tx);

    struct Impl;

private:
    std::unique_ptr<Impl> impl;
};

PeerLogicValidation* GetPeerLogic();

} // namespace bcp
