// Validation event bus (reference src/validationinterface.{h,cpp}: CValidationInterface
// callbacks UpdatedBlockTip, TransactionAddedToMempool, BlockConnected, BlockDisconnected,
// SetBestChain, Inventory, ResendWalletTransactions, BlockChecked, NewPoWValidBlock)
// plus the UI notifications of src/ui_interface.h used by the node (NotifyBlockTip,
// NotifyHeaderTip). Subscribers: wallet, ZMQ publisher, P2P logic, RPC long-poll.
#pragma once
#include "consensus/chain.h"
#include "consensus/validation_state.h"
#include "primitives/block.h"

#include <memory>
#include <mutex>
#include <vector>

namespace bcp {

class CValidationInterface {
public:
    virtual ~CValidationInterface() {}
    virtual void UpdatedBlockTip(const CBlockIndex* pindexNew, const CBlockIndex* pindexFork, bool fInitialDownload) {}
    virtual void TransactionAddedToMempool(const CTransactionRef& ptxn) {}
    virtual void TransactionRemovedFromMempool(const CTransactionRef& ptx) {}
    virtual void BlockConnected(const std::shared_ptr<const CBlock>& block, const CBlockIndex* pindex,
                                const std::vector<CTransactionRef>& txnConflicted) {}
    virtual void BlockDisconnected(const std::shared_ptr<const CBlock>& block) {}
    virtual void SetBestChain(const CBlockLocator& locator) {}
    virtual void Inventory(const uint256& hash) {}
    virtual void ResendWalletTransactions(int64_t nBestBlockTime) {}
    virtual void BlockChecked(const CBlock& block, const CValidationState& state) {}
    virtual void NewPoWValidBlock(const CBlockIndex* pindex, const std::shared_ptr<const CBlock>& block) {}
    virtual void NotifyHeaderTip(const CBlockIndex* pindex, bool fInitialDownload) {}
};

class MainSignals {
public:
    void Register(CValidationInterface* s);
    void Unregister(CValidationInterface* s);
    void UnregisterAll();
    void UpdatedBlockTip(const CBlockIndex* a, const CBlockIndex* b, bool ibd);
    void TransactionAddedToMempool(const CTransactionRef& tx);
    void TransactionRemovedFromMempool(const CTransactionRef& tx);
    void BlockConnected(const std::shared_ptr<const CBlock>& b, const CBlockIndex* p, const std::vector<CTransactionRef>& c);
    void BlockDisconnected(const std::shared_ptr<const CBlock>& b);
    void SetBestChain(const CBlockLocator& l);
    void Inventory(const uint256& h);
    void ResendWalletTransactions(int64_t t);
    void BlockChecked(const CBlock& b, const CValidationState& s);
    void NewPoWValidBlock(const CBlockIndex* p, const std::shared_ptr<const CBlock>& b);
    void NotifyHeaderTip(const CBlockIndex* p, bool ibd);

private:
    template <typename F> void Each(F f) {
        std::vector<CValidationInterface*> subs;
        {
            std::lock_guard<std::mutex> l(m);
            subs = list;
        }
        for (auto* s : subs) f(s);
    }
    std::mutex m;
    std::vector<CValidationInterface*> list;
};
MainSignals& GetMainSignals();

} // namespace bcp
