#include "node/signals.h"

#include <algorithm>

namespace bcp {

MainSignals& GetMainSignals() {
    static MainSignals s;
    return s;
}
void MainSignals::Register(CValidationInterface* s) {
    std::lock_guard<std::mutex> l(m);
    list.push_back(s);
}
void MainSignals::Unregister(CValidationInterface* s) {
    std::lock_guard<std::mutex> l(m);
    list.erase(std::remove(list.begin(), list.end(), s), list.end());
}
void MainSignals::UnregisterAll() {
    std::lock_guard<std::mutex> l(m);
    list.clear();
}
void MainSignals::UpdatedBlockTip(const CBlockIndex* a, const CBlockIndex* b, bool ibd) {
    Each([&](CValidationInterface* s) { s->UpdatedBlockTip(a, b, ibd); });
}
void MainSignals::TransactionAddedToMempool(const CTransactionRef& tx) {
    Each([&](CValidationInterface* s) { s->TransactionAddedToMempool(tx); });
}
void MainSignals::TransactionRemovedFromMempool(const CTransactionRef& tx) {
    Each([&](CValidationInterface* s) { s->TransactionRemovedFromMempool(tx); });
}
void MainSignals::BlockConnected(const std::shared_ptr<const CBlock>& b, const CBlockIndex* p,
                                 const std::vector<CTransactionRef>& c) {
    Each([&](CValidationInterface* s) { s->BlockConnected(b, p, c); });
}
void MainSignals::BlockDisconnected(const std::shared_ptr<const CBlock>& b) {
    Each([&](CValidationInterface* s) { s->BlockDisconnected(b); });
}
void MainSignals::SetBestChain(const CBlockLocator& l) {
    Each([&](CValidationInterface* s) { s->SetBestChain(l); });
}
void MainSignals::Inventory(const uint256& h) {
    Each([&](CValidationInterface* s) { s->Inventory(h); });
}
void MainSignals::ResendWalletTransactions(int64_t t) {
    Each([&](CValidationInterface* s) { s->ResendWalletTransactions(t); });
}
void MainSignals::BlockChecked(const CBlock& b, const CValidationState& st) {
    Each([&](CValidationInterface* s) { s->BlockChecked(b, st); });
}
void MainSignals::NewPoWValidBlock(const CBlockIndex* p, const std::shared_ptr<const CBlock>& b) {
    Each([&](CValidationInterface* s) { s->NewPoWValidBlock(p, b); });
}
void MainSignals::NotifyHeaderTip(const CBlockIndex* p, bool ibd) {
    Each([&](CValidationInterface* s) { s->NotifyHeaderTip(p, ibd); });
}

} // namespace bcp
