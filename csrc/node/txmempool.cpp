#include "node/txmempool.h"
#include "keys/key.h"
#include "consensus/tx_verify.h"
#include "node/policy.h"
#include "node/signals.h"
#include "util/strencodings.h"
#include "util/util.h"
#include "util/memusage.h"

#include <algorithm>
#include <queue>
#include <cmath>
#include <cstring>
#include <deque>
#include <stdexcept>

namespace bcp {

// ------------------------------------------------------------------ entry
// Heap usage of a transaction (reference core_memusage.h RecursiveDynamicUsage): the tx object
// in its make_shared block, its vin/vout arrays, and every script's byte buffer.
static size_t TxUsage(const CTransaction& tx) {
    size_t mem = memusage::MallocUsage(sizeof(CTransaction) + 2 * sizeof(long) + sizeof(void*)) +
                 memusage::DynamicUsage(tx.vin) + memusage::DynamicUsage(tx.vout);
    for (const CTxIn& in : tx.vin) mem += memusage::DynamicUsage(static_cast<const CScriptBase&>(in.scriptSig));
    for (const CTxOut& out : tx.vout)
        mem += memusage::DynamicUsage(static_cast<const CScriptBase&>(out.scriptPubKey));
    return mem;
}

CTxMemPoolEntry::CTxMemPoolEntry(const CTransactionRef& t, Amount fee, int64_t time, double priority,
                                 unsigned height, Amount inChain, bool cb, int64_t sigops, LockPoints lp)
    : tx(t), nFee(fee), nTime(time), entryPriority(priority), entryHeight(height), inChainInputValue(inChain),
      spendsCoinbase(cb), sigOpCount(sigops), lockPoints(lp) {
    nTxSize = tx->GetTotalSize();
    nModSize = nTxSize;
    for (const CTxIn& in : tx->vin) {
        const unsigned offset = 41U + std::min(110U, (unsigned)in.scriptSig.size());
        if (nModSize > offset) nModSize -= offset;
    }
    nUsageSize = TxUsage(*tx);
    nSizeWithDescendants = nTxSize;
    nModFeesWithDescendants = nFee;
    nSizeWithAncestors = nTxSize;
    nModFeesWithAncestors = nFee;
    nSigOpCountWithAncestors = sigOpCount;
}

double CTxMemPoolEntry::GetPriority(unsigned currentHeight) const {
    const double deltaPriority = nModSize ? ((double)(currentHeight - entryHeight) * inChainInputValue) / nModSize : 0;
    return entryPriority + deltaPriority;
}

// ------------------------------------------------------------------ pool
CTxMemPool::CTxMemPool(CBlockPolicyEstimator* est) : minerPolicyEstimator(est) {}

const CTxMemPool::setEntries& CTxMemPool::GetMemPoolParents(txiter it) const { return mapLinks.at(it).parents; }
const CTxMemPool::setEntries& CTxMemPool::GetMemPoolChildren(txiter it) const { return mapLinks.at(it).children; }

// Link sets are accounted incrementally (cachedLinkUsage) so DynamicMemoryUsage stays O(1).
void CTxMemPool::UpdateParent(txiter entry, txiter parent, bool add) {
    setEntries& s = mapLinks[entry].parents;
    if (add ? s.insert(parent).second : s.erase(parent) != 0) {
        if (add) cachedLinkUsage += memusage::IncrementalDynamicUsage(s);
        else cachedLinkUsage -= memusage::IncrementalDynamicUsage(s);
    }
}
void CTxMemPool::UpdateChild(txiter entry, txiter child, bool add) {
    setEntries& s = mapLinks[entry].children;
    if (add ? s.insert(child).second : s.erase(child) != 0) {
        if (add) cachedLinkUsage += memusage::IncrementalDynamicUsage(s);
        else cachedLinkUsage -= memusage::IncrementalDynamicUsage(s);
    }
}

bool CTxMemPool::CalculateMemPoolAncestors(const CTxMemPoolEntry& entry, setEntries& setAncestors,
                                           uint64_t limitAncestorCount, uint64_t limitAncestorSize,
                                           uint64_t limitDescendantCount, uint64_t limitDescendantSize,
                                           std::string& errString, bool fSearchForParents) const {
    setEntries parentHashes;
    const CTransaction& tx = entry.GetTx();
    if (fSearchForParents) {
        for (const CTxIn& in : tx.vin) {
            auto piter = TxMap().find(in.prevout.hash);
            if (piter != TxMap().end()) {
                parentHashes.insert(piter);
                if (parentHashes.size() + 1 > limitAncestorCount) {
                    errString = strprintf("too many unconfirmed parents [limit: %u]", (unsigned)limitAncestorCount);
                    return false;
                }
            }
        }
    } else {
        auto it = TxMap().find(tx.GetHash());
        parentHashes = GetMemPoolParents(it);
    }
    size_t totalSizeWithAncestors = entry.GetTxSize();
    while (!parentHashes.empty()) {
        txiter stageit = *parentHashes.begin();
        setAncestors.insert(stageit);
        parentHashes.erase(stageit);
        const CTxMemPoolEntry& s = *stageit->second;
        totalSizeWithAncestors += s.GetTxSize();
        if (s.GetSizeWithDescendants() + entry.GetTxSize() > limitDescendantSize) {
            errString = strprintf("exceeds descendant size limit for tx %s [limit: %u]",
                                  stageit->first.ToString().c_str(), (unsigned)limitDescendantSize);
            return false;
        }
        if (s.GetCountWithDescendants() + 1 > limitDescendantCount) {
            errString = strprintf("too many descendants for tx %s [limit: %u]", stageit->first.ToString().c_str(),
                                  (unsigned)limitDescendantCount);
            return false;
        }
        if (totalSizeWithAncestors > limitAncestorSize) {
            errString = strprintf("exceeds ancestor size limit [limit: %u]", (unsigned)limitAncestorSize);
            return false;
        }
        for (txiter p : GetMemPoolParents(stageit)) {
            if (!setAncestors.count(p)) parentHashes.insert(p);
            if (parentHashes.size() + setAncestors.size() + 1 > limitAncestorCount) {
                errString = strprintf("too many unconfirmed ancestors [limit: %u]", (unsigned)limitAncestorCount);
                return false;
            }
        }
    }
    return true;
}

void CTxMemPool::UpdateAncestorsOf(bool add, txiter it, setEntries& setAncestors) {
    for (txiter piter : GetMemPoolParents(it)) UpdateChild(piter, it, add);
    const int64_t updateCount = add ? 1 : -1;
    const int64_t updateSize = updateCount * (int64_t)it->second->GetTxSize();
    const Amount updateFee = updateCount * it->second->GetModifiedFee();
    for (txiter a : setAncestors) {
        CTxMemPoolEntry& e = *a->second;
        e.nSizeWithDescendants += updateSize;
        e.nModFeesWithDescendants += updateFee;
        e.nCountWithDescendants += updateCount;
    }
}

void CTxMemPool::UpdateEntryForAncestors(txiter it, const setEntries& setAncestors) {
    int64_t updateCount = setAncestors.size(), updateSize = 0, updateSigOps = 0;
    Amount updateFee = 0;
    for (txiter a : setAncestors) {
        updateSize += a->second->GetTxSize();
        updateFee += a->second->GetModifiedFee();
        updateSigOps += a->second->GetSigOpCount();
    }
    CTxMemPoolEntry& e = *it->second;
    e.nSizeWithAncestors += updateSize;
    e.nModFeesWithAncestors += updateFee;
    e.nCountWithAncestors += updateCount;
    e.nSigOpCountWithAncestors += updateSigOps;
}

void CTxMemPool::addUnchecked(const uint256& hash, const CTxMemPoolEntry& entry, bool validFeeEstimate) {
    std::lock_guard<CCriticalSection> l(cs);
    setEntries setAncestors;
    std::string dummy;
    const uint64_t nNoLimit = std::numeric_limits<uint64_t>::max();
    CalculateMemPoolAncestors(entry, setAncestors, nNoLimit, nNoLimit, nNoLimit, nNoLimit, dummy);
    addUnchecked(hash, entry, setAncestors, validFeeEstimate);
}

void CTxMemPool::addUnchecked(const uint256& hash, const CTxMemPoolEntry& entry, setEntries& setAncestors,
                              bool validFeeEstimate) {
    std::lock_guard<CCriticalSection> l(cs);
    auto ins = mapTx.emplace(hash, std::unique_ptr<CTxMemPoolEntry>(new CTxMemPoolEntry(entry)));
    txiter newit = ins.first;
    mapLinks.emplace(newit, Links());
    auto pos = mapDeltas.find(hash);
    if (pos != mapDeltas.end() && pos->second.second) {
        CTxMemPoolEntry& e = *newit->second;
        e.feeDelta = pos->second.second;
        e.nModFeesWithDescendants += e.feeDelta;
        e.nModFeesWithAncestors += e.feeDelta;
    }
    cachedInnerUsage += entry.DynamicMemoryUsage();
    const CTransaction& tx = newit->second->GetTx();
    std::set<uint256> setParentTransactions;
    for (const CTxIn& in : tx.vin) {
        mapNextTx.insert(std::make_pair(&in.prevout, &tx));
        setParentTransactions.insert(in.prevout.hash);
    }
    for (const uint256& ph : setParentTransactions) {
        auto pit = mapTx.find(ph);
        if (pit != mapTx.end()) UpdateParent(newit, pit, true);
    }
    UpdateAncestorsOf(true, newit, setAncestors);
    UpdateEntryForAncestors(newit, setAncestors);
    nTransactionsUpdated++;
    totalTxSize += entry.GetTxSize();
    if (minerPolicyEstimator)
        minerPolicyEstimator->processTransaction(hash, CFeeRate(entry.GetFee(), entry.GetTxSize()), entry.GetHeight(),
                                                 validFeeEstimate, entry.GetPriority(entry.GetHeight()));
}

void CTxMemPool::CalculateDescendants(txiter entryit, setEntries& setDescendants) {
    setEntries stage;
    if (!setDescendants.count(entryit)) stage.insert(entryit);
    while (!stage.empty()) {
        txiter it = *stage.begin();
        setDescendants.insert(it);
        stage.erase(it);
        for (txiter c : GetMemPoolChildren(it))
            if (!setDescendants.count(c)) stage.insert(c);
    }
}

void CTxMemPool::UpdateForRemoveFromMempool(const setEntries& entriesToRemove, bool updateDescendants) {
    const uint64_t nNoLimit = std::numeric_limits<uint64_t>::max();
    if (updateDescendants) {
        for (txiter removeIt : entriesToRemove) {
            setEntries setDescendants;
            CalculateDescendants(removeIt, setDescendants);
            setDescendants.erase(removeIt);
            const int64_t modifySize = -((int64_t)removeIt->second->GetTxSize());
            const Amount modifyFee = -removeIt->second->GetModifiedFee();
            const int64_t modifySigOps = -removeIt->second->GetSigOpCount();
            for (txiter d : setDescendants) {
                CTxMemPoolEntry& e = *d->second;
                e.nSizeWithAncestors += modifySize;
                e.nModFeesWithAncestors += modifyFee;
                e.nCountWithAncestors -= 1;
                e.nSigOpCountWithAncestors += modifySigOps;
            }
        }
    }
    for (txiter removeIt : entriesToRemove) {
        setEntries setAncestors;
        std::string dummy;
        CalculateMemPoolAncestors(*removeIt->second, setAncestors, nNoLimit, nNoLimit, nNoLimit, nNoLimit, dummy,
                                  false);
        UpdateAncestorsOf(false, removeIt, setAncestors);
    }
    for (txiter removeIt : entriesToRemove)
        for (txiter c : GetMemPoolChildren(removeIt)) UpdateParent(c, removeIt, false);
}

void CTxMemPool::removeUnchecked(txiter it, MemPoolRemovalReason reason) {
    CTransactionRef ptx = it->second->GetSharedTx();
    for (const CTxIn& in : ptx->vin) mapNextTx.erase(in.prevout);
    totalTxSize -= it->second->GetTxSize();
    cachedInnerUsage -= it->second->DynamicMemoryUsage();
    {
        auto li = mapLinks.find(it);
        if (li != mapLinks.end()) {
            cachedLinkUsage -= memusage::DynamicUsage(li->second.parents) + memusage::DynamicUsage(li->second.children);
            mapLinks.erase(li);
        }
    }
    const uint256 h = it->first;
    mapTx.erase(it);
    nTransactionsUpdated++;
    if (minerPolicyEstimator) minerPolicyEstimator->removeTx(h);
    if (reason != MemPoolRemovalReason::BLOCK) GetMainSignals().TransactionRemovedFromMempool(ptx);
}

void CTxMemPool::RemoveStaged(setEntries& stage, bool updateDescendants, MemPoolRemovalReason reason) {
    std::lock_guard<CCriticalSection> l(cs);
    UpdateForRemoveFromMempool(stage, updateDescendants);
    for (txiter it : stage) removeUnchecked(it, reason);
}

void CTxMemPool::removeRecursive(const CTransaction& origTx, MemPoolRemovalReason reason) {
    std::lock_guard<CCriticalSection> l(cs);
    setEntries txToRemove;
    auto origit = mapTx.find(origTx.GetHash());
    if (origit != mapTx.end()) {
        txToRemove.insert(origit);
    } else {
        // not in the pool (e.g. a block tx re-added after reorg failed): remove its spenders
        for (size_t i = 0; i < origTx.vout.size(); i++) {
            auto it = mapNextTx.find(COutPoint(origTx.GetHash(), (uint32_t)i));
            if (it == mapNextTx.end()) continue;
            auto nextit = mapTx.find(it->second->GetHash());
            if (nextit != mapTx.end()) txToRemove.insert(nextit);
        }
    }
    setEntries setAllRemoves;
    for (txiter it : txToRemove) CalculateDescendants(it, setAllRemoves);
    RemoveStaged(setAllRemoves, false, reason);
}

void CTxMemPool::removeForReorg(const CCoinsViewCache* pcoins, unsigned nMemPoolHeight, int flags,
                                const std::function<bool(const CTransaction&, LockPoints&, bool)>& checkLocks,
                                const std::function<bool(const LockPoints*)>& lpValid) {
    std::lock_guard<CCriticalSection> l(cs);
    (void)flags;
    setEntries txToRemove;
    for (auto it = mapTx.begin(); it != mapTx.end(); ++it) {
        const CTransaction& tx = it->second->GetTx();
        LockPoints lp = it->second->GetLockPoints();
        const bool validLP = lpValid(&lp);
        if (!checkLocks(tx, lp, validLP)) {
            txToRemove.insert(it);
        } else if (it->second->GetSpendsCoinbase()) {
            for (const CTxIn& in : tx.vin) {
                if (mapTx.count(in.prevout.hash)) continue;
                const Coin& coin = pcoins->AccessCoin(in.prevout);
                if (coin.IsSpent() ||
                    (coin.IsCoinBase() && (int64_t)nMemPoolHeight - coin.GetHeight() < COINBASE_MATURITY)) {
                    txToRemove.insert(it);
                    break;
                }
            }
        }
        if (!validLP) it->second->lockPoints = lp;
    }
    setEntries setAllRemoves;
    for (txiter it : txToRemove) CalculateDescendants(it, setAllRemoves);
    RemoveStaged(setAllRemoves, false, MemPoolRemovalReason::REORG);
}

void CTxMemPool::removeConflicts(const CTransaction& tx) {
    std::lock_guard<CCriticalSection> l(cs);
    for (const CTxIn& in : tx.vin) {
        auto it = mapNextTx.find(in.prevout);
        if (it == mapNextTx.end()) continue;
        const CTransaction& txConflict = *it->second;
        if (txConflict != tx) {
            ClearPrioritisation(txConflict.GetHash());
            removeRecursive(txConflict, MemPoolRemovalReason::CONFLICT);
        }
    }
}

void CTxMemPool::removeForBlock(const std::vector<CTransactionRef>& vtx, unsigned nBlockHeight) {
    std::lock_guard<CCriticalSection> l(cs);
    std::vector<uint256> confirmed;
    for (const auto& tx : vtx)
        if (mapTx.count(tx->GetHash())) confirmed.push_back(tx->GetHash());
    if (minerPolicyEstimator) minerPolicyEstimator->processBlock(nBlockHeight, confirmed);
    for (const auto& tx : vtx) {
        auto it = mapTx.find(tx->GetHash());
        if (it != mapTx.end()) {
            setEntries stage{it};
            RemoveStaged(stage, true, MemPoolRemovalReason::BLOCK);
        }
        removeConflicts(*tx);
        ClearPrioritisation(tx->GetHash());
    }
    lastRollingFeeUpdate = GetTime();
    blockSinceLastRollingFeeBump = true;
}

void CTxMemPool::clear() {
    std::lock_guard<CCriticalSection> l(cs);
    mapLinks.clear();
    mapTx.clear();
    mapNextTx.clear();
    totalTxSize = 0;
    cachedInnerUsage = 0;
    cachedLinkUsage = 0;
    lastRollingFeeUpdate = GetTime();
    blockSinceLastRollingFeeBump = false;
    rollingMinimumFeeRate = 0;
    ++nTransactionsUpdated;
}

int CTxMemPool::Expire(int64_t time) {
    std::lock_guard<CCriticalSection> l(cs);
    setEntries toremove;
    for (auto it = mapTx.begin(); it != mapTx.end(); ++it)
        if (it->second->GetTime() < time) toremove.insert(it);
    setEntries stage;
    for (txiter it : toremove) CalculateDescendants(it, stage);
    RemoveStaged(stage, false, MemPoolRemovalReason::EXPIRY);
    return (int)stage.size();
}

void CTxMemPool::trackPackageRemoved(const CFeeRate& rate) {
    if ((double)rate.GetFeePerK() > rollingMinimumFeeRate) {
        rollingMinimumFeeRate = (double)rate.GetFeePerK();
        blockSinceLastRollingFeeBump = false;
    }
}

CFeeRate CTxMemPool::GetMinFee(size_t sizelimit) const {
    std::lock_guard<CCriticalSection> l(cs);
    if (!blockSinceLastRollingFeeBump || rollingMinimumFeeRate == 0) return CFeeRate((Amount)rollingMinimumFeeRate);
    const int64_t time = GetTime();
    if (time > lastRollingFeeUpdate + 10) {
        double halflife = ROLLING_FEE_HALFLIFE;
        if (DynamicMemoryUsage() < sizelimit / 4) halflife /= 4;
        else if (DynamicMemoryUsage() < sizelimit / 2) halflife /= 2;
        rollingMinimumFeeRate = rollingMinimumFeeRate / std::pow(2.0, (time - lastRollingFeeUpdate) / halflife);
        lastRollingFeeUpdate = time;
        if (rollingMinimumFeeRate < (double)incrementalRelayFee.GetFeePerK() / 2) {
            rollingMinimumFeeRate = 0;
            return CFeeRate(0);
        }
    }
    return std::max(CFeeRate((Amount)rollingMinimumFeeRate), incrementalRelayFee);
}

static double DescendantScore(const CTxMemPoolEntry& e) {
    // max(own feerate, package feerate): the eviction key
    const double own = (double)e.GetModifiedFee() / e.GetTxSize();
    const double pkg = (double)e.GetModFeesWithDescendants() / e.GetSizeWithDescendants();
    return std::max(own, pkg);
}

void CTxMemPool::TrimToSize(size_t sizelimit, std::vector<COutPoint>* pvNoSpendsRemaining) {
    std::lock_guard<CCriticalSection> l(cs);
    unsigned nTxnRemoved = 0;
    CFeeRate maxFeeRateRemoved(0);
    if (DynamicMemoryUsage() <= sizelimit) return;
    // Eviction order = lowest descendant score first, newest first on ties, then lowest txid
    // (reference: the descendant_score index of mapTx). A lazy min-heap replaces the ordered
    // index: when a package goes, the ancestors it leaves behind are re-queued with their new
    // score, and a popped candidate whose score no longer matches is stale and skipped.
    struct Cand {
        double score;
        int64_t time;
        uint256 hash;
    };
    auto lowerPriority = [](const Cand& a, const Cand& b) {
        if (a.score != b.score) return a.score > b.score;
        if (a.time != b.time) return a.time < b.time;
        return b.hash < a.hash;
    };
    std::vector<Cand> init;
    init.reserve(mapTx.size());
    for (const auto& kv : mapTx) init.push_back({DescendantScore(*kv.second), kv.second->GetTime(), kv.first});
    std::priority_queue<Cand, std::vector<Cand>, decltype(lowerPriority)> heap(lowerPriority, std::move(init));
    while (!heap.empty() && DynamicMemoryUsage() > sizelimit) {
        const Cand c = heap.top();
        heap.pop();
        txiter worst = mapTx.find(c.hash);
        if (worst == mapTx.end() || DescendantScore(*worst->second) != c.score) continue;
        CFeeRate removed(worst->second->GetModFeesWithDescendants(), worst->second->GetSizeWithDescendants());
        removed += incrementalRelayFee;
        trackPackageRemoved(removed);
        maxFeeRateRemoved = std::max(maxFeeRateRemoved, removed);
        setEntries stage;
        CalculateDescendants(worst, stage);
        nTxnRemoved += stage.size();
        // ancestors outside the package lose descendants: their scores change
        std::set<uint256> touched;
        {
            std::vector<txiter> todo(stage.begin(), stage.end());
            while (!todo.empty()) {
                txiter t = todo.back();
                todo.pop_back();
                for (txiter p : GetMemPoolParents(t))
                    if (!stage.count(p) && touched.insert(p->first).second) todo.push_back(p);
            }
        }
        std::vector<CTransactionRef> txn;
        if (pvNoSpendsRemaining)
            for (txiter it : stage) txn.push_back(it->second->GetSharedTx());
        RemoveStaged(stage, false, MemPoolRemovalReason::SIZELIMIT);
        for (const uint256& h : touched) {
            auto it = mapTx.find(h);
            if (it != mapTx.end()) heap.push({DescendantScore(*it->second), it->second->GetTime(), h});
        }
        if (pvNoSpendsRemaining) {
            for (const auto& tx : txn)
                for (const CTxIn& in : tx->vin) {
                    if (exists(in.prevout.hash)) continue;
                    if (!mapNextTx.count(in.prevout)) pvNoSpendsRemaining->push_back(in.prevout);
                }
        }
    }
    if (maxFeeRateRemoved > CFeeRate(0))
        LogPrint(BCLog::MEMPOOL, "Removed %u txn, rolling minimum fee bumped to %lld\n", nTxnRemoved,
                 (long long)maxFeeRateRemoved.GetFeePerK());
}

void CTxMemPool::UpdateForDescendants(txiter updateIt, std::map<txiter, setEntries, IterCmp>& cached,
                                      const std::set<uint256>& setExclude) {
    setEntries stageEntries, setAllDescendants;
    stageEntries = GetMemPoolChildren(updateIt);
    while (!stageEntries.empty()) {
        txiter cit = *stageEntries.begin();
        setAllDescendants.insert(cit);
        stageEntries.erase(cit);
        for (txiter c : GetMemPoolChildren(cit)) {
            auto cacheIt = cached.find(c);
            if (cacheIt != cached.end()) {
                for (txiter cc : cacheIt->second) setAllDescendants.insert(cc);
            } else if (!setAllDescendants.count(c)) {
                stageEntries.insert(c);
            }
        }
    }
    int64_t modifySize = 0, modifyCount = 0;
    Amount modifyFee = 0;
    CTxMemPoolEntry& u = *updateIt->second;
    for (txiter d : setAllDescendants) {
        if (setExclude.count(d->first)) continue;
        modifySize += d->second->GetTxSize();
        modifyFee += d->second->GetModifiedFee();
        modifyCount++;
        cached[updateIt].insert(d);
        CTxMemPoolEntry& de = *d->second;
        de.nSizeWithAncestors += u.GetTxSize();
        de.nModFeesWithAncestors += u.GetModifiedFee();
        de.nCountWithAncestors += 1;
        de.nSigOpCountWithAncestors += u.GetSigOpCount();
    }
    u.nSizeWithDescendants += modifySize;
    u.nModFeesWithDescendants += modifyFee;
    u.nCountWithDescendants += modifyCount;
}

void CTxMemPool::UpdateTransactionsFromBlock(const std::vector<uint256>& vHashesToUpdate) {
    std::lock_guard<CCriticalSection> l(cs);
    std::map<txiter, setEntries, IterCmp> mapMemPoolDescendantsToUpdate;
    std::set<uint256> setAlreadyIncluded(vHashesToUpdate.begin(), vHashesToUpdate.end());
    for (auto hit = vHashesToUpdate.rbegin(); hit != vHashesToUpdate.rend(); ++hit) {
        auto it = mapTx.find(*hit);
        if (it == mapTx.end()) continue;
        setEntries setChildren;
        auto iter = mapNextTx.lower_bound(COutPoint(*hit, 0));
        for (; iter != mapNextTx.end() && iter->first->hash == *hit; ++iter) {
            auto childIter = mapTx.find(iter->second->GetHash());
            if (childIter == mapTx.end()) continue;
            if (setChildren.insert(childIter).second && !setAlreadyIncluded.count(childIter->first)) {
                UpdateChild(it, childIter, true);
                UpdateParent(childIter, it, true);
            }
        }
        UpdateForDescendants(it, mapMemPoolDescendantsToUpdate, setAlreadyIncluded);
    }
}

void CTxMemPool::PrioritiseTransaction(const uint256& hash, double dPriorityDelta, Amount nFeeDelta) {
    std::lock_guard<CCriticalSection> l(cs);
    auto& d = mapDeltas[hash];
    d.first += dPriorityDelta;
    d.second += nFeeDelta;
    auto it = mapTx.find(hash);
    if (it != mapTx.end()) {
        CTxMemPoolEntry& e = *it->second;
        e.feeDelta += nFeeDelta;
        e.nModFeesWithDescendants += nFeeDelta;
        e.nModFeesWithAncestors += nFeeDelta;
        setEntries setAncestors;
        std::string dummy;
        const uint64_t nNoLimit = std::numeric_limits<uint64_t>::max();
        CalculateMemPoolAncestors(e, setAncestors, nNoLimit, nNoLimit, nNoLimit, nNoLimit, dummy, false);
        for (txiter a : setAncestors) a->second->nModFeesWithDescendants += nFeeDelta;
        setEntries setDescendants;
        CalculateDescendants(it, setDescendants);
        setDescendants.erase(it);
        for (txiter dd : setDescendants) dd->second->nModFeesWithAncestors += nFeeDelta;
        ++nTransactionsUpdated;
    }
    LogPrintf("PrioritiseTransaction: %s priority += %f, fee += %lld\n", hash.ToString().c_str(), dPriorityDelta,
              (long long)nFeeDelta);
}

void CTxMemPool::ApplyDeltas(const uint256& hash, double& dPriorityDelta, Amount& nFeeDelta) const {
    std::lock_guard<CCriticalSection> l(cs);
    auto pos = mapDeltas.find(hash);
    if (pos == mapDeltas.end()) return;
    dPriorityDelta += pos->second.first;
    nFeeDelta += pos->second.second;
}
void CTxMemPool::ClearPrioritisation(const uint256& hash) {
    std::lock_guard<CCriticalSection> l(cs);
    mapDeltas.erase(hash);
}
std::map<uint256, std::pair<double, Amount>> CTxMemPool::GetDeltas() const {
    std::lock_guard<CCriticalSection> l(cs);
    return mapDeltas;
}

bool CTxMemPool::TransactionWithinChainLimit(const uint256& txid, size_t chainLimit) const {
    std::lock_guard<CCriticalSection> l(cs);
    auto it = mapTx.find(txid);
    return it == mapTx.end() ||
           (it->second->GetCountWithAncestors() < chainLimit && it->second->GetCountWithDescendants() < chainLimit);
}

bool CTxMemPool::exists(const uint256& hash) const {
    std::lock_guard<CCriticalSection> l(cs);
    return mapTx.count(hash) > 0;
}
CTransactionRef CTxMemPool::get(const uint256& hash) const {
    std::lock_guard<CCriticalSection> l(cs);
    auto it = mapTx.find(hash);
    return it == mapTx.end() ? nullptr : it->second->GetSharedTx();
}
const CTxMemPoolEntry* CTxMemPool::GetEntry(const uint256& hash) const {
    std::lock_guard<CCriticalSection> l(cs);
    auto it = mapTx.find(hash);
    return it == mapTx.end() ? nullptr : it->second.get();
}
TxMempoolInfo CTxMemPool::info(const uint256& hash) const {
    std::lock_guard<CCriticalSection> l(cs);
    auto it = mapTx.find(hash);
    if (it == mapTx.end()) return TxMempoolInfo();
    const CTxMemPoolEntry& e = *it->second;
    return TxMempoolInfo{e.GetSharedTx(), e.GetTime(), CFeeRate(e.GetFee(), e.GetTxSize()), e.GetModifiedFee() - e.GetFee()};
}
std::vector<TxMempoolInfo> CTxMemPool::infoAll() const {
    std::lock_guard<CCriticalSection> l(cs);
    std::vector<TxMempoolInfo> r;
    for (const auto* e : SortedByDepthAndScore())
        r.push_back(TxMempoolInfo{e->GetSharedTx(), e->GetTime(), CFeeRate(e->GetFee(), e->GetTxSize()),
                                  e->GetModifiedFee() - e->GetFee()});
    return r;
}
void CTxMemPool::queryHashes(std::vector<uint256>& vtxid) const {
    std::lock_guard<CCriticalSection> l(cs);
    vtxid.clear();
    for (const auto* e : SortedByDepthAndScore()) vtxid.push_back(e->GetTx().GetHash());
}
bool CTxMemPool::HasNoInputsOf(const CTransaction& tx) const {
    for (const CTxIn& in : tx.vin)
        if (exists(in.prevout.hash)) return false;
    return true;
}
bool CTxMemPool::isSpent(const COutPoint& outpoint) const {
    std::lock_guard<CCriticalSection> l(cs);
    return mapNextTx.count(outpoint) > 0;
}
const CTransaction* CTxMemPool::GetConflictTx(const COutPoint& prevout) const {
    std::lock_guard<CCriticalSection> l(cs);
    auto it = mapNextTx.find(prevout);
    return it == mapNextTx.end() ? nullptr : it->second;
}
std::vector<const CTxMemPoolEntry*> CTxMemPool::GetAncestors(const uint256& hash) const {
    std::lock_guard<CCriticalSection> l(cs);
    std::vector<const CTxMemPoolEntry*> r;
    auto it = mapTx.find(hash);
    if (it == mapTx.end()) return r;
    setEntries setAncestors;
    std::string dummy;
    const uint64_t nNoLimit = std::numeric_limits<uint64_t>::max();
    CalculateMemPoolAncestors(*it->second, setAncestors, nNoLimit, nNoLimit, nNoLimit, nNoLimit, dummy, false);
    for (txiter a : setAncestors) r.push_back(a->second.get());
    return r;
}
std::vector<const CTxMemPoolEntry*> CTxMemPool::GetDescendants(const uint256& hash) const {
    std::lock_guard<CCriticalSection> l(cs);
    std::vector<const CTxMemPoolEntry*> r;
    auto it = TxMap().find(hash);
    if (it == TxMap().end()) return r;
    setEntries d;
    const_cast<CTxMemPool*>(this)->CalculateDescendants(it, d);
    d.erase(it);
    for (txiter x : d) r.push_back(x->second.get());
    return r;
}

static double AncestorScore(const CTxMemPoolEntry& e) {
    const double own = (double)e.GetModifiedFee() / e.GetTxSize();
    const double pkg = (double)e.GetModFeesWithAncestors() / e.GetSizeWithAncestors();
    return std::min(own, pkg);
}

std::vector<CTxMemPool::txiter> CTxMemPool::SortedByAncestorScore() {
    std::lock_guard<CCriticalSection> l(cs);
    std::vector<txiter> v;
    v.reserve(mapTx.size());
    for (auto it = mapTx.begin(); it != mapTx.end(); ++it) v.push_back(it);
    std::sort(v.begin(), v.end(), [](const txiter& a, const txiter& b) {
        const double sa = AncestorScore(*a->second), sb = AncestorScore(*b->second);
        if (sa != sb) return sa > sb;
        return a->first < b->first;
    });
    return v;
}

std::vector<const CTxMemPoolEntry*> CTxMemPool::SortedByDepthAndScore() const {
    std::lock_guard<CCriticalSection> l(cs);
    std::vector<const CTxMemPoolEntry*> v;
    for (const auto& kv : mapTx) v.push_back(kv.second.get());
    std::sort(v.begin(), v.end(), [](const CTxMemPoolEntry* a, const CTxMemPoolEntry* b) {
        if (a->GetCountWithAncestors() != b->GetCountWithAncestors())
            return a->GetCountWithAncestors() < b->GetCountWithAncestors();
        const double sa = DescendantScore(*a), sb = DescendantScore(*b);
        if (sa != sb) return sa > sb;
        return a->GetTx().GetHash() < b->GetTx().GetHash();
    });
    return v;
}

std::vector<CTransactionRef> CTxMemPool::AllTransactions() const {
    std::lock_guard<CCriticalSection> l(cs);
    std::vector<CTransactionRef> r;
    for (const auto* e : SortedByDepthAndScore()) r.push_back(e->GetSharedTx());
    return r;
}

unsigned long CTxMemPool::size() const {
    std::lock_guard<CCriticalSection> l(cs);
    return mapTx.size();
}
uint64_t CTxMemPool::GetTotalTxSize() const {
    std::lock_guard<CCriticalSection> l(cs);
    return totalTxSize;
}
size_t CTxMemPool::DynamicMemoryUsage() const {
    std::lock_guard<CCriticalSection> l(cs);
    // index nodes + entries + link sets (reference CTxMemPool::DynamicMemoryUsage)
    return memusage::DynamicUsage(mapTx) + mapTx.size() * memusage::MallocUsage(sizeof(CTxMemPoolEntry)) +
           memusage::MallocUsage(sizeof(memusage::stl_tree_node) + 2 * sizeof(void*)) * mapNextTx.size() +
           memusage::DynamicUsage(mapLinks) + cachedLinkUsage + memusage::DynamicUsage(mapDeltas) + cachedInnerUsage;
}
unsigned CTxMemPool::GetTransactionsUpdated() const {
    std::lock_guard<CCriticalSection> l(cs);
    return nTransactionsUpdated;
}
void CTxMemPool::AddTransactionsUpdated(unsigned n) {
    std::lock_guard<CCriticalSection> l(cs);
    nTransactionsUpdated += n;
}

void CTxMemPool::check(const CCoinsViewCache* pcoins, int spendHeight) const {
    if (nCheckFrequency == 0) return;
    if (GetRandInt(1 << 30) >= (int)(nCheckFrequency >> 2)) return;
    std::lock_guard<CCriticalSection> l(cs);
    uint64_t checkTotal = 0;
    CCoinsViewCache mempoolDuplicate(const_cast<CCoinsViewCache*>(pcoins));
    for (const auto& kv : mapTx) {
        const CTxMemPoolEntry& e = *kv.second;
        checkTotal += e.GetTxSize();
        const CTransaction& tx = e.GetTx();
        for (const CTxIn& in : tx.vin) {
            auto it2 = mapTx.find(in.prevout.hash);
            if (it2 != mapTx.end()) {
                if (in.prevout.n >= it2->second->GetTx().vout.size()) throw std::logic_error("mempool: bad parent output");
            } else if (!pcoins->HaveCoin(in.prevout)) {
                throw std::logic_error("mempool: input missing");
            }
            auto nx = mapNextTx.find(in.prevout);
            if (nx == mapNextTx.end() || nx->second != &tx) throw std::logic_error("mempool: mapNextTx inconsistent");
        }
        // ancestor aggregates must match a fresh computation
        setEntries setAncestors;
        std::string dummy;
        const uint64_t nNoLimit = std::numeric_limits<uint64_t>::max();
        CalculateMemPoolAncestors(e, setAncestors, nNoLimit, nNoLimit, nNoLimit, nNoLimit, dummy);
        uint64_t size = e.GetTxSize();
        Amount fees = e.GetModifiedFee();
        for (auto a : setAncestors) {
            size += a->second->GetTxSize();
            fees += a->second->GetModifiedFee();
        }
        if (e.GetCountWithAncestors() != setAncestors.size() + 1 || e.GetSizeWithAncestors() != size ||
            e.GetModFeesWithAncestors() != fees)
            throw std::logic_error("mempool: ancestor state inconsistent for " + kv.first.ToString());
    }
    (void)spendHeight;
    if (checkTotal != totalTxSize) throw std::logic_error("mempool: total size mismatch");
    size_t links = 0;
    for (const auto& lk : mapLinks) links += memusage::DynamicUsage(lk.second.parents) + memusage::DynamicUsage(lk.second.children);
    if (links != cachedLinkUsage) throw std::logic_error("mempool: link usage accounting mismatch");
}

// ------------------------------------------------------------------ coins view
bool CCoinsViewMemPool::GetCoin(const COutPoint& outpoint, Coin& coin) const {
    CTransactionRef ptx = mempool.get(outpoint.hash);
    if (ptx) {
        if (outpoint.n < ptx->vout.size()) {
            coin = Coin(ptx->vout[outpoint.n], MEMPOOL_HEIGHT, false);
            return true;
        }
        return false;
    }
    return base->GetCoin(outpoint, coin) && !coin.IsSpent();
}
bool CCoinsViewMemPool::HaveCoin(const COutPoint& outpoint) const {
    CTransactionRef ptx = mempool.get(outpoint.hash);
    if (ptx) return outpoint.n < ptx->vout.size();
    return base->HaveCoin(outpoint);
}

// ------------------------------------------------------------------ fee estimator
// Reference policy/fees.cpp: per-bucket exponentially decayed (0.998/block) counts of how many
// blocks transactions took to confirm; an estimate for a target is the lowest bucket group
// (scanning from the top, grouping until enough data) whose in-target confirmation rate is
// >= 95%. Fee rates bucket from 1000 to 1e7 sat/kB, priorities from 1e6 to 1e16, 1.1x / 2x apart.
static const double MIN_FEE_BUCKET = 1000, MAX_FEE_BUCKET = 1e7, FEE_SPACING = 1.1;
static const double MIN_PRI_BUCKET = 1e6, MAX_PRI_BUCKET = 1e16, PRI_SPACING = 2;
static const double DECAY = 0.998, MIN_SUCCESS = 0.95, SUFFICIENT_TXS = 1.0;
static const uint32_t FEE_ESTIMATES_VERSION = 170001;

void CBlockPolicyEstimator::Stats::Init(double lo, double hi, double spacing) {
    buckets.clear();
    for (double b = lo; b <= hi; b *= spacing) buckets.push_back(b);
    buckets.push_back(1e99);
    confAvg.assign(MAX_TARGET + 1, std::vector<double>(buckets.size(), 0.0));
    txAvg.assign(buckets.size(), 0.0);
}
int CBlockPolicyEstimator::Stats::BucketFor(double v) const {
    const int b = (int)(std::lower_bound(buckets.begin(), buckets.end(), v) - buckets.begin());
    return std::min(b, (int)buckets.size() - 1);
}
void CBlockPolicyEstimator::Stats::Decay(double d) {
    for (auto& row : confAvg)
        for (double& x : row) x *= d;
    for (double& x : txAvg) x *= d;
}
void CBlockPolicyEstimator::Stats::Record(int blocks, int bucket) {
    for (int t = std::max(1, blocks); t <= MAX_TARGET; t++) confAvg[t][bucket] += 1;
    txAvg[bucket] += 1;
}
double CBlockPolicyEstimator::Stats::Estimate(int confTarget, double minValue) const {
    if (confTarget < 1 || confTarget > MAX_TARGET) return -1;
    double nConf = 0, nTotal = 0;
    int best = -1;
    for (int b = (int)buckets.size() - 1; b >= 0; b--) {
        nConf += confAvg[confTarget][b];
        nTotal += txAvg[b];
        if (nTotal >= SUFFICIENT_TXS) {
            if (nConf / nTotal >= MIN_SUCCESS) best = b;
            else break;
            nConf = nTotal = 0;
        }
    }
    if (best < 0) return -1;
    const double v = best < (int)buckets.size() - 1 ? buckets[best] : buckets[buckets.size() - 2];
    return std::max(v, minValue);
}

CBlockPolicyEstimator::CBlockPolicyEstimator() {
    feeStats.Init(MIN_FEE_BUCKET, MAX_FEE_BUCKET, FEE_SPACING);
    priStats.Init(MIN_PRI_BUCKET, MAX_PRI_BUCKET, PRI_SPACING);
}
void CBlockPolicyEstimator::processTransaction(const uint256& txid, const CFeeRate& rate, unsigned height,
                                               bool valid, double priority) {
    if (!valid) return;
    std::lock_guard<std::mutex> l(cs);
    // fee payers are tracked by fee rate; zero-fee txs with a meaningful priority by priority
    if (rate.GetFeePerK() > 0) mapTracked[txid] = Tracked{height, feeStats.BucketFor((double)rate.GetFeePerK()), false};
    else if (priority >= MIN_PRI_BUCKET) mapTracked[txid] = Tracked{height, priStats.BucketFor(priority), true};
}
void CBlockPolicyEstimator::removeTx(const uint256& txid) {
    std::lock_guard<std::mutex> l(cs);
    mapTracked.erase(txid);
}
void CBlockPolicyEstimator::processBlock(unsigned height, const std::vector<uint256>& confirmed) {
    std::lock_guard<std::mutex> l(cs);
    if (height <= bestHeight) return;
    bestHeight = height;
    feeStats.Decay(DECAY);
    priStats.Decay(DECAY);
    for (const uint256& h : confirmed) {
        auto it = mapTracked.find(h);
        if (it == mapTracked.end()) continue;
        const int blocks = std::max(1, (int)height - (int)it->second.height);
        (it->second.priority ? priStats : feeStats).Record(blocks, it->second.bucket);
        mapTracked.erase(it);
    }
}
CFeeRate CBlockPolicyEstimator::estimateFee(int confTarget) const {
    std::lock_guard<std::mutex> l(cs);
    const double v = feeStats.Estimate(confTarget, 0);
    return CFeeRate(v < 0 ? 0 : (Amount)v);
}
CFeeRate CBlockPolicyEstimator::estimateSmartFee(int confTarget, int* answerFoundAtTarget) const {
    for (int t = std::max(1, confTarget); t <= MAX_TARGET; t++) {
        CFeeRate r = estimateFee(t);
        if (r.GetFeePerK() > 0) {
            if (answerFoundAtTarget) *answerFoundAtTarget = t;
            return r;
        }
    }
    if (answerFoundAtTarget) *answerFoundAtTarget = MAX_TARGET;
    return CFeeRate(0);
}
double CBlockPolicyEstimator::estimatePriority(int confTarget) const {
    std::lock_guard<std::mutex> l(cs);
    return priStats.Estimate(confTarget, 0);
}
double CBlockPolicyEstimator::estimateSmartPriority(int confTarget, int* answerFoundAtTarget) const {
    for (int t = std::max(1, confTarget); t <= MAX_TARGET; t++) {
        const double p = estimatePriority(t);
        if (p >= 0) {
            if (answerFoundAtTarget) *answerFoundAtTarget = t;
            return p;
        }
    }
    if (answerFoundAtTarget) *answerFoundAtTarget = MAX_TARGET;
    return -1;
}

bool CBlockPolicyEstimator::Write(const std::string& path) const {
    std::vector<unsigned char> out;
    {
        std::lock_guard<std::mutex> l(cs);
        VectorWriter w(out, SER_DISK, PROTOCOL_VERSION);
        auto wd = [&](double x) { // doubles as their IEEE-754 bit patterns
            uint64_t u;
            memcpy(&u, &x, 8);
            w << u;
        };
        w << FEE_ESTIMATES_VERSION << bestHeight;
        for (const Stats* st : {&feeStats, &priStats}) {
            w << (uint64_t)st->buckets.size();
            for (double b : st->buckets) wd(b);
            for (const auto& row : st->confAvg)
                for (double x : row) wd(x);
            for (double x : st->txAvg) wd(x);
        }
    }
    const std::string tmp = path + ".new";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const bool ok = fwrite(out.data(), 1, out.size(), f) == out.size();
    fclose(f);
    return ok && rename(tmp.c_str(), path.c_str()) == 0;
}

bool CBlockPolicyEstimator::Read(const std::string& path) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<unsigned char> data;
    unsigned char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) data.insert(data.end(), buf, buf + n);
    fclose(f);
    try {
        SpanReader r(data.data(), data.size(), SER_DISK, PROTOCOL_VERSION);
        auto rd = [&](double& x) {
            uint64_t u;
            r >> u;
            memcpy(&x, &u, 8);
        };
        uint32_t version;
        unsigned height;
        r >> version >> height;
        if (version != FEE_ESTIMATES_VERSION) return false;
        Stats loaded[2];
        for (Stats& st : loaded) {
            uint64_t nb;
            r >> nb;
            if (nb == 0 || nb > 1000) throw std::runtime_error("bad bucket count");
            st.buckets.resize(nb);
            for (double& b : st.buckets) rd(b);
            st.confAvg.assign(MAX_TARGET + 1, std::vector<double>(nb));
            for (auto& row : st.confAvg)
                for (double& x : row) rd(x);
            st.txAvg.resize(nb);
            for (double& x : st.txAvg) rd(x);
        }
        std::lock_guard<std::mutex> l(cs);
        feeStats = loaded[0];
        priStats = loaded[1];
        bestHeight = height;
    } catch (const std::exception& e) {
        LogPrintf("CBlockPolicyEstimator::Read(): unable to read policy estimator data (non-fatal): %s\n", e.what());
        return false;
    }
    return true;
}

FeeFilterRounder::FeeFilterRounder(const CFeeRate& minIncrementalFee) {
    const double minFeeLimit = std::max((double)1, (double)minIncrementalFee.GetFeePerK() / 2);
    feeset.insert(0);
    for (double b = minFeeLimit; b <= MAX_FEE_BUCKET; b *= FEE_SPACING) feeset.insert(b);
}
Amount FeeFilterRounder::round(Amount currentMinFee) {
    auto it = feeset.lower_bound((double)currentMinFee);
    if ((it != feeset.begin() && GetRand(3) != 0) || it == feeset.end()) --it;
    return (Amount)*it;
}

} // namespace bcp
