// Transaction memory pool.
// Parity: reference src/txmempool.{h,cpp}: CTxMemPoolEntry (fee, size, time, height,
// priority, sigops, lock points, ancestor/descendant aggregates incl. modified fees),
// indices by txid / descendant score / entry time / ancestor score, mapNextTx,
// CalculateMemPoolAncestors with -limitancestor*/-limitdescendant*, addUnchecked,
// removeRecursive/removeForReorg/removeConflicts/removeForBlock, Expire, TrimToSize
// with the rolling minimum fee (halflife 12 h), PrioritiseTransaction/ApplyDeltas,
// CCoinsViewMemPool, check(), and reference src/policy/fees.cpp fee estimation
// (simplified bucketed confirmation-time estimator).
#pragma once
#include "node/coins.h"
#include "primitives/amount.h"
#include "primitives/transaction.h"
#include "util/sync.h"

#include "util/indirectmap.h"

#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <unordered_map>
#include <vector>

namespace bcp {

class CBlockIndex;
static const uint32_t MEMPOOL_HEIGHT = 0x7FFFFFFF;

struct LockPoints {
    int height = 0;
    int64_t time = 0;
    const CBlockIndex* maxInputBlock = nullptr;
};

class CTxMemPoolEntry {
public:
    CTxMemPoolEntry(const CTransactionRef& tx, Amount fee, int64_t time, double entryPriority, unsigned entryHeight,
                    Amount inChainInputValue, bool spendsCoinbase, int64_t sigOpCount, LockPoints lp);
    const CTransaction& GetTx() const { return *tx; }
    CTransactionRef GetSharedTx() const { return tx; }
    Amount GetFee() const { return nFee; }
    size_t GetTxSize() const { return nTxSize; }
    int64_t GetTime() const { return nTime; }
    unsigned GetHeight() const { return entryHeight; }
    int64_t GetSigOpCount() const { return sigOpCount; }
    Amount GetModifiedFee() const { return nFee + feeDelta; }
    size_t DynamicMemoryUsage() const { return nUsageSize; }
    const LockPoints& GetLockPoints() const { return lockPoints; }
    bool GetSpendsCoinbase() const { return spendsCoinbase; }
    double GetPriority(unsigned currentHeight) const;

    uint64_t GetCountWithDescendants() const { return nCountWithDescendants; }
    uint64_t GetSizeWithDescendants() const { return nSizeWithDescendants; }
    Amount GetModFeesWithDescendants() const { return nModFeesWithDescendants; }
    uint64_t GetCountWithAncestors() const { return nCountWithAncestors; }
    uint64_t GetSizeWithAncestors() const { return nSizeWithAncestors; }
    Amount GetModFeesWithAncestors() const { return nModFeesWithAncestors; }
    int64_t GetSigOpCountWithAncestors() const { return nSigOpCountWithAncestors; }

    mutable size_t vTxHashesIdx = 0;

private:
    friend class CTxMemPool;
    CTransactionRef tx;
    Amount nFee;
    size_t nTxSize, nModSize, nUsageSize;
    int64_t nTime;
    double entryPriority;
    unsigned entryHeight;
    Amount inChainInputValue;
    bool spendsCoinbase;
    int64_t sigOpCount;
    Amount feeDelta = 0;
    LockPoints lockPoints;
    uint64_t nCountWithDescendants = 1, nSizeWithDescendants;
    Amount nModFeesWithDescendants;
    uint64_t nCountWithAncestors = 1, nSizeWithAncestors;
    Amount nModFeesWithAncestors;
    int64_t nSigOpCountWithAncestors;
};

enum class MemPoolRemovalReason { UNKNOWN, EXPIRY, SIZELIMIT, REORG, BLOCK, CONFLICT, REPLACED };

struct TxMempoolInfo {
    CTransactionRef tx;
    int64_t nTime = 0;
    CFeeRate feeRate;
    Amount nFeeDelta = 0;
};

// Simplified fee estimator: per-feerate-bucket exponentially decayed confirmation stats.
class CBlockPolicyEstimator {
public:
    CBlockPolicyEstimator();
    // priority < 0: not tracked for priority (reference fees.h priStats; free txs with
    // priority are tracked there, fee payers in feeStats)
    void processTransaction(const uint256& txid, const CFeeRate& rate, unsigned height, bool validForEstimation,
                            double priority = -1);
    void processBlock(unsigned height, const std::vector<uint256>& confirmedTxids);
    void removeTx(const uint256& txid);
    CFeeRate estimateFee(int confTarget) const;
    CFeeRate estimateSmartFee(int confTarget, int* answerFoundAtTarget) const;
    double estimatePriority(int confTarget) const;
    double estimateSmartPriority(int confTarget, int* answerFoundAtTarget) const;
    // fee_estimates.dat (reference CBlockPolicyEstimator::Write/Read, txmempool.cpp:954-990)
    bool Write(const std::string& path) const;
    bool Read(const std::string& path);

private:
    // One decayed confirmation table over value buckets (fee rate in sat/kB, or priority).
    struct Stats {
        std::vector<double> buckets;              // upper bucket bounds
        std::vector<std::vector<double>> confAvg; // [target][bucket] decayed confirmed counts
        std::vector<double> txAvg;                // [bucket] decayed totals
        void Init(double lo, double hi, double spacing);
        int BucketFor(double v) const;
        void Decay(double d);
        void Record(int blocks, int bucket);
        double Estimate(int confTarget, double minValue) const;
    };
    struct Tracked {
        unsigned height;
        int bucket;
        bool priority; // tracked in priStats instead of feeStats
    };
    Stats feeStats, priStats;
    std::map<uint256, Tracked> mapTracked;
    unsigned bestHeight = 0;
    static const int MAX_TARGET = 25;
    mutable std::mutex cs;
};

// Rounds the fee filter we announce to peers to a coarse, randomized bucket so the exact
// mempool minimum fee does not fingerprint the node (reference policy/fees.h FeeFilterRounder).
class FeeFilterRounder {
public:
    explicit FeeFilterRounder(const CFeeRate& minIncrementalFee);
    Amount round(Amount currentMinFee);

private:
    std::set<double> feeset;
};

class CTxMemPool {
public:
    typedef std::map<uint256, std::unique_ptr<CTxMemPoolEntry>>::iterator txiter;
    struct IterCmp {
        bool operator()(const txiter& a, const txiter& b) const { return a->first < b->first; }
    };
    typedef std::set<txiter, IterCmp> setEntries;

    explicit CTxMemPool(CBlockPolicyEstimator* estimator = nullptr);
    mutable CCriticalSection cs{"mempool.cs"};

    void addUnchecked(const uint256& hash, const CTxMemPoolEntry& entry, setEntries& setAncestors,
                      bool validFeeEstimate = true);
    void addUnchecked(const uint256& hash, const CTxMemPoolEntry& entry, bool validFeeEstimate = true);
    bool CalculateMemPoolAncestors(const CTxMemPoolEntry& entry, setEntries& setAncestors, uint64_t limitAncestorCount,
                                   uint64_t limitAncestorSize, uint64_t limitDescendantCount,
                                   uint64_t limitDescendantSize, std::string& errString,
                                   bool fSearchForParents = true) const EXCLUSIVE_LOCKS_REQUIRED(cs);
    void CalculateDescendants(txiter it, setEntries& setDescendants) EXCLUSIVE_LOCKS_REQUIRED(cs);

    void removeRecursive(const CTransaction& tx, MemPoolRemovalReason reason = MemPoolRemovalReason::UNKNOWN);
    void removeForReorg(const CCoinsViewCache* pcoins, unsigned nMemPoolHeight, int flags,
                        const std::function<bool(const CTransaction&, LockPoints&, bool)>& checkLocks,
                        const std::function<bool(const LockPoints*)>& lpValid);
    void removeConflicts(const CTransaction& tx);
    void removeForBlock(const std::vector<CTransactionRef>& vtx, unsigned nBlockHeight);
    void RemoveStaged(setEntries& stage, bool updateDescendants, MemPoolRemovalReason reason);
    void clear();
    int Expire(int64_t time);
    void TrimToSize(size_t sizelimit, std::vector<COutPoint>* pvNoSpendsRemaining = nullptr);
    CFeeRate GetMinFee(size_t sizelimit) const;
    void UpdateTransactionsFromBlock(const std::vector<uint256>& hashesToUpdate);

    void PrioritiseTransaction(const uint256& hash, double dPriorityDelta, Amount nFeeDelta);
    void ApplyDeltas(const uint256& hash, double& dPriorityDelta, Amount& nFeeDelta) const;
    void ClearPrioritisation(const uint256& hash);
    std::map<uint256, std::pair<double, Amount>> GetDeltas() const;

    bool exists(const uint256& hash) const;
    // true unless the transaction is in the pool with chainLimit or more ancestors or
    // descendants (reference txmempool.cpp TransactionWithinChainLimit)
    bool TransactionWithinChainLimit(const uint256& txid, size_t chainLimit) const;
    CTransactionRef get(const uint256& hash) const;
    const CTxMemPoolEntry* GetEntry(const uint256& hash) const;
    TxMempoolInfo info(const uint256& hash) const;
    std::vector<TxMempoolInfo> infoAll() const;
    void queryHashes(std::vector<uint256>& vtxid) const;
    bool HasNoInputsOf(const CTransaction& tx) const;
    bool isSpent(const COutPoint& outpoint) const;
    const CTransaction* GetConflictTx(const COutPoint& prevout) const;
    std::vector<const CTxMemPoolEntry*> GetAncestors(const uint256& hash) const;
    std::vector<const CTxMemPoolEntry*> GetDescendants(const uint256& hash) const;
    // entries sorted by ancestor score (mining order) / descendant score (eviction order)
    std::vector<txiter> SortedByAncestorScore();
    std::vector<const CTxMemPoolEntry*> SortedByDepthAndScore() const;
    std::vector<CTransactionRef> AllTransactions() const;
    void CompactParents(txiter it, setEntries& out) const EXCLUSIVE_LOCKS_REQUIRED(cs);
    const setEntries& GetMemPoolParents(txiter it) const EXCLUSIVE_LOCKS_REQUIRED(cs);
    const setEntries& GetMemPoolChildren(txiter it) const EXCLUSIVE_LOCKS_REQUIRED(cs);
    txiter MapTxEnd() EXCLUSIVE_LOCKS_REQUIRED(cs) { return mapTx.end(); }
    txiter Find(const uint256& h) EXCLUSIVE_LOCKS_REQUIRED(cs) { return mapTx.find(h); }

    unsigned long size() const;
    uint64_t GetTotalTxSize() const;
    size_t DynamicMemoryUsage() const;
    unsigned GetTransactionsUpdated() const;
    void AddTransactionsUpdated(unsigned n);
    void check(const CCoinsViewCache* pcoins, int spendHeight) const;
    void setSanityCheck(double dFrequency) { nCheckFrequency = (uint32_t)(dFrequency * 4294967295.0); }
    CBlockPolicyEstimator* Estimator() { return minerPolicyEstimator; }

    indirectmap<COutPoint, const CTransaction*> mapNextTx GUARDED_BY(cs); // keys point into the spending txs

private:
    // mapTx for const members that hand out (mutable) iterators
    std::map<uint256, std::unique_ptr<CTxMemPoolEntry>>& TxMap() const EXCLUSIVE_LOCKS_REQUIRED(cs) {
        return const_cast<CTxMemPool*>(this)->mapTx;
    }
    struct Links {
        setEntries parents, children;
    };
    void UpdateParent(txiter entry, txiter parent, bool add) EXCLUSIVE_LOCKS_REQUIRED(cs);
    void UpdateChild(txiter entry, txiter child, bool add) EXCLUSIVE_LOCKS_REQUIRED(cs);
    void UpdateAncestorsOf(bool add, txiter it, setEntries& setAncestors) EXCLUSIVE_LOCKS_REQUIRED(cs);
    void UpdateEntryForAncestors(txiter it, const setEntries& setAncestors) EXCLUSIVE_LOCKS_REQUIRED(cs);
    void UpdateForRemoveFromMempool(const setEntries& entriesToRemove, bool updateDescendants) EXCLUSIVE_LOCKS_REQUIRED(cs);
    void UpdateForDescendants(txiter updateIt, std::map<txiter, setEntries, IterCmp>& cachedDescendants,
                              const std::set<uint256>& setExclude) EXCLUSIVE_LOCKS_REQUIRED(cs);
    void removeUnchecked(txiter entry, MemPoolRemovalReason reason) EXCLUSIVE_LOCKS_REQUIRED(cs);
    void trackPackageRemoved(const CFeeRate& rate) EXCLUSIVE_LOCKS_REQUIRED(cs);

    std::map<uint256, std::unique_ptr<CTxMemPoolEntry>> mapTx GUARDED_BY(cs);
    std::map<txiter, Links, IterCmp> mapLinks GUARDED_BY(cs);
    std::map<uint256, std::pair<double, Amount>> mapDeltas GUARDED_BY(cs);
    uint64_t totalTxSize GUARDED_BY(cs) = 0;
    uint64_t cachedInnerUsage GUARDED_BY(cs) = 0;
    uint64_t cachedLinkUsage GUARDED_BY(cs) = 0; // parents/children set nodes
    unsigned nTransactionsUpdated GUARDED_BY(cs) = 0;
    uint32_t nCheckFrequency = 0;
    mutable int64_t lastRollingFeeUpdate GUARDED_BY(cs) = 0;
    mutable bool blockSinceLastRollingFeeBump GUARDED_BY(cs) = false;
    mutable double rollingMinimumFeeRate GUARDED_BY(cs) = 0;
    CBlockPolicyEstimator* minerPolicyEstimator;
    static const int ROLLING_FEE_HALFLIFE = 60 * 60 * 12;
};

// Coins view that also sees mempool outputs (height MEMPOOL_HEIGHT).
class CCoinsViewMemPool : public CCoinsViewBacked {
public:
    CCoinsViewMemPool(CCoinsView* base, const CTxMemPool& pool) : CCoinsViewBacked(base), mempool(pool) {}
    bool GetCoin(const COutPoint& outpoint, Coin& coin) const override;
    bool HaveCoin(const COutPoint& outpoint) const override;

private:
    const CTxMemPool& mempool;
};

} // namespace bcp
