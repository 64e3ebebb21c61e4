// Mempool acceptance and persistence.
// Parity: reference src/validation.cpp AcceptToMemoryPoolWorker :666-995 (standardness,
// conflicts, missing inputs, BIP68, sigops, min-fee/priority/free-rate limits, absurd
// fee, ancestor limits, STANDARD then MANDATORY flag script checks, size limiting),
// CheckSequenceLocks :366, TestLockPointValidity :347, LimitMempoolSize :572,
// LoadMempool/DumpMempool :4948-5070 (mempool.dat v1: count, (tx, time, feedelta)*, deltas).
#include "node/policy.h"
#include "node/signals.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "script/interpreter.h"
#include "util/strencodings.h"

#include <cmath>

namespace bcp {

static const uint8_t REJECT_HIGHFEE = 0x100 & 0xff; // internal codes (not sent on the wire)
static const unsigned REJECT_ALREADY_KNOWN_CODE = 0x101;
static const unsigned REJECT_CONFLICT_CODE = 0x102;

bool Chainstate::TestLockPointValidity(const LockPoints* lp) const {
    if (lp->maxInputBlock && !chainActive.Contains(lp->maxInputBlock)) return false;
    return true;
}

bool Chainstate::CheckSequenceLocks(const CTransaction& tx, int flags, LockPoints* lp, bool useExistingLockPoints) {
    CBlockIndex* tip = chainActive.Tip();
    CBlockIndex index;
    index.pprev = tip;
    index.nHeight = tip->nHeight + 1;
    std::pair<int, int64_t> lockPair;
    if (useExistingLockPoints) {
        lockPair.first = lp->height;
        lockPair.second = lp->time;
    } else {
        CCoinsViewMemPool viewMemPool(pcoinsTip.get(), *mempool);
        std::vector<int> prevheights(tx.vin.size());
        for (size_t i = 0; i < tx.vin.size(); i++) {
            Coin coin;
            if (!viewMemPool.GetCoin(tx.vin[i].prevout, coin)) return error("%s: Missing input", __func__);
            prevheights[i] = coin.GetHeight() == MEMPOOL_HEIGHT ? tip->nHeight + 1 : (int)coin.GetHeight();
        }
        lockPair = CalculateSequenceLocks(tx, flags, &prevheights, index);
        if (lp) {
            lp->height = lockPair.first;
            lp->time = lockPair.second;
            int maxInputHeight = 0;
            for (int h : prevheights)
                if (h != tip->nHeight + 1) maxInputHeight = std::max(maxInputHeight, h);
            lp->maxInputBlock = tip->GetAncestor(maxInputHeight);
        }
    }
    return EvaluateSequenceLocks(index, lockPair);
}

void Chainstate::LimitMempoolSize(size_t limit, unsigned long age) {
    if (!mempool) return;
    const int expired = mempool->Expire(GetTime() - (int64_t)age);
    if (expired != 0) LogPrint(BCLog::MEMPOOL, "Expired %i transactions from the memory pool\n", expired);
    std::vector<COutPoint> vNoSpendsRemaining;
    mempool->TrimToSize(limit, &vNoSpendsRemaining);
    for (const COutPoint& removed : vNoSpendsRemaining) pcoinsTip->Uncache(removed);
}

bool Chainstate::AcceptToMemoryPoolWorker(CValidationState& state, const CTransactionRef& ptx, bool fLimitFree,
                                          bool* pfMissingInputs, int64_t nAcceptTime, bool fOverrideMempoolLimit,
                                          Amount nAbsurdFee, std::vector<COutPoint>& coins_to_uncache, Amount* feeOut) {
    const CTransaction& tx = *ptx;
    const uint256 txid = tx.GetHash();
    if (pfMissingInputs) *pfMissingInputs = false;
    if (!CheckRegularTransaction(tx, state, true)) return false;
    std::string reason;
    if (fRequireStandard && !IsStandardTx(tx, reason)) return state.DoS(0, false, REJECT_NONSTANDARD, reason);
    CValidationState ctxState;
    if (!ContextualCheckTransactionForCurrentBlock(tx, ctxState, STANDARD_LOCKTIME_VERIFY_FLAGS))
        return state.DoS(0, false, REJECT_NONSTANDARD, ctxState.GetRejectReason(), ctxState.CorruptionPossible(),
                         ctxState.GetDebugMessage());
    if (mempool->exists(txid)) return state.Invalid(false, REJECT_ALREADY_KNOWN_CODE, "txn-already-in-mempool");
    {
        std::lock_guard<CCriticalSection> lp(mempool->cs);
        for (const CTxIn& in : tx.vin)
            if (mempool->mapNextTx.count(in.prevout))
                return state.Invalid(false, REJECT_CONFLICT_CODE, "txn-mempool-conflict");
    }
    CCoinsView dummy;
    CCoinsViewCache view(&dummy);
    Amount nValueIn = 0;
    LockPoints lp;
    {
        std::lock_guard<CCriticalSection> lpool(mempool->cs);
        CCoinsViewMemPool viewMemPool(pcoinsTip.get(), *mempool);
        view.SetBackend(viewMemPool);
        for (size_t out = 0; out < tx.vout.size(); out++) {
            COutPoint outpoint(txid, (uint32_t)out);
            const bool had = pcoinsTip->HaveCoinInCache(outpoint);
            if (view.HaveCoin(outpoint)) {
                if (!had) coins_to_uncache.push_back(outpoint);
                return state.Invalid(false, REJECT_ALREADY_KNOWN_CODE, "txn-already-known");
            }
        }
        for (const CTxIn& in : tx.vin) {
            if (!pcoinsTip->HaveCoinInCache(in.prevout)) coins_to_uncache.push_back(in.prevout);
            if (!view.HaveCoin(in.prevout)) {
                if (pfMissingInputs) *pfMissingInputs = true;
                return false;
            }
        }
        if (!view.HaveInputs(tx)) return state.Invalid(false, REJECT_DUPLICATE, "bad-txns-inputs-spent");
        view.GetBestBlock();
        nValueIn = view.GetValueIn(tx);
        view.SetBackend(dummy);
        if (!CheckSequenceLocks(tx, STANDARD_LOCKTIME_VERIFY_FLAGS, &lp))
            return state.DoS(0, false, REJECT_NONSTANDARD, "non-BIP68-final");
    }
    if (fRequireStandard && !AreInputsStandard(tx, view))
        return state.Invalid(false, REJECT_NONSTANDARD, "bad-txns-nonstandard-inputs");
    const int64_t nSigOpsCount = (int64_t)GetTransactionSigOpCount(tx, view, STANDARD_SCRIPT_VERIFY_FLAGS);
    const Amount nValueOut = tx.GetValueOut();
    const Amount nFees = nValueIn - nValueOut;
    Amount nModifiedFees = nFees;
    double nPriorityDummy = 0;
    mempool->ApplyDeltas(txid, nPriorityDummy, nModifiedFees);
    Amount inChainInputValue = 0;
    const double dPriority = GetPriority(tx, view, chainActive.Height(), inChainInputValue);
    bool fSpendsCoinbase = false;
    for (const CTxIn& in : tx.vin)
        if (view.AccessCoin(in.prevout).IsCoinBase()) {
            fSpendsCoinbase = true;
            break;
        }
    CTxMemPoolEntry entry(ptx, nFees, nAcceptTime, dPriority, (unsigned)chainActive.Height(), inChainInputValue,
                          fSpendsCoinbase, nSigOpsCount, lp);
    const unsigned nSize = (unsigned)entry.GetTxSize();
    if (nSigOpsCount > (int64_t)MAX_STANDARD_TX_SIGOPS)
        return state.DoS(0, false, REJECT_NONSTANDARD, "bad-txns-too-many-sigops", false,
                         strprintf("%lld", (long long)nSigOpsCount));
    const size_t maxMempool = (size_t)gArgs.GetArg("-maxmempool", (int64_t)DEFAULT_MAX_MEMPOOL_SIZE) * 1000000;
    const Amount mempoolRejectFee = mempool->GetMinFee(maxMempool).GetFee(nSize);
    if (mempoolRejectFee > 0 && nModifiedFees < mempoolRejectFee)
        return state.DoS(0, false, REJECT_INSUFFICIENTFEE, "mempool min fee not met", false,
                         strprintf("%lld < %lld", (long long)nFees, (long long)mempoolRejectFee));
    if (gArgs.GetBoolArg("-relaypriority", DEFAULT_RELAYPRIORITY) && nModifiedFees < minRelayTxFee.GetFee(nSize) &&
        !AllowFree(entry.GetPriority(chainActive.Height() + 1)))
        return state.DoS(0, false, REJECT_INSUFFICIENTFEE, "insufficient priority");
    if (fLimitFree && nModifiedFees < minRelayTxFee.GetFee(nSize)) {
        // continuously rate-limit free (really, very-low-fee) transactions
        static std::mutex csFreeLimiter;
        static double dFreeCount = 0;
        static int64_t nLastTime = 0;
        const int64_t nNow = GetTime();
        std::lock_guard<std::mutex> fl(csFreeLimiter);
        dFreeCount *= std::pow(1.0 - 1.0 / 600.0, (double)(nNow - nLastTime));
        nLastTime = nNow;
        if (dFreeCount + nSize >= gArgs.GetArg("-limitfreerelay", (int64_t)DEFAULT_LIMITFREERELAY) * 10 * 1000)
            return state.DoS(0, false, REJECT_INSUFFICIENTFEE, "rate limited free transaction");
        dFreeCount += nSize;
    }
    if (nAbsurdFee != 0 && nFees > nAbsurdFee)
        return state.Invalid(false, REJECT_HIGHFEE, "absurdly-high-fee",
                             strprintf("%lld > %lld", (long long)nFees, (long long)nAbsurdFee));
    CTxMemPool::setEntries setAncestors;
    const size_t nLimitAncestors = (size_t)gArgs.GetArg("-limitancestorcount", (int64_t)DEFAULT_ANCESTOR_LIMIT);
    const size_t nLimitAncestorSize = (size_t)gArgs.GetArg("-limitancestorsize", (int64_t)DEFAULT_ANCESTOR_SIZE_LIMIT) * 1000;
    const size_t nLimitDescendants = (size_t)gArgs.GetArg("-limitdescendantcount", (int64_t)DEFAULT_DESCENDANT_LIMIT);
    const size_t nLimitDescendantSize =
        (size_t)gArgs.GetArg("-limitdescendantsize", (int64_t)DEFAULT_DESCENDANT_SIZE_LIMIT) * 1000;
    std::string errString;
    {
        std::lock_guard<CCriticalSection> lpool(mempool->cs); // the walk reads mapTx / mapLinks
        if (!mempool->CalculateMemPoolAncestors(entry, setAncestors, nLimitAncestors, nLimitAncestorSize,
                                                nLimitDescendants, nLimitDescendantSize, errString))
            return state.DoS(0, false, REJECT_NONSTANDARD, "too-long-mempool-chain", false, errString);
    }
    uint32_t scriptVerifyFlags = STANDARD_SCRIPT_VERIFY_FLAGS;
    if (!params.RequireStandard())
        scriptVerifyFlags = (uint32_t)gArgs.GetArg("-promiscuousmempoolflags", (int64_t)scriptVerifyFlags);
    PrecomputedTransactionData txdata(tx);
    if (!CheckInputs(tx, state, view, true, scriptVerifyFlags, true, txdata)) return false;
    // also check against the flags of the next block (populates the caches for ConnectBlock)
    const uint32_t currentBlockScriptVerifyFlags = GetBlockScriptFlags(chainActive.Tip());
    CValidationState st2;
    if (!CheckInputs(tx, st2, view, true, currentBlockScriptVerifyFlags, true, txdata)) {
        if (!CheckInputs(tx, state, view, true, MANDATORY_SCRIPT_VERIFY_FLAGS, true, txdata))
            return error("%s: ConnectInputs failed against MANDATORY but not STANDARD flags %s, %s", __func__,
                         txid.ToString().c_str(), FormatStateMessage(state).c_str());
    }
    const bool validForFeeEstimation = !IsInitialBlockDownload() && mempool->HasNoInputsOf(tx);
    mempool->addUnchecked(txid, entry, setAncestors, validForFeeEstimation);
    if (!fOverrideMempoolLimit) {
        LimitMempoolSize(maxMempool, (unsigned long)gArgs.GetArg("-mempoolexpiry", (int64_t)DEFAULT_MEMPOOL_EXPIRY) * 60 * 60);
        if (!mempool->exists(txid)) return state.DoS(0, false, REJECT_INSUFFICIENTFEE, "mempool full");
    }
    if (feeOut) *feeOut = nFees;
    GetMainSignals().TransactionAddedToMempool(ptx);
    return true;
}

bool Chainstate::AcceptToMemoryPool(CValidationState& state, const CTransactionRef& tx, bool fLimitFree,
                                    bool* pfMissingInputs, bool fOverrideMempoolLimit, Amount nAbsurdFee,
                                    int64_t nAcceptTime, Amount* feeOut) {
    if (!mempool) return state.Error("no mempool");
    std::lock_guard<CCriticalSection> l(cs_main);
    std::vector<COutPoint> coins_to_uncache;
    const bool res = AcceptToMemoryPoolWorker(state, tx, fLimitFree, pfMissingInputs, nAcceptTime ? nAcceptTime : GetTime(),
                                              fOverrideMempoolLimit, nAbsurdFee, coins_to_uncache, feeOut);
    if (!res)
        for (const COutPoint& o : coins_to_uncache) pcoinsTip->Uncache(o);
    CValidationState stateDummy;
    FlushStateToDisk(stateDummy, FLUSH_STATE_PERIODIC);
    return res;
}

void Chainstate::UpdateMempoolForReorg(const std::vector<CTransactionRef>& disconnected, bool fAddToMempool) {
    std::vector<uint256> vHashUpdate;
    for (const auto& ptx : disconnected) {
        CValidationState stateDummy;
        if (!fAddToMempool || ptx->IsCoinBase() ||
            !AcceptToMemoryPool(stateDummy, ptx, false, nullptr, true)) {
            mempool->removeRecursive(*ptx, MemPoolRemovalReason::REORG);
        } else if (mempool->exists(ptx->GetHash())) {
            vHashUpdate.push_back(ptx->GetHash());
        }
    }
    mempool->UpdateTransactionsFromBlock(vHashUpdate);
}

static const uint64_t MEMPOOL_DUMP_VERSION = 1;

bool Chainstate::LoadMempool(const std::string& path) {
    if (!mempool) return false;
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<unsigned char> data;
    unsigned char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) data.insert(data.end(), buf, buf + n);
    fclose(f);
    int64_t count = 0, failed = 0, skipped = 0;
    const int64_t nExpiryTimeout = gArgs.GetArg("-mempoolexpiry", (int64_t)DEFAULT_MEMPOOL_EXPIRY) * 60 * 60;
    try {
        SpanReader r(data.data(), data.size(), SER_DISK, PROTOCOL_VERSION);
        uint64_t version, num;
        r >> version;
        if (version != MEMPOOL_DUMP_VERSION) return false;
        r >> num;
        const int64_t nNow = GetTime();
        while (num--) {
            CMutableTransaction mtx;
            int64_t nTime, nFeeDelta;
            r >> mtx >> nTime >> nFeeDelta;
            CTransactionRef tx = MakeTransactionRef(std::move(mtx));
            if (nFeeDelta) mempool->PrioritiseTransaction(tx->GetHash(), 0, nFeeDelta);
            CValidationState state;
            if (nTime + nExpiryTimeout > nNow) {
                std::lock_guard<CCriticalSection> l(cs_main);
                std::vector<COutPoint> unc;
                if (AcceptToMemoryPoolWorker(state, tx, true, nullptr, nTime, false, 0, unc, nullptr)) count++;
                else failed++;
            } else {
                skipped++;
            }
        }
        std::map<uint256, int64_t> mapDeltas;
        r >> mapDeltas;
        for (const auto& d : mapDeltas) mempool->PrioritiseTransaction(d.first, 0, d.second);
    } catch (const std::exception& e) {
        LogPrintf("Failed to deserialize mempool data on disk: %s. Continuing anyway.\n", e.what());
        return false;
    }
    LogPrintf("Imported mempool transactions from disk: %lld successes, %lld failed, %lld expired\n", (long long)count,
              (long long)failed, (long long)skipped);
    return true;
}

bool Chainstate::DumpMempool(const std::string& path) {
    if (!mempool) return false;
    std::map<uint256, int64_t> mapDeltas;
    std::vector<TxMempoolInfo> vinfo;
    {
        std::lock_guard<CCriticalSection> l(mempool->cs);
        for (const auto& d : mempool->GetDeltas()) mapDeltas[d.first] = d.second.second;
        vinfo = mempool->infoAll();
    }
    std::vector<unsigned char> out;
    VectorWriter w(out, SER_DISK, PROTOCOL_VERSION);
    w << MEMPOOL_DUMP_VERSION << (uint64_t)vinfo.size();
    for (const auto& i : vinfo) {
        w << *i.tx << (int64_t)i.nTime << (int64_t)i.nFeeDelta;
        mapDeltas.erase(i.tx->GetHash());
    }
    w << mapDeltas;
    const std::string tmp = path + ".new";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const bool ok = fwrite(out.data(), 1, out.size(), f) == out.size() && FileCommit(f);
    fclose(f);
    if (!ok || !RenameOver(tmp, path)) return false;
    return true;
}

} // namespace bcp
