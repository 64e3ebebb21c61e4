#include "consensus/tx_verify.h"
#include "node/coins.h"
#include "script/interpreter.h"
#include "util/strencodings.h"

#include <algorithm>
#include <set>

namespace bcp {

bool IsFinalTx(const CTransaction& tx, int nBlockHeight, int64_t nBlockTime) {
    if (tx.nLockTime == 0) return true;
    const int64_t lockTime = tx.nLockTime;
    const int64_t limit = lockTime < LOCKTIME_THRESHOLD ? nBlockHeight : nBlockTime;
    if (lockTime < limit) return true;
    for (const auto& in : tx.vin)
        if (in.nSequence != CTxIn::SEQUENCE_FINAL) return false;
    return true;
}

std::pair<int, int64_t> CalculateSequenceLocks(const CTransaction& tx, int flags, std::vector<int>* prevHeights,
                                               const CBlockIndex& block) {
    int nMinHeight = -1;
    int64_t nMinTime = -1;
    const bool enforce = (uint32_t)tx.nVersion >= 2 && (flags & LOCKTIME_VERIFY_SEQUENCE);
    if (!enforce) return {nMinHeight, nMinTime};
    for (size_t i = 0; i < tx.vin.size(); i++) {
        const CTxIn& in = tx.vin[i];
        if (in.nSequence & CTxIn::SEQUENCE_LOCKTIME_DISABLE_FLAG) {
            (*prevHeights)[i] = 0; // does not constrain
            continue;
        }
        const int nCoinHeight = (*prevHeights)[i];
        if (in.nSequence & CTxIn::SEQUENCE_LOCKTIME_TYPE_FLAG) {
            const int64_t nCoinTime = block.GetAncestor(std::max(nCoinHeight - 1, 0))->GetMedianTimePast();
            nMinTime = std::max(nMinTime, nCoinTime +
                                              (int64_t)((in.nSequence & CTxIn::SEQUENCE_LOCKTIME_MASK)
                                                        << CTxIn::SEQUENCE_LOCKTIME_GRANULARITY) -
                                              1);
        } else {
            nMinHeight = std::max(nMinHeight, nCoinHeight + (int)(in.nSequence & CTxIn::SEQUENCE_LOCKTIME_MASK) - 1);
        }
    }
    return {nMinHeight, nMinTime};
}

bool EvaluateSequenceLocks(const CBlockIndex& block, std::pair<int, int64_t> lockPair) {
    const int64_t nBlockTime = block.pprev->GetMedianTimePast();
    return !(lockPair.first >= block.nHeight || lockPair.second >= nBlockTime);
}

bool SequenceLocks(const CTransaction& tx, int flags, std::vector<int>* prevHeights, const CBlockIndex& block) {
    return EvaluateSequenceLocks(block, CalculateSequenceLocks(tx, flags, prevHeights, block));
}

uint64_t GetSigOpCountWithoutP2SH(const CTransaction& tx) {
    uint64_t n = 0;
    for (const auto& in : tx.vin) n += in.scriptSig.GetSigOpCount(false);
    for (const auto& out : tx.vout) n += out.scriptPubKey.GetSigOpCount(false);
    return n;
}

uint64_t GetP2SHSigOpCount(const CTransaction& tx, const CCoinsViewCache& inputs) {
    if (tx.IsCoinBase()) return 0;
    uint64_t n = 0;
    for (const auto& in : tx.vin) {
        const CTxOut& prev = inputs.GetOutputFor(in);
        if (prev.scriptPubKey.IsPayToScriptHash()) n += prev.scriptPubKey.GetSigOpCount(in.scriptSig);
    }
    return n;
}

uint64_t GetTransactionSigOpCount(const CTransaction& tx, const CCoinsViewCache& inputs, int flags) {
    uint64_t n = GetSigOpCountWithoutP2SH(tx);
    if (tx.IsCoinBase()) return n;
    if (flags & SCRIPT_VERIFY_P2SH) n += GetP2SHSigOpCount(tx, inputs);
    return n;
}

static bool CheckTransactionCommon(const CTransaction& tx, CValidationState& state, bool fCheckDuplicateInputs) {
    if (tx.vin.empty()) return state.DoS(10, false, REJECT_INVALID, "bad-txns-vin-empty");
    if (tx.vout.empty()) return state.DoS(10, false, REJECT_INVALID, "bad-txns-vout-empty");
    if (tx.GetTotalSize() > MAX_TX_SIZE) return state.DoS(100, false, REJECT_INVALID, "bad-txns-oversize");
    Amount nValueOut = 0;
    for (const auto& out : tx.vout) {
        if (out.nValue < 0) return state.DoS(100, false, REJECT_INVALID, "bad-txns-vout-negative");
        if (out.nValue > MAX_MONEY) return state.DoS(100, false, REJECT_INVALID, "bad-txns-vout-toolarge");
        nValueOut += out.nValue;
        if (!MoneyRange(nValueOut)) return state.DoS(100, false, REJECT_INVALID, "bad-txns-txouttotal-toolarge");
    }
    if (GetSigOpCountWithoutP2SH(tx) > MAX_TX_SIGOPS_COUNT)
        return state.DoS(100, false, REJECT_INVALID, "bad-txn-sigops");
    if (fCheckDuplicateInputs) {
        std::set<COutPoint> seen;
        for (const auto& in : tx.vin)
            if (!seen.insert(in.prevout).second)
                return state.DoS(100, false, REJECT_INVALID, "bad-txns-inputs-duplicate");
    }
    return true;
}

bool CheckCoinbase(const CTransaction& tx, CValidationState& state, bool fCheckDuplicateInputs) {
    if (!tx.IsCoinBase()) return state.DoS(100, false, REJECT_INVALID, "bad-cb-missing", false, "first tx is not coinbase");
    if (!CheckTransactionCommon(tx, state, fCheckDuplicateInputs)) return false;
    if (tx.vin[0].scriptSig.size() < 2 || tx.vin[0].scriptSig.size() > 100)
        return state.DoS(100, false, REJECT_INVALID, "bad-cb-length");
    return true;
}

bool CheckRegularTransaction(const CTransaction& tx, CValidationState& state, bool fCheckDuplicateInputs) {
    if (tx.IsCoinBase()) return state.DoS(100, false, REJECT_INVALID, "bad-tx-coinbase");
    if (!CheckTransactionCommon(tx, state, fCheckDuplicateInputs)) return false;
    for (const auto& in : tx.vin)
        if (in.prevout.IsNull()) return state.DoS(10, false, REJECT_INVALID, "bad-txns-prevout-null");
    return true;
}

namespace Consensus {
bool CheckTxInputs(const CTransaction& tx, CValidationState& state, const CCoinsViewCache& inputs, int nSpendHeight) {
    if (!inputs.HaveInputs(tx)) return state.Invalid(false, 0, "", "Inputs unavailable");
    Amount nValueIn = 0;
    for (const auto& in : tx.vin) {
        const Coin& coin = inputs.AccessCoin(in.prevout);
        if (coin.IsCoinBase() && nSpendHeight - (int)coin.GetHeight() < COINBASE_MATURITY)
            return state.Invalid(false, REJECT_INVALID, "bad-txns-premature-spend-of-coinbase",
                                 strprintf("tried to spend coinbase at depth %d", nSpendHeight - (int)coin.GetHeight()));
        nValueIn += coin.GetTxOut().nValue;
        if (!MoneyRange(coin.GetTxOut().nValue) || !MoneyRange(nValueIn))
            return state.DoS(100, false, REJECT_INVALID, "bad-txns-inputvalues-outofrange");
    }
    const Amount out = tx.GetValueOut();
    if (nValueIn < out)
        return state.DoS(100, false, REJECT_INVALID, "bad-txns-in-belowout", false,
                         strprintf("value in (%s) < value out (%s)", FormatMoney(nValueIn).c_str(),
                                   FormatMoney(out).c_str()));
    const Amount fee = nValueIn - out;
    if (fee < 0) return state.DoS(100, false, REJECT_INVALID, "bad-txns-fee-negative");
    if (!MoneyRange(fee)) return state.DoS(100, false, REJECT_INVALID, "bad-txns-fee-outofrange");
    return true;
}
} // namespace Consensus

} // namespace bcp
