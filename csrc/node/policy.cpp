#include "node/policy.h"
#include "script/interpreter.h"

namespace bcp {

CFeeRate incrementalRelayFee(DEFAULT_INCREMENTAL_RELAY_FEE);
CFeeRate dustRelayFee(DUST_RELAY_TX_FEE);
CFeeRate minRelayTxFee(1000);
unsigned int nBytesPerSigOp = DEFAULT_BYTES_PER_SIGOP;
bool fIsBareMultisigStd = DEFAULT_PERMIT_BAREMULTISIG;
bool fRequireStandard = true;

bool IsStandard(const CScript& spk, txnouttype& whichType) {
    std::vector<std::vector<unsigned char>> sol;
    if (!Solver(spk, whichType, sol)) return false;
    if (whichType == TX_MULTISIG) {
        const unsigned char m = sol.front()[0], n = sol.back()[0];
        if (n < 1 || n > 3) return false;
        if (m < 1 || m > n) return false;
    } else if (whichType == TX_NULL_DATA && (!fAcceptDatacarrier || spk.size() > nMaxDatacarrierBytes)) {
        return false;
    }
    return whichType != TX_NONSTANDARD;
}

bool IsStandardTx(const CTransaction& tx, std::string& reason) {
    if (tx.nVersion > CTransaction::MAX_STANDARD_VERSION || tx.nVersion < 1) {
        reason = "version";
        return false;
    }
    if (tx.GetTotalSize() >= MAX_STANDARD_TX_SIZE) {
        reason = "tx-size";
        return false;
    }
    for (const CTxIn& in : tx.vin) {
        // 1650 bytes: 15-of-15 P2SH multisig with compressed keys, with room to spare
        if (in.scriptSig.size() > 1650) {
            reason = "scriptsig-size";
            return false;
        }
        if (!in.scriptSig.IsPushOnly()) {
            reason = "scriptsig-not-pushonly";
            return false;
        }
    }
    unsigned nDataOut = 0;
    txnouttype t;
    for (const CTxOut& out : tx.vout) {
        if (!IsStandard(out.scriptPubKey, t)) {
            reason = "scriptpubkey";
            return false;
        }
        if (t == TX_NULL_DATA) {
            nDataOut++;
        } else if (t == TX_MULTISIG && !fIsBareMultisigStd) {
            reason = "bare-multisig";
            return false;
        } else if (IsDust(out, dustRelayFee)) {
            reason = "dust";
            return false;
        }
    }
    if (nDataOut > 1) {
        reason = "multi-op-return";
        return false;
    }
    return true;
}

bool AreInputsStandard(const CTransaction& tx, const CCoinsViewCache& inputs) {
    if (tx.IsCoinBase()) return true;
    for (const CTxIn& in : tx.vin) {
        const CTxOut& prev = inputs.GetOutputFor(in);
        std::vector<std::vector<unsigned char>> sol;
        txnouttype t;
        if (!Solver(prev.scriptPubKey, t, sol)) return false;
        if (t == TX_SCRIPTHASH) {
            std::vector<std::vector<unsigned char>> stack;
            if (!EvalScript(stack, in.scriptSig, SCRIPT_VERIFY_NONE, BaseSignatureChecker())) return false;
            if (stack.empty()) return false;
            CScript sub(stack.back().begin(), stack.back().end());
            if (sub.GetSigOpCount(true) > MAX_P2SH_SIGOPS) return false;
        }
    }
    return true;
}

Amount GetDustThreshold(const CTxOut& txout, const CFeeRate& fee) {
    if (txout.scriptPubKey.IsUnspendable()) return 0;
    // cost of spending: the output plus a typical P2PKH input (32+4+1+107+4)
    size_t nSize = GetSerializeSize(txout) + (32 + 4 + 1 + 107 + 4);
    return 3 * fee.GetFee(nSize);
}

double GetPriority(const CTransaction& tx, const CCoinsViewCache& view, int nHeight, Amount& inChainInputValue) {
    inChainInputValue = 0;
    if (tx.IsCoinBase()) return 0.0;
    double dResult = 0.0;
    for (const CTxIn& in : tx.vin) {
        const Coin& coin = view.AccessCoin(in.prevout);
        if (coin.IsSpent()) continue;
        if ((int)coin.GetHeight() <= nHeight) {
            dResult += (double)coin.GetTxOut().nValue * (nHeight - (int)coin.GetHeight());
            inChainInputValue += coin.GetTxOut().nValue;
        }
    }
    // priority = sum(value * age) / modified size
    unsigned nSize = tx.GetTotalSize();
    for (const CTxIn& in : tx.vin) {
        const unsigned offset = 41U + std::min(110U, (unsigned)in.scriptSig.size());
        if (nSize > offset) nSize -= offset;
    }
    return nSize == 0 ? 0.0 : dResult / nSize;
}

} // namespace bcp
