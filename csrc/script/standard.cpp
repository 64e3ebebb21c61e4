#include "script/standard.h"

namespace bcp {

bool fAcceptDatacarrier = true;
unsigned nMaxDatacarrierBytes = MAX_OP_RETURN_RELAY;

const char* GetTxnOutputType(txnouttype t) {
    switch (t) {
    case TX_NONSTANDARD: return "nonstandard";
    case TX_PUBKEY: return "pubkey";
    case TX_PUBKEYHASH: return "pubkeyhash";
    case TX_SCRIPTHASH: return "scripthash";
    case TX_MULTISIG: return "multisig";
    case TX_NULL_DATA: return "nulldata";
    }
    return nullptr;
}

static bool IsPubKeyPush(const std::vector<unsigned char>& v) { return v.size() >= 33 && v.size() <= 65; }
static bool IsSmallInteger(opcodetype op) { return op == OP_0 || (op >= OP_1 && op <= OP_16); }

// Direct template matching (same accepted language as the reference's template walker).
bool Solver(const CScript& spk, txnouttype& typeRet, std::vector<std::vector<unsigned char>>& sol) {
    sol.clear();
    typeRet = TX_NONSTANDARD;
    if (spk.IsPayToScriptHash()) {
        typeRet = TX_SCRIPTHASH;
        sol.emplace_back(spk.begin() + 2, spk.begin() + 22);
        return true;
    }
    if (spk.size() >= 1 && spk[0] == OP_RETURN && spk.IsPushOnly(spk.begin() + 1)) {
        typeRet = TX_NULL_DATA;
        return true;
    }
    // tokenize
    std::vector<std::pair<opcodetype, std::vector<unsigned char>>> ops;
    CScript::const_iterator pc = spk.begin();
    while (pc < spk.end()) {
        opcodetype op;
        std::vector<unsigned char> data;
        if (!spk.GetOp(pc, op, data)) return false;
        ops.emplace_back(op, std::move(data));
    }
    auto is_push = [](opcodetype op) { return op >= 0 && op <= OP_PUSHDATA4; };
    // <pubkey> CHECKSIG
    if (ops.size() == 2 && is_push(ops[0].first) && IsPubKeyPush(ops[0].second) && ops[1].first == OP_CHECKSIG) {
        typeRet = TX_PUBKEY;
        sol.push_back(ops[0].second);
        return true;
    }
    // DUP HASH160 <20> EQUALVERIFY CHECKSIG
    if (ops.size() == 5 && ops[0].first == OP_DUP && ops[1].first == OP_HASH160 && is_push(ops[2].first) &&
        ops[2].second.size() == 20 && ops[3].first == OP_EQUALVERIFY && ops[4].first == OP_CHECKSIG) {
        typeRet = TX_PUBKEYHASH;
        sol.push_back(ops[2].second);
        return true;
    }
    // m <pubkey>... n CHECKMULTISIG
    if (ops.size() >= 4 && IsSmallInteger(ops[0].first) && ops.back().first == OP_CHECKMULTISIG &&
        IsSmallInteger(ops[ops.size() - 2].first)) {
        for (size_t i = 1; i + 2 < ops.size(); ++i)
            if (!is_push(ops[i].first) || !IsPubKeyPush(ops[i].second)) return false;
        const int m = CScript::DecodeOP_N(ops[0].first);
        const int n = CScript::DecodeOP_N(ops[ops.size() - 2].first);
        const int nkeys = (int)ops.size() - 3;
        if (m < 1 || n < 1 || m > n || nkeys != n) return false;
        typeRet = TX_MULTISIG;
        sol.push_back({(unsigned char)m});
        for (size_t i = 1; i + 2 < ops.size(); ++i) sol.push_back(ops[i].second);
        sol.push_back({(unsigned char)n});
        return true;
    }
    return false;
}

bool ExtractDestination(const CScript& spk, CTxDestination& addressRet) {
    std::vector<std::vector<unsigned char>> sol;
    txnouttype t;
    if (!Solver(spk, t, sol)) return false;
    if (t == TX_PUBKEY) {
        CPubKey pk(sol[0]);
        if (!pk.IsValid()) return false;
        addressRet = pk.GetID();
        return true;
    }
    if (t == TX_PUBKEYHASH) {
        addressRet = CKeyID(uint160(sol[0]));
        return true;
    }
    if (t == TX_SCRIPTHASH) {
        addressRet = CScriptID(uint160(sol[0]));
        return true;
    }
    return false;
}

bool ExtractDestinations(const CScript& spk, txnouttype& typeRet, std::vector<CTxDestination>& addressRet,
                         int& nRequiredRet) {
    addressRet.clear();
    std::vector<std::vector<unsigned char>> sol;
    if (!Solver(spk, typeRet, sol)) return false;
    if (typeRet == TX_NULL_DATA) return false;
    if (typeRet == TX_MULTISIG) {
        nRequiredRet = sol.front()[0];
        for (size_t i = 1; i + 1 < sol.size(); i++) {
            CPubKey pk(sol[i]);
            if (!pk.IsValid()) continue;
            addressRet.push_back(pk.GetID());
        }
        return !addressRet.empty();
    }
    nRequiredRet = 1;
    CTxDestination d;
    if (!ExtractDestination(spk, d)) return false;
    addressRet.push_back(d);
    return true;
}

CScript GetScriptForDestination(const CTxDestination& dest) {
    CScript s;
    const std::vector<unsigned char> h(dest.hash.begin(), dest.hash.end());
    if (dest.type == DestType::KEYID) s << OP_DUP << OP_HASH160 << h << OP_EQUALVERIFY << OP_CHECKSIG;
    else if (dest.type == DestType::SCRIPTID) s << OP_HASH160 << h << OP_EQUAL;
    return s;
}

CScript GetScriptForRawPubKey(const CPubKey& pubkey) {
    CScript s;
    s << pubkey.Raw() << OP_CHECKSIG;
    return s;
}

CScript GetScriptForMultisig(int nRequired, const std::vector<CPubKey>& keys) {
    CScript s;
    s << CScript::EncodeOP_N(nRequired);
    for (const CPubKey& k : keys) s << k.Raw();
    s << CScript::EncodeOP_N((int)keys.size()) << OP_CHECKMULTISIG;
    return s;
}

} // namespace bcp
