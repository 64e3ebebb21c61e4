#include "script/sign.h"

namespace bcp {

typedef std::vector<unsigned char> valtype;

// ------------------------------------------------------------------ keystore
bool CBasicKeyStore::AddKeyPubKey(const CKey& key, const CPubKey& pubkey) {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    mapKeys[pubkey.GetID()] = key;
    return true;
}
bool CBasicKeyStore::HaveKey(const CKeyID& a) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    return mapKeys.count(a) > 0;
}
bool CBasicKeyStore::GetKey(const CKeyID& a, CKey& out) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    auto it = mapKeys.find(a);
    if (it == mapKeys.end()) return false;
    out = it->second;
    return true;
}
std::set<CKeyID> CBasicKeyStore::GetKeys() const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    std::set<CKeyID> r;
    for (const auto& kv : mapKeys) r.insert(kv.first);
    return r;
}
bool CBasicKeyStore::GetPubKey(const CKeyID& a, CPubKey& out) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    CKey k;
    if (GetKey(a, k)) {
        out = k.GetPubKey();
        return true;
    }
    auto it = mapWatchKeys.find(a);
    if (it == mapWatchKeys.end()) return false;
    out = it->second;
    return true;
}
bool CBasicKeyStore::AddCScript(const CScript& s) {
    if (s.size() > (size_t)MAX_SCRIPT_ELEMENT_SIZE) return false; // redeemScript must be pushable
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    mapScripts[CScriptID(s)] = s;
    return true;
}
bool CBasicKeyStore::HaveCScript(const CScriptID& h) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    return mapScripts.count(h) > 0;
}
bool CBasicKeyStore::GetCScript(const CScriptID& h, CScript& out) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    auto it = mapScripts.find(h);
    if (it == mapScripts.end()) return false;
    out = it->second;
    return true;
}
static bool ExtractPubKey(const CScript& dest, CPubKey& pubKeyOut) {
    // P2PK scripts: remember the key so the wallet can watch both forms
    std::vector<valtype> sol;
    txnouttype t;
    if (!Solver(dest, t, sol) || t != TX_PUBKEY) return false;
    pubKeyOut = CPubKey(sol[0]);
    return pubKeyOut.IsFullyValid();
}
bool CBasicKeyStore::AddWatchOnly(const CScript& dest) {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    setWatchOnly.insert(dest);
    CPubKey pk;
    if (ExtractPubKey(dest, pk)) mapWatchKeys[pk.GetID()] = pk;
    return true;
}
bool CBasicKeyStore::RemoveWatchOnly(const CScript& dest) {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    setWatchOnly.erase(dest);
    CPubKey pk;
    if (ExtractPubKey(dest, pk)) mapWatchKeys.erase(pk.GetID());
    return true;
}
bool CBasicKeyStore::HaveWatchOnly(const CScript& dest) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    return setWatchOnly.count(dest) > 0;
}
bool CBasicKeyStore::HaveWatchOnly() const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    return !setWatchOnly.empty();
}

// ------------------------------------------------------------------ creators
bool TransactionSignatureCreator::CreateSig(valtype& sig, const CKeyID& keyid, const CScript& scriptCode) const {
    CKey key;
    if (!keystore->GetKey(keyid, key)) return false;
    const uint256 hash = SignatureHash(scriptCode, *txTo, nIn, nHashType, amount, nullptr, SCRIPT_ENABLE_SIGHASH_FORKID);
    if (!key.Sign(hash, sig)) return false;
    sig.push_back((unsigned char)nHashType);
    return true;
}

namespace {
class DummySignatureChecker : public BaseSignatureChecker {
public:
    bool CheckSig(const valtype&, const valtype&, const CScript&, uint32_t, bool) const override { return true; }
};
const DummySignatureChecker dummyChecker;
} // namespace

const BaseSignatureChecker& DummySignatureCreator::Checker() const { return dummyChecker; }
bool DummySignatureCreator::CreateSig(valtype& sig, const CKeyID&, const CScript&) const {
    // Maximum-size placeholder DER signature (fee estimation).
    sig.assign(72, 0);
    sig[0] = 0x30;
    sig[1] = 69;
    sig[2] = 0x02;
    sig[3] = 33;
    sig[4] = 0x01;
    sig[4 + 33] = 0x02;
    sig[5 + 33] = 32;
    sig[6 + 33] = 0x01;
    sig[6 + 33 + 32] = SIGHASH_ALL | SIGHASH_FORKID;
    return true;
}

// ------------------------------------------------------------------ produce
static bool Sign1(const CKeyID& id, const BaseSignatureCreator& c, const CScript& code, std::vector<valtype>& ret) {
    valtype sig;
    if (!c.CreateSig(sig, id, code)) return false;
    ret.push_back(sig);
    return true;
}

static bool SignN(const std::vector<valtype>& multisig, const BaseSignatureCreator& c, const CScript& code,
                  std::vector<valtype>& ret) {
    int nSigned = 0;
    const int nRequired = multisig.front()[0];
    for (size_t i = 1; i + 1 < multisig.size() && nSigned < nRequired; i++) {
        CKeyID id = CPubKey(multisig[i]).GetID();
        if (Sign1(id, c, code, ret)) ++nSigned;
    }
    return nSigned == nRequired;
}

static bool SignStep(const BaseSignatureCreator& c, const CScript& spk, std::vector<valtype>& ret,
                     txnouttype& whichType) {
    ret.clear();
    std::vector<valtype> sol;
    if (!Solver(spk, whichType, sol)) return false;
    CKeyID id;
    switch (whichType) {
    case TX_NONSTANDARD:
    case TX_NULL_DATA:
        return false;
    case TX_PUBKEY:
        id = CPubKey(sol[0]).GetID();
        return Sign1(id, c, spk, ret);
    case TX_PUBKEYHASH: {
        id = CKeyID(uint160(sol[0]));
        if (!Sign1(id, c, spk, ret)) return false;
        CPubKey pk;
        c.KeyStore().GetPubKey(id, pk);
        ret.push_back(pk.Raw());
        return true;
    }
    case TX_SCRIPTHASH: {
        CScript redeem;
        if (c.KeyStore().GetCScript(CScriptID(uint160(sol[0])), redeem)) {
            ret.push_back(valtype(redeem.begin(), redeem.end()));
            return true;
        }
        return false;
    }
    case TX_MULTISIG:
        ret.push_back(valtype()); // CHECKMULTISIG dummy
        return SignN(sol, c, spk, ret);
    }
    return false;
}

static CScript PushAll(const std::vector<valtype>& values) {
    CScript r;
    for (const valtype& v : values) {
        if (v.empty()) r << OP_0;
        else if (v.size() == 1 && v[0] >= 1 && v[0] <= 16) r << CScript::EncodeOP_N(v[0]);
        else r << v;
    }
    return r;
}

bool ProduceSignature(const BaseSignatureCreator& creator, const CScript& fromPubKey, SignatureData& sigdata) {
    std::vector<valtype> result;
    txnouttype whichType;
    bool solved = SignStep(creator, fromPubKey, result, whichType);
    CScript subscript;
    if (solved && whichType == TX_SCRIPTHASH) {
        // the redeem script is signed as the scriptPubKey, then pushed last
        subscript = CScript(result[0].begin(), result[0].end());
        solved = solved && SignStep(creator, subscript, result, whichType) && whichType != TX_SCRIPTHASH;
        result.push_back(valtype(subscript.begin(), subscript.end()));
    }
    sigdata.scriptSig = PushAll(result);
    return solved && VerifyScript(sigdata.scriptSig, fromPubKey, STANDARD_SCRIPT_VERIFY_FLAGS, creator.Checker());
}

SignatureData DataFromTransaction(const CMutableTransaction& tx, unsigned nIn) {
    return SignatureData(tx.vin[nIn].scriptSig);
}
void UpdateTransaction(CMutableTransaction& tx, unsigned nIn, const SignatureData& data) {
    tx.vin[nIn].scriptSig = data.scriptSig;
}

bool SignSignature(const CKeyStore& keystore, const CScript& fromPubKey, CMutableTransaction& txTo, unsigned nIn,
                   Amount amount, uint32_t nHashType) {
    CTransaction txConst(txTo);
    TransactionSignatureCreator creator(&keystore, &txConst, nIn, amount, nHashType);
    SignatureData sd;
    const bool ok = ProduceSignature(creator, fromPubKey, sd);
    UpdateTransaction(txTo, nIn, sd);
    return ok;
}

// ------------------------------------------------------------------ combine
static std::vector<valtype> EvalPushes(const CScript& s) {
    std::vector<valtype> st;
    EvalScript(st, s, SCRIPT_VERIFY_STRICTENC, BaseSignatureChecker());
    return st;
}

static std::vector<valtype> CombineMultisig(const CScript& spk, const BaseSignatureChecker& checker,
                                            const std::vector<valtype>& sol, const std::vector<valtype>& s1,
                                            const std::vector<valtype>& s2) {
    std::set<valtype> allsigs;
    for (const valtype& v : s1)
        if (!v.empty()) allsigs.insert(v);
    for (const valtype& v : s2)
        if (!v.empty()) allsigs.insert(v);
    const unsigned nSigsRequired = sol.front()[0];
    const unsigned nPubKeys = (unsigned)sol.size() - 2;
    std::map<valtype, valtype> sigs;
    for (const valtype& sig : allsigs) {
        for (unsigned i = 0; i < nPubKeys; i++) {
            const valtype& pk = sol[i + 1];
            if (sigs.count(pk)) continue;
            if (checker.CheckSig(sig, pk, spk, STANDARD_SCRIPT_VERIFY_FLAGS)) {
                sigs[pk] = sig;
                break;
            }
        }
    }
    unsigned nSigsHave = 0;
    std::vector<valtype> result;
    result.push_back(valtype()); // dummy
    for (unsigned i = 0; i < nPubKeys && nSigsHave < nSigsRequired; i++) {
        auto it = sigs.find(sol[i + 1]);
        if (it != sigs.end()) {
            result.push_back(it->second);
            ++nSigsHave;
        }
    }
    for (unsigned i = nSigsHave; i < nSigsRequired; i++) result.push_back(valtype());
    return result;
}

static std::vector<valtype> CombineSignaturesImpl(const CScript& spk, const BaseSignatureChecker& checker,
                                                  txnouttype t, const std::vector<valtype>& sol,
                                                  std::vector<valtype> s1, std::vector<valtype> s2) {
    switch (t) {
    case TX_NONSTANDARD:
    case TX_NULL_DATA:
        return s1.size() >= s2.size() ? s1 : s2;
    case TX_PUBKEY:
    case TX_PUBKEYHASH:
        if (s1.empty() || s1[0].empty()) return s2;
        return s1;
    case TX_SCRIPTHASH: {
        if (s1.empty() || s1.back().empty()) return s2;
        if (s2.empty() || s2.back().empty()) return s1;
        valtype spk2 = s1.back();
        CScript pubKey2(spk2.begin(), spk2.end());
        txnouttype t2;
        std::vector<valtype> sol2;
        Solver(pubKey2, t2, sol2);
        s1.pop_back();
        s2.pop_back();
        std::vector<valtype> r = CombineSignaturesImpl(pubKey2, checker, t2, sol2, s1, s2);
        r.push_back(spk2);
        return r;
    }
    case TX_MULTISIG:
        return CombineMultisig(spk, checker, sol, s1, s2);
    }
    return {};
}

SignatureData CombineSignatures(const CScript& spk, const BaseSignatureChecker& checker, const SignatureData& a,
                                const SignatureData& b) {
    txnouttype t;
    std::vector<valtype> sol;
    Solver(spk, t, sol);
    return SignatureData(PushAll(CombineSignaturesImpl(spk, checker, t, sol, EvalPushes(a.scriptSig), EvalPushes(b.scriptSig))));
}

} // namespace bcp
