// Key store and transaction signing.
// Parity: reference src/keystore.{h,cpp} (CBasicKeyStore: keys, redeem scripts,
// watch-only) and src/script/sign.{h,cpp} (TransactionSignatureCreator,
// DummySignatureCreator (72-byte placeholder sigs for fee estimation),
// ProduceSignature/SignSignature/CombineSignatures, default SIGHASH_ALL|FORKID in callers).
#pragma once
#include "util/sync.h"
#include "keys/key.h"
#include "script/interpreter.h"
#include "script/standard.h"

#include <map>
#include <mutex>
#include <set>

namespace bcp {

class CKeyStore {
public:
    virtual ~CKeyStore() {}
    virtual bool AddKeyPubKey(const CKey& key, const CPubKey& pubkey) = 0;
    bool AddKey(const CKey& key) { return AddKeyPubKey(key, key.GetPubKey()); }
    virtual bool HaveKey(const CKeyID& address) const = 0;
    virtual bool GetKey(const CKeyID& address, CKey& keyOut) const = 0;
    virtual std::set<CKeyID> GetKeys() const = 0;
    virtual bool GetPubKey(const CKeyID& address, CPubKey& out) const = 0;
    virtual bool AddCScript(const CScript& redeemScript) = 0;
    virtual bool HaveCScript(const CScriptID& hash) const = 0;
    virtual bool GetCScript(const CScriptID& hash, CScript& out) const = 0;
    virtual bool AddWatchOnly(const CScript& dest) = 0;
    virtual bool RemoveWatchOnly(const CScript& dest) = 0;
    virtual bool HaveWatchOnly(const CScript& dest) const = 0;
    virtual bool HaveWatchOnly() const = 0;
};

class CBasicKeyStore : public CKeyStore {
public:
    bool AddKeyPubKey(const CKey& key, const CPubKey& pubkey) override;
    bool HaveKey(const CKeyID& address) const override;
    bool GetKey(const CKeyID& address, CKey& keyOut) const override;
    std::set<CKeyID> GetKeys() const override;
    bool GetPubKey(const CKeyID& address, CPubKey& out) const override;
    bool AddCScript(const CScript& redeemScript) override;
    bool HaveCScript(const CScriptID& hash) const override;
    bool GetCScript(const CScriptID& hash, CScript& out) const override;
    bool AddWatchOnly(const CScript& dest) override;
    bool RemoveWatchOnly(const CScript& dest) override;
    bool HaveWatchOnly(const CScript& dest) const override;
    bool HaveWatchOnly() const override;

protected:
    mutable CCriticalSection cs_KeyStore{"cs_KeyStore"};
    std::map<CKeyID, CKey> mapKeys;
    std::map<CKeyID, CPubKey> mapWatchKeys;
    std::map<CScriptID, CScript> mapScripts;
    std::set<CScript> setWatchOnly;
};

class BaseSignatureCreator {
public:
    explicit BaseSignatureCreator(const CKeyStore* ks) : keystore(ks) {}
    virtual ~BaseSignatureCreator() {}
    const CKeyStore& KeyStore() const { return *keystore; }
    virtual const BaseSignatureChecker& Checker() const = 0;
    virtual bool CreateSig(std::vector<unsigned char>& sig, const CKeyID& keyid, const CScript& scriptCode) const = 0;

protected:
    const CKeyStore* keystore;
};

class TransactionSignatureCreator : public BaseSignatureCreator {
public:
    TransactionSignatureCreator(const CKeyStore* ks, const CTransaction* txTo, unsigned nIn, Amount amount,
                                uint32_t nHashType = SIGHASH_ALL | SIGHASH_FORKID)
        : BaseSignatureCreator(ks), txTo(txTo), nIn(nIn), amount(amount), nHashType(nHashType),
          checker(txTo, nIn, amount) {}
    const BaseSignatureChecker& Checker() const override { return checker; }
    bool CreateSig(std::vector<unsigned char>& sig, const CKeyID& keyid, const CScript& scriptCode) const override;

private:
    const CTransaction* txTo;
    unsigned nIn;
    Amount amount;
    uint32_t nHashType;
    TransactionSignatureChecker checker;
};

class DummySignatureCreator : public BaseSignatureCreator {
public:
    explicit DummySignatureCreator(const CKeyStore* ks) : BaseSignatureCreator(ks) {}
    const BaseSignatureChecker& Checker() const override;
    bool CreateSig(std::vector<unsigned char>& sig, const CKeyID& keyid, const CScript& scriptCode) const override;
};

struct SignatureData {
    CScript scriptSig;
    SignatureData() {}
    explicit SignatureData(const CScript& s) : scriptSig(s) {}
};

bool ProduceSignature(const BaseSignatureCreator& creator, const CScript& scriptPubKey, SignatureData& sigdata);
bool SignSignature(const CKeyStore& keystore, const CScript& fromPubKey, CMutableTransaction& txTo, unsigned nIn,
                   Amount amount, uint32_t nHashType);
SignatureData CombineSignatures(const CScript& scriptPubKey, const BaseSignatureChecker& checker,
                                const SignatureData& a, const SignatureData& b);
SignatureData DataFromTransaction(const CMutableTransaction& tx, unsigned nIn);
void UpdateTransaction(CMutableTransaction& tx, unsigned nIn, const SignatureData& data);

} // namespace bcp
